// common.h — shared host/device definitions for the gfx950 DSP library.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <type_traits>
#include "../../include/mi_av1dsp.h"

// Kernel timelines (diagnostic builds only, -DMI_KTL): lane 0 of every workgroup stores
// s_memrealtime stamps (100 MHz) at phase boundaries into ktl_buf[blockIdx.x * 8 + k], slot 7 =
// the XCC id. Each translation unit has its own buffer pointer, set from the host through
// mi_ktl_set_<unit> (no relocatable device code).
#ifdef MI_KTL
#define MI_KTL_DEFINE(unit)                                                                        \
    __device__ unsigned long long *ktl_buf;                                                        \
    extern "C" int mi_ktl_set_##unit(void *p) {                                                    \
        return hipMemcpyToSymbol(HIP_SYMBOL(ktl_buf), &p, sizeof(p)) == hipSuccess ? 0 : -5;     \
    }
#define KTL(k)                                                                                     \
    do {                                                                                           \
        if (ktl_buf && threadIdx.x == 0) {                                                         \
            ktl_buf[(size_t)blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();              \
            if ((k) == 0) {                                                                        \
                unsigned x_;                                                                       \
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x_));                  \
                ktl_buf[(size_t)blockIdx.x * 8 + 7] = x_ & 0xf;                                    \
            }                                                                                      \
        }                                                                                          \
    } while (0)
// slot k <- an arbitrary value (e.g. the work class of the workgroup)
#define KTLV(k, v)                                                                                 \
    do {                                                                                           \
        if (ktl_buf && threadIdx.x == 0) ktl_buf[(size_t)blockIdx.x * 8 + (k)] = (unsigned long long)(v); \
    } while (0)
#else
#define MI_KTL_DEFINE(unit)
#define KTL(k) do {} while (0)
#define KTLV(k, v) do {} while (0)
#endif

namespace mi {

// A field of the kernel-argument struct (the kernel's only argument) at a run-time byte
// offset: a scalar load from the kernarg segment. Indexing a by-value argument struct with a
// run-time index makes the compiler copy it to scratch, and compile-time selects keep every
// candidate live in SGPRs; this loads only the entry the workgroup needs.
template <typename T>
__device__ __forceinline__ T karg_at(size_t off) {
    typedef const T __attribute__((address_space(4))) *CT;
    typedef const char __attribute__((address_space(4))) *CC;
    return *(CT)((CC)__builtin_amdgcn_kernarg_segment_ptr() + off);
}
// field[idx] of the argument struct S
#define KARG_OF(S, field, idx) \
    ::mi::karg_at<typename std::remove_cv<typename std::remove_reference<decltype(((S *)0)->field[0])>::type>::type>( \
        offsetof(S, field) + sizeof(((S *)0)->field[0]) * (size_t)(idx))

// The dispatcher hands workgroup b to XCD b % 8 (MI355X: 8 XCDs, each with its own 4 MB L2).
// xcd_block renumbers the grid so that XCD k walks one contiguous chunk of the work list:
// neighbouring work items (adjacent tiles, spatially sorted blocks) then share one L2 instead
// of fetching the same lines into several. Bijective on [0, n). Used where it measured faster
// (CDEF 57.1 -> 54.7 us, deblock 48.9 -> 47.2 us at 4K10); MC, itx, LR and film grain lost 6-15 %
// with it (their cost per workgroup varies along the list, so equal-count chunks per XCD end
// unevenly), so they keep the hardware order.
__device__ inline int xcd_block(int b, int n) {
    const int x = b & 7, q = n >> 3, r = n & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// RectTxfmSize -> dimensions (src/levels.rs:46-82) and the inverse-transform row shift
// (src/itx.rs:439-457; C src/itx_tmpl.c:142-160).
struct TxDim { int w, h, shift; };
__host__ __device__ constexpr TxDim tx_dim(int tx) {
    constexpr TxDim t[19] = {
        { 4, 4, 0 },   { 8, 8, 1 },   { 16, 16, 2 }, { 32, 32, 2 }, { 64, 64, 2 },
        { 4, 8, 0 },   { 8, 4, 0 },   { 8, 16, 1 },  { 16, 8, 1 },  { 16, 32, 1 },
        { 32, 16, 1 }, { 32, 64, 1 }, { 64, 32, 1 }, { 4, 16, 1 },  { 16, 4, 1 },
        { 8, 32, 2 },  { 32, 8, 2 },  { 16, 64, 2 }, { 64, 16, 2 },
    };
    return t[tx];
}
__host__ __device__ constexpr int imin_c(int a, int b) { return a < b ? a : b; }
__host__ __device__ constexpr int imax_c(int a, int b) { return a > b ? a : b; }

// Lanes per transform block in the itx kernel: one lane per row in the row pass, one lane
// per column in the column pass.
__host__ __device__ constexpr int itx_lanes(int tx) {
    return imax_c(imin_c(tx_dim(tx).h, 32), tx_dim(tx).w);
}
// one-wave workgroups: 4K10 itx 34.1 -> 30.2 us (no cross-wave barriers; r04)
constexpr int kItxThreads = 64;
__host__ __device__ constexpr int itx_blocks_per_wg(int tx) { return kItxThreads / itx_lanes(tx); }
// Rounds of itx_blocks_per_wg blocks per workgroup: the small sizes' loads of all rounds are in
// flight together (4-lane blocks: 4 rounds; 8-lane blocks: 1 (banded grid, 4K10: 49.8 vs
// 50.7-51.3 us with 2; 4 rounds 56-58)).
#ifndef MI_ITX_SMALL_ROUNDS
#define MI_ITX_SMALL_ROUNDS 4
#endif
__host__ __device__ constexpr int itx_rounds(int tx) { return itx_lanes(tx) <= 4 ? MI_ITX_SMALL_ROUNDS : 1; }

// Which transform types are legal for a size (src/itx.rs:400-457): 16 types for sizes up to
// 16 on both sides except 16x16 (12 types), DCT_DCT + IDTX when a side is 32, DCT_DCT only
// when a side is 64. WHT_WHT (16) only for 4x4.
__host__ __device__ constexpr bool itx_type_valid(int tx, int txtp) {
    const TxDim d = tx_dim(tx);
    const int m = imax_c(d.w, d.h);
    if (txtp == 16) return tx == 0;
    if (m == 64) return txtp == 0;
    if (m == 32) return txtp == 0 || txtp == 9;
    if (d.w == 16 && d.h == 16) return txtp <= 11;
    return txtp < 16;
}

struct ItxArgs {
    uint8_t *plane[3];
    int64_t stride[3];
    const MiTxBlock *blocks;
    uint8_t *coef;
    int bdmax;
    int zero_coefs;
    int wg_start[39];   // first workgroup of the i-th range in grid order (kItxLaunchOrder)
    int wg_size[38];    // tx size of the i-th range, | kItxDcRange for a range of DC runs
    int blk_start[20];  // block ranges per tx size (enum order, as the caller groups them)
    // nbands 8: inside a size the blocks are further grouped by horizontal picture band (band q
    // = blocks[band_start[s][q] .. band_start[s][q + 1])), and band q's workgroups get grid
    // indices = q mod 8, i.e. run on XCD q (the dispatcher's round robin): every pixel line of
    // the band is fetched into, and written back from, one XCD's L2 whichever sizes touch it
    int band_start[19][9];
    // DC runs (mi_itx_frame_runs): the blocks [band_start[s][q], dc_end[s][q]) of a band are
    // DC-only (DCT_DCT, eob < 1) and take the DC path (itx_dc); the rest of the band the
    // transform path. dc_end[s][q] == band_start[s][q] when the caller gives no runs.
    int dc_end[19][8];
    int nbands;         // 1 or 8
    int pw[3], ph[3];   // plane extents (128-aligned picture area; 0 = no such plane)
    int *err;           // device error word: set when a descriptor is rejected
    // MI_ITX_DC_DEFER: the DC runs write their scaled DC into this per-4x4-unit map instead of
    // adding it to the pixels (the next mi_deblock_frame_dc adds it while staging); entry =
    // (dc_tag << 16) | (dc & 0xffff), plane p at dc_map + dc_off[p], dc_stride[p] entries a row
    uint32_t *dc_map;
    int64_t dc_off[3];
    int dc_stride[3];
    uint32_t dc_tag;
};
// the DC map of one picture geometry: one entry per 4x4 unit of the 128-aligned plane areas
struct DcMapGeom {
    int64_t off[3];
    int stride[3], rows[3];
    size_t entries;
};
inline DcMapGeom dc_map_geom(int w, int h, int layout) {
    DcMapGeom g{};
    const int aw = (w + 127) & ~127, ah = (h + 127) & ~127;
    const int sh = layout == 1 || layout == 2, sv = layout == 1;
    size_t n = 0;
    for (int p = 0; p < (layout ? 3 : 1); p++) {
        g.off[p] = (int64_t)n;
        g.stride[p] = (p ? aw >> sh : aw) >> 2;
        g.rows[p] = (p ? ah >> sv : ah) >> 2;
        n += (size_t)g.stride[p] * g.rows[p];
    }
    g.entries = n;
    return g;
}

// Legal TxfmType values of a RectTxfmSize (itx.rs:400-457, 1072-1110): bit t set when the
// reference's itxfm_add[tx][t] slot is filled.
// The stored coefficients of one block (MiTxBlock): the dense min(w,32) x min(h,32) layout
// (column-major, column height min(h,32)), or with MI_TX_PACKED the CW x CH corner stored
// row-major (coefficient (x, y) at y * CW + x, every other one zero).
struct TxCoefShape { int cw, ch; };
__host__ __device__ inline TxCoefShape tx_coef_shape(uint8_t flags, int sw, int sh) {
    if (flags & MI_TX_PACKED) return { (int)MI_TX_PACKED_CW(flags), (int)MI_TX_PACKED_CH(flags) };
    return { sw, sh };
}
// a descriptor's flags are legal for a block of sw x sh stored coefficients at arena offset
// coef_off (a packed corner starts on a 4-coefficient boundary: its rows are vector loads;
// int16 corners only in the int32 arenas of 10/12-bit frames)
__host__ __device__ inline bool tx_flags_ok(uint8_t flags, int sw, int sh, uint32_t coef_off, bool hbd) {
    if (!flags) return true;
    return (flags & MI_TX_PACKED) && (!(flags & MI_TX_I16) || hbd) && (int)MI_TX_PACKED_CW(flags) <= sw &&
           (int)MI_TX_PACKED_CH(flags) <= sh && (coef_off & 3) == 0;
}

#ifdef __HIPCC__
// Lane j's row of a block's coefficients (x = 0 .. SW-1) for the row transform. Dense: one word
// per x at j + x * SH (consecutive lanes read consecutive words). Packed: the row's CW
// coefficients are contiguous, read as 4-coefficient vectors (16 B for int32, 8 B for int16)
// with a guard per vector, not per coefficient; rows j >= CH and columns >= CW read as zero.
template <int SW, int SH, typename Cf>
__device__ __forceinline__ void tx_load_row(const Cf *cf, uint8_t flags, int j, int (&v)[SW]) {
    if (flags & MI_TX_PACKED) {
        const int cw = (int)MI_TX_PACKED_CW(flags), ch = (int)MI_TX_PACKED_CH(flags);
        const Cf *rp = cf + j * cw;
        const int16_t *rh = reinterpret_cast<const int16_t *>(cf) + j * cw;   // MI_TX_I16
        const bool i16 = sizeof(Cf) == 4 && (flags & MI_TX_I16);
#pragma unroll
        for (int g = 0; g < SW / 4; g++) {
            if (j < ch && 4 * g < cw) {
                if (sizeof(Cf) == 2 || i16) {
                    const uint2 q = *reinterpret_cast<const uint2 *>((sizeof(Cf) == 2 ? reinterpret_cast<const int16_t *>(rp) : rh) + 4 * g);
                    v[4 * g] = (int)(int16_t)(q.x & 0xffff); v[4 * g + 1] = (int)(int16_t)(q.x >> 16);
                    v[4 * g + 2] = (int)(int16_t)(q.y & 0xffff); v[4 * g + 3] = (int)(int16_t)(q.y >> 16);
                } else {
                    const int4 q = *reinterpret_cast<const int4 *>(rp + 4 * g);
                    v[4 * g] = q.x; v[4 * g + 1] = q.y; v[4 * g + 2] = q.z; v[4 * g + 3] = q.w;
                }
            } else {
                v[4 * g] = v[4 * g + 1] = v[4 * g + 2] = v[4 * g + 3] = 0;
            }
        }
    } else {
#pragma unroll
        for (int x = 0; x < SW; x++) v[x] = (int)cf[j + x * SH];
    }
}
// zero what tx_load_row read (itxfm_add consumes its coefficients)
template <int SW, int SH, typename Cf>
__device__ __forceinline__ void tx_zero_row(Cf *cf, uint8_t flags, int j) {
    if (flags & MI_TX_PACKED) {
        const int cw = (int)MI_TX_PACKED_CW(flags), ch = (int)MI_TX_PACKED_CH(flags);
        Cf *rp = cf + j * cw;
        int16_t *rh = reinterpret_cast<int16_t *>(cf) + j * cw;   // MI_TX_I16
        const bool i16 = sizeof(Cf) == 4 && (flags & MI_TX_I16);
#pragma unroll
        for (int g = 0; g < SW / 4; g++)
            if (j < ch && 4 * g < cw) {
                if (sizeof(Cf) == 2 || i16)
                    *reinterpret_cast<uint2 *>((sizeof(Cf) == 2 ? reinterpret_cast<int16_t *>(rp) : rh) + 4 * g) = make_uint2(0, 0);
                else *reinterpret_cast<int4 *>(rp + 4 * g) = make_int4(0, 0, 0, 0);
            }
    } else {
#pragma unroll
        for (int x = 0; x < SW; x++) cf[j + x * SH] = 0;
    }
}
#endif

__host__ __device__ constexpr uint32_t itx_legal_types(int tx) {
    return tx == 0 ? 0x1ffffu
         : imax_c(tx_dim(tx).w, tx_dim(tx).h) == 64 ? 0x1u
         : imax_c(tx_dim(tx).w, tx_dim(tx).h) == 32 ? 0x201u
         : (tx_dim(tx).w == 16 && tx_dim(tx).h == 16) ? 0xfffu : 0xffffu;
}
// order of the tx sizes in the itx grid: the 64-point sizes first (few workgroups, the longest),
// then the 32-point sizes, then every size with both sides <= 16
// (4x4 right after the 64-point sizes: its 64-block workgroups live longest after them, 14.9 us
// in the round-6 timeline, and started last among the long ones; 27.43-27.52 against
// 27.69-27.74 us for the DC-deferred stage, profiles/r06_itx_order.txt)
#ifndef MI_ITX_ORDER
#define MI_ITX_ORDER 4, 11, 12, 0, 17, 18, 3, 9, 10, 15, 16, 1, 2, 5, 6, 7, 8, 13, 14
#endif
constexpr int kItxLaunchOrder[19] = { MI_ITX_ORDER };
constexpr int kItxBands = 8;
constexpr int kItxDcRange = 32;   // wg_size flag: the range's workgroups run DC runs
// DC path geometry of a size: chunks of min(w, 8) pixels, kItxDcItems chunks per lane, up to
// 128 blocks per workgroup
constexpr int kItxDcItems = 16;
__host__ __device__ constexpr int itx_dc_blocks(int tx) {
    return imax_c(1, imin_c(128, 64 * kItxDcItems / (tx_dim(tx).h * (tx_dim(tx).w < 8 ? 1 : tx_dim(tx).w / 8))));
}
// fills wg_start / wg_size / blk_start (and the band table when band_start, [19][9], is given;
// DC runs when dc_end, [19][8], is given too); returns the grid size
int itx_fill_schedule(ItxArgs &a, const uint32_t *size_start, const uint32_t *band_start = nullptr,
                      const uint32_t *dc_end = nullptr);

// launcher (itx.hip)
int launch_itx_frame(const ItxArgs &a, int nwg, int bpc, hipStream_t s);

struct LfArgs {
    uint8_t *plane[3];
    int64_t stride[3];
    const uint32_t *level;     // [u8;4] packed little-endian
    int64_t b4_stride;
    const MiAv1Filter *masks;
    int sb128w, sb128h;
    int w4, h4, ss_hor, ss_ver, bdmax, bdm8, filter_uv;
    int blk_start[4];          // flattened workgroup ranges per plane
    int units_x[3], rows[3];   // thread space per plane
    uint8_t lim_e[64], lim_i[64];
};
// fused out-of-place deblock (lf_tile_kernel): kLfTW x kLfTH plane tiles
#ifndef MI_LF_TW
#define MI_LF_TW 64   // 64x64 measured fastest at 4K10: 29.6 us vs 34.9 (128x64), 32.5 (32x64)
#endif
#ifndef MI_LF_TH
#define MI_LF_TH 128   // 64x128 tiles, 512 lanes: 29.0-29.2 us at 4K10 against 31.5-32.3 for 64x64 (256 lanes)
#endif
#ifndef MI_LF_LPR
#define MI_LF_LPR 4   // lanes per tile row
#endif
constexpr int kLfTW = MI_LF_TW, kLfTH = MI_LF_TH;
constexpr int kLfThreads = kLfTH * MI_LF_LPR;   // lf_tile_kernel workgroup: 256 lanes per 64 tile rows
struct LfTileArgs {
    const uint8_t *src[3];
    uint8_t *dst[3];
    int64_t stride[3];
    const uint32_t *level;
    int64_t b4_stride;
    const MiAv1Filter *masks;
    int sb128w, w4, h4, ss_hor, ss_ver, bdmax, bdm8;
    int cols_ux[3], cols_rows[3];   // column edges: unit columns, pixel rows per plane
    int rows_px[3], rows_uy[3];     // row edges: pixel columns, unit rows per plane
    int pw[3], ph[3], tiles_x[3];   // staged plane area (128-aligned picture), tiles per row
    int tile_start[4];
    uint8_t lim_e[64], lim_i[64];
    // mi_deblock_frame_dc: the DC map of mi_itx_frame_runs(MI_ITX_DC_DEFER) (null: none); its
    // entries tagged dc_tag are added to the staged pixels (ItxArgs::dc_map's layout)
    const uint32_t *dc_map;
    int64_t dc_off[3];
    int dc_stride[3];
    uint32_t dc_tag;
};
int launch_deblock_tiles(const LfTileArgs &a, int bpc, hipStream_t s);
// launchers (lf.hip)
int launch_deblock(const LfArgs &cols, const LfArgs &rows, int bpc, hipStream_t s);

struct CdefArgs {
    const uint8_t *src[3];
    uint8_t *dst[3];
    int64_t stride[3];
    const MiAv1Filter *masks;
    int sb128w, tiles_x;
    int bw4, bh4;                 // frame size in 4-px units, 8-px aligned (f->bw, f->bh)
    int ss_hor, ss_ver, layout;
    int bdm8, damping;            // damping already includes bitdepth_min_8
    uint8_t y_strength[8], uv_strength[8];
    const int32_t *order;         // workgroup -> 64x64 unit (null: xcd_block's grid order)
};
// launchers (cdef.hip)
int launch_cdef(const CdefArgs &a, int tiles, int bpc, hipStream_t s);

struct McArgs {
    uint8_t *dst[3];
    int64_t dst_stride[2];
    const uint8_t *ref[7][3];
    int64_t ref_stride[7][2];
    int ref_w[7][3], ref_h[7][3];    // plane dimensions (clamp bounds)
    const MiMcBlock *blocks;
    uint8_t *masks;
    int16_t *tmp;                    // MI_MC_PREP arena
    int bpc, ib, bias, bdmax, layout;
    int nrefs;                       // valid entries of ref / ref_stride / ref_w / ref_h
    int seg_ss_hor, seg_ss_ver;      // w_mask[chr_layout_idx] subsampling of the SEG mask
    uint32_t class_start[2 * MI_MC_NCLASS + 1];
    uint32_t first_wave[2][MI_MC_NCLASS + 1];
    // one grid with in-launch hand-off (mi_mc_frame_sync): a SEG unit's tiles publish their
    // mask with `sc1` word stores and set seg_flags[(mask_off >> 4) * 32 + tile] = seg_epoch;
    // chroma MASK units flagged MI_MC_AFTER_SEG wait for them (null: no hand-off)
    uint32_t *seg_flags;
    uint32_t seg_epoch;
    uint32_t seg_nflags;             // entries of seg_flags: a flag index at or past it is an error
    int *err;
};
// launchers (mc.hip): mc_plan fills first_wave[g] and returns the wave count of group g
int mc_plan(McArgs &a, int g);
int launch_mc(const McArgs &a, int g, int waves, hipStream_t s);

// scaled references, warp, combine (mc_ext.hip): McArgs supplies pictures and bit depth;
// `units` is the device array of the entry point, cur_w / cur_h the current frame's luma size
int launch_mc_scaled(const McArgs &a, const MiMcBlock *units, int n, int cur_w, int cur_h, hipStream_t s);
int launch_mc_warp(const McArgs &a, const MiWarpBlock *blocks, int n, hipStream_t s);
int launch_mc_combine(const McArgs &a, const MiMcCombine *units, int n, hipStream_t s);

struct SuperresArgs {
    const uint8_t *src[3];
    uint8_t *dst[3];
    int64_t src_stride[2], dst_stride[2];
    int src_w[3], dst_w[3], h[3];   // per plane: resize source width (4 * f->bw), output width, rows
    int step[2], start[2];          // luma, chroma
    int bpc, nplanes, chunks;       // chunks: 256-px output segments per row (max over planes)
};
int launch_superres(const SuperresArgs &a, hipStream_t s);

struct IpredArgs {
    uint8_t *dst[3];
    int64_t stride[2];
    const MiIpredBlock *blocks;
    const uint8_t *edges;
    const int16_t *ac;
    const uint8_t *idx;
    const MiIntraBlock *iblocks;     // mi_intra_blocks
    const uint8_t *pal;
    int bpc, bdmax;
};
// persistent fused intra reconstruction (ipred.hip): frame f is worked on by XCD f % 8
// edge granules per frame (ipred.hip GranCtx: per plane, a column-boundary array then a
// row-boundary array of 8-B {two pixels, epoch} records); host: the allocation
__host__ __device__ inline size_t gran_count(int pw, int ph, int ss_hor, int ss_ver, int nplanes) {
    size_t n = 0;
    for (int p = 0; p < nplanes; p++) {
        const int w = p ? pw >> ss_hor : pw, h = p ? ph >> ss_ver : ph;
        n += (size_t)((w >> 2) + 1) * (h >> 1) + (size_t)((h >> 2) + 1) * (w >> 1);
    }
    return n;
}

struct IntraReconFrame {
    IpredArgs ip;                 // picture planes / strides, iblocks, ac, idx, pal, bpc, bdmax
    const MiTxBlock *tx;
    uint8_t *coef;
    const int32_t *dep_start, *deps;
    uint32_t *done;               // epoch when reconstructed: block i's flag is done[base + i],
                                  // dependency d's is done[d] (a strip's deps index its frame)
    int *head;                    // queue head
    int n, base;
    uint16_t pw, ph;              // luma plane extent (128-aligned picture area)
    uint8_t ss_hor, ss_ver, nplanes, pad_;
    uint32_t goff;                // edge granules (IntraReconArgs::gran): this frame's first one
};
constexpr int kIrMaxFrames = 24;     // descriptors travel as kernel arguments (4 KB limit)
struct IntraReconArgs {
    IntraReconFrame fr[kIrMaxFrames];   // queue f (a frame, or a strip of one) on XCD f % 8
    int *xcd_rank;                // [8] worker counters (zeroed per launch)
    int *err;
    int *dbg;                     // MI_IR_DEBUG builds: host-mapped progress words
    int *desc_err;                // rejected descriptors (skipped; reported as -EINVAL)
    // edge granules (null: off): per frame and plane, the right column of every block at its
    // 4-px column boundary and its bottom row at its row boundary, as 8-B {two pixels, epoch}
    // records a consumer polls instead of a done flag plus pixel loads (ipred.hip)
    unsigned long long *gran;
    // MI_IR_TIMELINE (diagnostics): 16 s_memrealtime stamps per unit, parallel to the done words:
    // unit stamps at tl + 32 * (byte address of its done word), tl biased by the host
    uintptr_t tl;
    uint32_t epoch;
    int nframes, zero_coefs;
};
static_assert(sizeof(IntraReconArgs) <= 4096, "kernel argument limit");
int launch_intra_recon(const IntraReconArgs &a, int bpc, int wg_per_xcd, hipStream_t s);
// launchers (ipred.hip)
int launch_ipred(const IpredArgs &a, int n, hipStream_t s);
int launch_intra(const IpredArgs &a, int n, hipStream_t s);

struct LrArgs {
    const uint8_t *src[3];        // CDEF output C
    const uint8_t *lpf[3];        // deblocked D (rows across stripe edges)
    uint8_t *dst[3];
    int64_t stride[3];
    const MiAv1Restoration *lr_mask;
    int sb128w, restore, bd, ss_hor, ss_ver;
    int unit_log2[2];
    int pw[3], ph[3], tw[3], tiles_x[3];
    int blk_start[4];
    const int32_t *order;         // workgroup -> tile (null: grid order)
};
// launchers (lr.hip)
int launch_lr(const LrArgs &a, int bpc, hipStream_t s);

// Wiener taps (centre +128 folded for every bit depth) or self-guided strengths / weights
struct LrTileParams {
    bool wiener;
    int fh[7], fv[7];
    int s0, s1, w0, w1;
};
struct LrCallArgs {
    const uint8_t *p, *lpf, *left;   // staged unit pixels (column 0 = unit column 0), lpf rows 0-7, left [h][4]
    uint8_t *out;                     // packed w x h
    int64_t ps;                       // pixel stride of p and lpf (elements)
    int w, h, edges, bd;
    LrTileParams tp;
};
int launch_lr_call(const LrCallArgs &a, int bpc, hipStream_t s);

constexpr int kFgItems = 1;   // wave-items (512-px row segments) per wave in fg_apply_kernel (8K10 apply: 1 -> 72.5 us, 4 -> 75.7, 8 -> 78.4)

struct FgArgs {
    MiFilmGrainData data;
    const uint8_t *src[3];
    uint8_t *dst[3];
    int64_t stride[3];
    int16_t *lut;                 // [3][73][82]
    uint8_t *scaling;             // [3][4096]
    uint8_t *offsets;             // [nrows][nblocks]
    int bpc, layout, ss_x, ss_y, w, h, is_id, nrows, nblocks;
    int pw[3], ph[3], chunks[3], grain[3];
    int blk_start[4];
    // per-call (table) mode; all zero for frames
    const int16_t *lut_y;         // generate_grain_uv: the caller's luma template [73][82]; only plane uv_only
    int uv_only;                  //   1 + uv
    int row0;                     // block-row number of offsets row 0 (row seeds)
    int row_off;                  // offsets row of image row 0 (1 when a previous block row overlaps)
};
// launchers (fg.hip)
int init_fg_tables();
int launch_fg(const FgArgs &a, hipStream_t s, bool prep, bool apply);
int launch_fg_call(const FgArgs &a, hipStream_t s);

// ---- per-call (table-compatible) entry points: single-block kernels ----
struct LfCallArgs {
    uint8_t *dst;
    int64_t stride;
    const uint8_t *lvl;             // [32][2]: unit level, neighbour level
    uint32_t vmask[3];
    int cls, dir, bdm8, bdmax;
    uint8_t lim_e[64], lim_i[64];
};
int launch_lf_sb_call(const LfCallArgs &a, int bpc, hipStream_t s);   // lf.hip

struct CdefCallArgs {
    const uint8_t *dst, *left, *top, *bottom;   // dst: the block (read); left: [h][2]
    uint8_t *out;                               // filter: w x h packed; dir: {dir, var}
    int64_t stride;
    int w, h, pri, sec, dir, damping, edges, bdm8;
};
int launch_cdef_call(const CdefCallArgs &a, int bpc, bool dir, hipStream_t s);   // cdef.hip

struct CflAcArgs {
    int16_t *ac;
    const uint8_t *y;
    int64_t stride;
    int w_pad, h_pad, cw, ch, ss_hor, ss_ver;
};
int launch_cfl_ac(const CflAcArgs &a, int bpc, hipStream_t s);   // ipred.hip

struct McCallArgs {
    uint8_t *dst;                 // put / combine destination (pixels)
    const uint8_t *src;           // put / prep source at the block origin; blend: tmp pixels; emu: clamped rect
    int16_t *tmp1;                // prep output, or the first combine input
    const int16_t *tmp2;
    const uint8_t *mask;          // mask / blend input
    uint8_t *mask_out;            // w_mask output
    int64_t dst_stride, src_stride;
    int w, h, mx, my, filter2d, prep, op, weight, sign, ss_hor, ss_ver, iw, ih;
    int abcd[4];                  // warp
    int dx, dy;                   // scaled
    int bpc, ib, bias, bdmax;
};
// kind 0 put / prep, 1 combine (op), 2 emu_edge, 3 warp8x8(t), 4 resize, 5 scaled (mc_call.hip)
int launch_mc_call(const McCallArgs &a, int kind, hipStream_t s);

} // namespace mi
