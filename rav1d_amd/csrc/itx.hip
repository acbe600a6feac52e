// itx.hip — batched inverse transform + add for a whole frame on gfx950.
//
// Replaces the per-block itxfm_add[tx][txtp] calls made from recon (rav1d src/recon.rs:
// 1781-1788, 2674-2682, 3116, 4013). Semantics per block are inv_txfm_add_rust
// (src/itx.rs:64-188; C src/itx_tmpl.c:40-100) and the lossless WHT (src/itx.rs:475-526).
//
// Mapping. Blocks arrive grouped by tx size (inside a size, DC-only blocks first and then by
// position keeps control flow wave-uniform and lets neighbouring blocks of a workgroup share
// pixel lines). One launch per frame; a 256-lane workgroup takes BPW blocks of one size:
//   1. every lane reads its block descriptor and immediately issues the loads of the
//      destination pixels it will own in step 4 (4-pixel row chunks, 4/8-byte vector loads),
//      so they are in flight during the transforms;
//   2. lane j runs the 1-D row transform of row j in VGPRs (coefficients read straight from
//      the arena's column-major layout: consecutive lanes read consecutive words) and writes
//      the shifted/clipped row to LDS;
//   3. lane j runs the 1-D column transform of column j and writes (c + 8) >> 4 back to LDS;
//   4. lanes add the residual rows to their prefetched pixel chunks and store them as vectors.
// DC-only blocks skip 2 and 3. Butterflies live entirely in VGPRs; no MFMA (small fixed
// integer networks, not contractions).
#include "common.h"
#include "itx_1d.h"
#include <algorithm>
#include <type_traits>

MI_KTL_DEFINE(itx)

namespace mi {

// TxfmType -> 1-D kinds (levels.rs TxfmType is VERT_HORZ; itx_tmpl.c:196-233)
__constant__ uint8_t k_col_kind[16] = { KD, KA, KD, KA, KF, KD, KF, KA, KF, KI, KD, KI, KA, KI, KF, KI };
__constant__ uint8_t k_row_kind[16] = { KD, KD, KA, KA, KD, KF, KF, KF, KA, KI, KI, KD, KI, KA, KI, KF };

__host__ __device__ constexpr bool itx_is_large(int tx) {
    return tx_dim(tx).w >= 32 || tx_dim(tx).h >= 32;
}
template <int TX>
__host__ __device__ constexpr int itx_lds_elems() {
    return itx_blocks_per_wg(TX) * imin_c(tx_dim(TX).h, 32) * (tx_dim(TX).w + 1);
}
__host__ __device__ constexpr int itx_lds_max(bool large) {
    int m = 0;
    for (int t = 0; t < 19; t++)
        if (itx_is_large(t) == large) {
            const int e = itx_blocks_per_wg(t) * imin_c(tx_dim(t).h, 32) * (tx_dim(t).w + 1);
            m = e > m ? e : m;
        }
    return m;
}

template <typename Px> struct Vec4;
template <> struct Vec4<uint8_t> { using T = uint32_t; };
template <> struct Vec4<uint16_t> { using T = uint2; };

template <typename Px>
__device__ __forceinline__ void unpack4(const typename Vec4<Px>::T &v, int *o) {
    if constexpr (sizeof(Px) == 1) {
        o[0] = v & 0xff; o[1] = (v >> 8) & 0xff; o[2] = (v >> 16) & 0xff; o[3] = v >> 24;
    } else {
        o[0] = v.x & 0xffff; o[1] = v.x >> 16; o[2] = v.y & 0xffff; o[3] = v.y >> 16;
    }
}
template <typename Px>
__device__ __forceinline__ typename Vec4<Px>::T pack4(const int *o) {
    if constexpr (sizeof(Px) == 1) {
        return (uint32_t)o[0] | ((uint32_t)o[1] << 8) | ((uint32_t)o[2] << 16) | ((uint32_t)o[3] << 24);
    } else {
        uint2 v;
        v.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
        v.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
        return v;
    }
}

// An int of the kernel-argument struct at a run-time byte offset: a scalar load from the
// kernarg segment. Indexing the by-value ItxArgs with a run-time index would copy it to
// scratch, and the compile-time-index selects used before kept every table entry live in SGPRs
// (hundreds of SGPR spills); this reads only the entries a workgroup needs.
__device__ __forceinline__ int karg_i32(size_t off) {
    typedef const int __attribute__((address_space(4))) *CI;
    typedef const char __attribute__((address_space(4))) *CC;
    return *(CI)((CC)__builtin_amdgcn_kernarg_segment_ptr() + off);
}
#define KARG(field, idx) karg_i32(offsetof(ItxArgs, field) + 4 * (size_t)(idx))

// a[i] for i in 0..2 as selects (a dynamic index into the kernel-argument struct would make
// the compiler copy the whole struct to scratch)
template <typename T> __device__ __forceinline__ T sel3(const T (&v)[3], int i) { return i == 0 ? v[0] : i == 1 ? v[1] : v[2]; }

template <int TX, typename Px, typename Cf, typename Lt, bool Wide>
__device__ __forceinline__ void itx_size(const ItxArgs &a, int lwg, Lt *lds) {
    constexpr TxDim D = tx_dim(TX);
    constexpr int Wd = D.w, Ht = D.h, SH = imin_c(Ht, 32), SW = imin_c(Wd, 32);
    constexpr int TPB = itx_lanes(TX), BPW = kItxThreads / TPB, ROUNDS = itx_rounds(TX);
    constexpr int LS = Wd + 1;                        // padded LDS row stride
    constexpr bool Rect2 = (Wd == 2 * Ht) || (Ht == 2 * Wd);
    constexpr int Shift = D.shift, Rnd = (1 << Shift) >> 1;
    constexpr int CPR = Wd / 4;                       // 4-px chunks per row
    constexpr int NCH = (Ht * CPR + TPB - 1) / TPB;   // chunks per lane
    using V = typename Vec4<Px>::T;

    const int t = threadIdx.x;
    const int lb = t / TPB, j = t % TPB;
    // this workgroup's block range: the whole size, or (banded grid) band lwg % 8 of it
    int bs = a.blk_start[TX], be = a.blk_start[TX + 1], k = lwg;
    if (a.nbands > 1) {
        const int q = lwg & 7;
        k = lwg >> 3;
        bs = KARG(dc_end, TX * 8 + q);            // after the band's DC run (itx_dc)
        be = KARG(band_start, TX * 9 + q + 1);
    }
#ifdef MI_KTL
    {
        // (timeline builds) the block range known: the kernel-argument reads are done
        asm volatile("" ::"s"(bs), "s"(be));
        KTL(3);
    }
#endif
    // per-plane arguments as locals (selected by value, never by address into the kernarg)
    uint8_t *const plane3[3] = { a.plane[0], a.plane[1], a.plane[2] };
    const int64_t stride3[3] = { a.stride[0], a.stride[1], a.stride[2] };
    const int pw3[3] = { a.pw[0], a.pw[1], a.pw[2] }, ph3[3] = { a.ph[0], a.ph[1], a.ph[2] };
    const int bdmax = a.bdmax;
    Lt *tmp = lds + lb * SH * LS;

    // ---- 1. every round's descriptor, destination chunks and DC coefficient in flight at
    // once: small blocks carry little work per load, so a workgroup takes ROUNDS x BPW of
    // them and overlaps their memory latency instead of paying it once per round ----
    MiTxBlock bk[ROUNDS];
    bool vk[ROUNDS];
    int dk[ROUNDS];
    V pk[ROUNDS][NCH];
    // multi-round sizes: every round's coefficient row too, so that later rounds do not pay a
    // load latency each (lane j < SH reads row j: SW coefficients)
    constexpr int CR = ROUNDS > 1 ? ROUNDS : 1, CW = ROUNDS > 1 ? SW : 1;
    int ck[CR][CW];
#pragma unroll
    for (int rd = 0; rd < ROUNDS; rd++) {
        const int bi = bs + (k * ROUNDS + rd) * BPW + lb;
        bool valid = bi < be;
        MiTxBlock b{};
        if (valid) {
            b = a.blocks[bi];
            // a descriptor the reference could never issue (wrong size group, a type the
            // size's table slot lacks, a rectangle outside its plane) is skipped and reported
            const bool ok = b.tx == TX && b.txtp < 17 && ((itx_legal_types(TX) >> b.txtp) & 1) &&
                            tx_flags_ok(b.flags, SW, SH, b.coef_off, sizeof(Cf) == 4) &&
                            b.plane < 3 && b.x + Wd <= sel3(pw3, b.plane) && b.y + Ht <= sel3(ph3, b.plane);
            if (!ok) {
                valid = false;
                if (j == 0) atomicOr(a.err, 2);
            }
        }
        const uint8_t *pbase = sel3(plane3, b.plane) + (int64_t)b.y * sel3(stride3, b.plane) + (int64_t)b.x * sizeof(Px);
        const int64_t st = sel3(stride3, b.plane);
#pragma unroll
        for (int c4 = 0; c4 < NCH; c4++) {
            const int c = j + c4 * TPB;
            if (valid && c < Ht * CPR)
                pk[rd][c4] = *reinterpret_cast<const V *>(pbase + (int64_t)(c / CPR) * st + (c % CPR) * 4 * sizeof(Px));
        }
        dk[rd] = valid && b.txtp == 0 && b.eob < 1 ? (int)(reinterpret_cast<const Cf *>(a.coef) + b.coef_off)[0] : 0;
        if constexpr (ROUNDS > 1) {
            const Cf *cq = reinterpret_cast<const Cf *>(a.coef) + b.coef_off;
            const bool need = valid && !(b.txtp == 0 && b.eob < 1) && j < SH;
            if (need) tx_load_row<CW, SH, Cf>(cq, b.flags, j, ck[rd]);
            else
#pragma unroll
                for (int x = 0; x < CW; x++) ck[rd][x] = 0;
        }
        bk[rd] = b;
        vk[rd] = valid;
    }
#ifdef MI_KTL
    {
        // (timeline builds) the first descriptor's arrival: every load above is already issued
        const unsigned d0 = bk[0].coef_off;
        asm volatile("" ::"v"(d0));
        KTL(1);
    }
#endif

    int row_lo, col_lo;
    if constexpr (sizeof(Px) == 1) { row_lo = -32768; col_lo = -32768; }
    else { row_lo = (int)((unsigned)~bdmax << 7); col_lo = (int)((unsigned)~bdmax << 5); }
    const int row_hi = ~row_lo, col_hi = ~col_lo;

#pragma unroll
    for (int rd = 0; rd < ROUNDS; rd++) {
    const MiTxBlock b = bk[rd];
    const bool valid = vk[rd];
    V pix[NCH];
#pragma unroll
    for (int c4 = 0; c4 < NCH; c4++) pix[c4] = pk[rd][c4];
    Cf *cf = reinterpret_cast<Cf *>(a.coef) + b.coef_off;
    const bool wht = (TX == 0) && b.txtp == 16;
    const bool dconly = b.txtp == 0 && b.eob < 1;
    uint8_t *pbase = sel3(plane3, b.plane) + (int64_t)b.y * sel3(stride3, b.plane) + (int64_t)b.x * sizeof(Px);
    const int64_t st = sel3(stride3, b.plane);

    int dc = 0;
    if (valid && dconly) {
        dc = dk[rd];
        if (Rect2) dc = (dc * 181 + 128) >> 8;
        dc = (dc * 181 + 128) >> 8;
        dc = (dc + Rnd) >> Shift;
        dc = (dc * 181 + 128 + 2048) >> 12;
    }
    // ---- 2. row pass ----
    if (valid && !dconly && j < SH) {
        int r[Wd];
#pragma unroll
        for (int x = 0; x < Wd; x++) r[x] = 0;
        int cv[SW];
        if constexpr (ROUNDS > 1) {
#pragma unroll
            for (int x = 0; x < SW; x++) cv[x] = ck[rd][x];
        } else {
            tx_load_row<SW, SH, Cf>(cf, b.flags, j, cv);
        }
#pragma unroll
        for (int x = 0; x < SW; x++) {
            if constexpr (Rect2) r[x] = (cv[x] * 181 + 128) >> 8;
            else r[x] = cv[x];
        }
        if (a.zero_coefs) tx_zero_row<SW, SH, Cf>(cf, b.flags, j);
        if constexpr (TX == 0) {
            if (wht) {
#pragma unroll
                for (int x = 0; x < 4; x++) r[x] >>= 2;
                iwht4(r);
#pragma unroll
                for (int x = 0; x < 4; x++) tmp[j * LS + x] = (Lt)r[x];
            }
        }
        if (!wht) {
            itx1d<Wide, Wd>(k_row_kind[b.txtp], r, row_lo, row_hi);
#pragma unroll
            for (int x = 0; x < Wd; x++)
                tmp[j * LS + x] = (Lt)clampi((r[x] + Rnd) >> Shift, col_lo, col_hi);
        }
    }
    __syncthreads();
    if (rd == 0) KTL(2);

    // ---- 3. column pass: residual back into LDS (rows >= SH are reused as needed) ----
    int colres[Ht];
    if (valid && !dconly && j < Wd) {
        int c[Ht];
#pragma unroll
        for (int y = 0; y < Ht; y++) c[y] = y < SH ? (int)tmp[y * LS + j] : 0;
        if (wht) {
            if constexpr (TX == 0) {
                iwht4(c);
#pragma unroll
                for (int y = 0; y < 4; y++) colres[y] = c[y];
            }
        } else {
            itx1d<Wide, Ht>(k_col_kind[b.txtp], c, col_lo, col_hi);
#pragma unroll
            for (int y = 0; y < Ht; y++) colres[y] = (c[y] + 8) >> 4;
        }
    }
    if constexpr (Ht > SH) {
        // 64-row blocks: the LDS slab only holds 32 rows; write the residual in two halves
        __syncthreads();
#pragma unroll
        for (int half = 0; half < 2; half++) {
            if (valid && !dconly && j < Wd) {
#pragma unroll
                for (int y = 0; y < SH; y++) tmp[y * LS + j] = (Lt)colres[half * SH + y];
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < NCH; k++) {
                const int c = j + k * TPB;
                const int y = c / CPR;
                if (valid && c < Ht * CPR && (y / SH) == half) {
                    int px[4];
                    unpack4<Px>(pix[k], px);
                    const int x0 = (c % CPR) * 4;
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        px[q] = clampi(px[q] + (dconly ? dc : (int)tmp[(y - half * SH) * LS + x0 + q]), 0, bdmax);
                    *reinterpret_cast<V *>(pbase + (int64_t)y * st + x0 * sizeof(Px)) = pack4<Px>(px);
                }
            }
            __syncthreads();
        }
    } else {
        __syncthreads();
        if (valid && !dconly && j < Wd) {
#pragma unroll
            for (int y = 0; y < Ht; y++) tmp[y * LS + j] = (Lt)colres[y];
        }
        __syncthreads();
        // ---- 4. add + vector stores ----
#pragma unroll
        for (int k = 0; k < NCH; k++) {
            const int c = j + k * TPB;
            if (valid && c < Ht * CPR) {
                const int y = c / CPR, x0 = (c % CPR) * 4;
                int px[4];
                unpack4<Px>(pix[k], px);
#pragma unroll
                for (int q = 0; q < 4; q++)
                    px[q] = clampi(px[q] + (dconly ? dc : (int)tmp[y * LS + x0 + q]), 0, bdmax);
                *reinterpret_cast<V *>(pbase + (int64_t)y * st + x0 * sizeof(Px)) = pack4<Px>(px);
            }
        }
    }
    if (valid && dconly && j == 0 && a.zero_coefs) cf[0] = 0;
    if (ROUNDS > 1) __syncthreads();     // the next round reuses this block's LDS rows
    }
}

// DC runs (mi_itx_frame_runs). A DC-only block (DCT_DCT, eob < 1) adds one constant to its
// pixels: the DC coefficient scaled as inv_txfm_add_rust's dc_only path does (src/itx.rs:64-188:
// rect2 scaling, the row shift, the final * 181 >> 12 with rounding). In the size paths such a
// block costs a transform workgroup's whole latency chain for 32-512 bytes; here a one-wave
// workgroup takes itx_dc_blocks(TX) consecutive blocks of one band's DC run: lanes fetch the
// descriptors and DC coefficients into LDS, then sweep the blocks' rows in chunks of min(w, 8)
// pixels, kItxDcItems chunks per lane with every load in flight before the first add.
// Consecutive lanes take a row's chunks, then the next rows, then the next block, so a run of
// neighbouring blocks (sorted by position) is read and written in whole line segments.
template <typename Px, int CP> struct DcVec;
template <> struct DcVec<uint16_t, 8> { using T = uint4; };
template <> struct DcVec<uint16_t, 4> { using T = uint2; };
template <> struct DcVec<uint8_t, 8> { using T = uint2; };
template <> struct DcVec<uint8_t, 4> { using T = uint32_t; };

// pixels + dc, clipped to [0, bdmax], on a vector of CP pixels
template <typename Px, typename V>
__device__ __forceinline__ V dc_add(V v, int dc, int bdmax) {
    constexpr int NW = sizeof(V) / 4;
    uint32_t w[NW];
    __builtin_memcpy(w, &v, sizeof(V));
#pragma unroll
    for (int i = 0; i < NW; i++) {
        if constexpr (sizeof(Px) == 2) {
            const int lo = clampi((int)(w[i] & 0xffff) + dc, 0, bdmax), hi = clampi((int)(w[i] >> 16) + dc, 0, bdmax);
            w[i] = (uint32_t)lo | ((uint32_t)hi << 16);
        } else {
            uint32_t o = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) o |= (uint32_t)clampi((int)((w[i] >> (8 * b)) & 0xff) + dc, 0, bdmax) << (8 * b);
            w[i] = o;
        }
    }
    __builtin_memcpy(&v, w, sizeof(V));
    return v;
}

struct ItxDcRec {
    uint8_t *base;   // the block's top-left pixel; null: skipped
    int st;          // plane stride in bytes
    int dc;          // the constant added to every pixel
};

template <int TX, typename Px, typename Cf>
__device__ __forceinline__ void itx_dc(const ItxArgs &a, int lwg, uint8_t *lds) {
    constexpr TxDim D = tx_dim(TX);
    constexpr int W = D.w, H = D.h, Shift = D.shift, Rnd = (1 << Shift) >> 1;
    constexpr bool Rect2 = (W == 2 * H) || (H == 2 * W);
    constexpr int CP = W < 8 ? W : 8, CW = W / CP, IPB = H * CW, NB = itx_dc_blocks(TX);
    using V = typename DcVec<Px, CP>::T;
    const int lane = threadIdx.x;
    const int q = lwg & 7, k = lwg >> 3;
    const int bs = KARG(band_start, TX * 9 + q) + k * NB;
    const int nb = min(NB, KARG(dc_end, TX * 8 + q) - bs);
    uint8_t *const plane3[3] = { a.plane[0], a.plane[1], a.plane[2] };
    const int64_t stride3[3] = { a.stride[0], a.stride[1], a.stride[2] };
    const int pw3[3] = { a.pw[0], a.pw[1], a.pw[2] }, ph3[3] = { a.ph[0], a.ph[1], a.ph[2] };
    const int64_t dco3[3] = { a.dc_off[0], a.dc_off[1], a.dc_off[2] };
    const int dcs3[3] = { a.dc_stride[0], a.dc_stride[1], a.dc_stride[2] };
    ItxDcRec *rec = reinterpret_cast<ItxDcRec *>(lds);
    // descriptors -> records (base, stride) in LDS; each lane keeps its blocks' DC coefficient
    // load in flight and writes the scaled DC only after the pixel loads below are issued, so
    // that the coefficient and pixel round trips overlap
    constexpr int NR = (NB + 63) / 64;
    int dcv[NR];
    const Cf *dcp[NR];
#pragma unroll
    for (int rr = 0; rr < NR; rr++) {
        const int t = rr * 64 + lane;
        dcp[rr] = nullptr;
        if (t < NB) {
            ItxDcRec r{ nullptr, 0, 0 };
            if (t < nb) {
                const MiTxBlock b = a.blocks[bs + t];
                // a block the run may not hold (another size, not DC-only, outside its plane) is
                // skipped and reported, as the transform path does
                const bool ok = b.tx == TX && b.txtp == 0 && b.eob < 1 && b.plane < 3 &&
                                b.x + W <= sel3(pw3, b.plane) && b.y + H <= sel3(ph3, b.plane);
                if (ok) {
                    dcp[rr] = reinterpret_cast<const Cf *>(a.coef) + b.coef_off;
                    if (a.dc_map) {
                        // MI_ITX_DC_DEFER: the block's first entry of the DC map
                        const int ms = sel3(dcs3, b.plane);
                        r.base = reinterpret_cast<uint8_t *>(a.dc_map + sel3(dco3, b.plane) + (int64_t)(b.y >> 2) * ms + (b.x >> 2));
                        r.st = ms * 4;
                    } else {
                        const int64_t st = sel3(stride3, b.plane);
                        r.base = sel3(plane3, b.plane) + (int64_t)b.y * st + (int64_t)b.x * sizeof(Px);
                        r.st = (int)st;
                    }
                } else {
                    atomicOr(a.err, 2);
                }
            }
            rec[t] = r;
        }
    }
#pragma unroll
    for (int rr = 0; rr < NR; rr++) dcv[rr] = dcp[rr] ? (int)dcp[rr][0] : 0;
    if (a.dc_map) {
        // deferred: every 4x4 unit of the run's blocks gets its block's tagged DC
        constexpr int UW = W / 4, IPBM = UW * (H / 4);
        static_assert(IPBM * NB <= 64 * kItxDcItems, "map items fit the pixel sweep's budget");
#pragma unroll
        for (int rr = 0; rr < NR; rr++) {
            const int t = rr * 64 + lane;
            if (dcp[rr]) {
                int dc = dcv[rr];
                if (a.zero_coefs) *const_cast<Cf *>(dcp[rr]) = 0;
                if (Rect2) dc = (dc * 181 + 128) >> 8;
                dc = (dc * 181 + 128) >> 8;
                dc = (dc + Rnd) >> Shift;
                dc = (dc * 181 + 128 + 2048) >> 12;
                rec[t].dc = dc;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kItxDcItems; i++) {
            const int j = lane + 64 * i, blk = j / IPBM;
            if (i * 64 < IPBM * NB && blk < nb) {
                const ItxDcRec r = rec[blk];
                if (r.base)
                    *reinterpret_cast<uint32_t *>(r.base + (int64_t)((j / UW) % (H / 4)) * r.st + (j % UW) * 4) =
                        (a.dc_tag << 16) | ((uint32_t)r.dc & 0xffffu);
            }
        }
        return;
    }
    __syncthreads();
    V px[kItxDcItems];
#pragma unroll
    for (int i = 0; i < kItxDcItems; i++) {
        const int j = lane + 64 * i, blk = j / IPB;
        if (blk < nb) {
            const ItxDcRec r = rec[blk];
            if (r.base)
                px[i] = *reinterpret_cast<const V *>(r.base + (int64_t)((j / CW) % H) * r.st + (j % CW) * CP * (int)sizeof(Px));
        }
    }
    // the scaled DC of every block into its record (src/itx.rs:64-188 dc_only path)
#pragma unroll
    for (int rr = 0; rr < NR; rr++) {
        const int t = rr * 64 + lane;
        if (dcp[rr]) {
            int dc = dcv[rr];
            if (a.zero_coefs) *const_cast<Cf *>(dcp[rr]) = 0;
            if (Rect2) dc = (dc * 181 + 128) >> 8;
            dc = (dc * 181 + 128) >> 8;
            dc = (dc + Rnd) >> Shift;
            dc = (dc * 181 + 128 + 2048) >> 12;
            rec[t].dc = dc;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kItxDcItems; i++) {
        const int j = lane + 64 * i, blk = j / IPB;
        if (blk < nb) {
            const ItxDcRec r = rec[blk];
            if (r.base)
                *reinterpret_cast<V *>(r.base + (int64_t)((j / CW) % H) * r.st + (j % CW) * CP * (int)sizeof(Px)) =
                    dc_add<Px, V>(px[i], r.dc, a.bdmax);
        }
    }
}

// One launch for every size. The workgroups of the 64- and 32-point sizes come first in the
// grid: they are few but the longest (a 64-point transform per lane, ~15 us at 4K10), so they
// start first and the small sizes fill the machine around them. Measured against two launches
// (sides <= 16, then the rest, each with its own register budget: 66 / 127 VGPRs): 56.3 ->
// 46.4 us at 4K10; the small sizes lose little from the larger register budget, the large
// ones stop being a serial tail.
// (64-point transforms on lane pairs, a persistent grid, and a schedule interleaving every size
// in 4 or 8 rounds were measured slower and removed: DESIGN.md §5)
template <typename Px, typename Cf, typename Lt, bool Wide>
#ifndef MI_ITX_MIN_WAVES
#define MI_ITX_MIN_WAVES 4   // waves per SIMD the register budget must allow (5: 96 VGPRs + 128 B of
                             // spills, 27.8 us; 6: 80 + 220 B, 32.2; 4: 27.6-27.8; r06_itx_waves.txt)
#endif
__global__ __launch_bounds__(kItxThreads, MI_ITX_MIN_WAVES) void itx_frame_kernel(ItxArgs a) {
    __shared__ Lt lds[itx_lds_max(true) > itx_lds_max(false) ? itx_lds_max(true) : itx_lds_max(false)];
    KTL(0);
    const int wg = blockIdx.x;
    // the size range holding this workgroup, with compile-time indices only (a runtime index
    // into the kernel-argument struct makes the compiler copy it to scratch)
    int i = 0;
    for (int k = 1; k < 38; k++)
        if (wg >= KARG(wg_start, k)) i = k;
    const int s = KARG(wg_size, i);
    const int lwg = wg - KARG(wg_start, i);
#ifdef MI_KTL
    {
        // (timeline builds) the size known, before the jump into its path
        asm volatile("" ::"s"(s), "s"(lwg));
        KTL(4);
    }
#endif
    static_assert(sizeof(lds) >= 128 * sizeof(ItxDcRec), "LDS for the DC path's records");
    switch (s) {
#define CASE(n) case n: itx_size<n, Px, Cf, Lt, Wide>(a, lwg, lds); break; \
                case n | kItxDcRange: itx_dc<n, Px, Cf>(a, lwg, reinterpret_cast<uint8_t *>(lds)); break;
        CASE(0) CASE(1) CASE(2) CASE(5) CASE(6) CASE(7) CASE(8) CASE(13) CASE(14)
        CASE(3) CASE(9) CASE(10) CASE(15) CASE(16)
        CASE(4) CASE(11) CASE(12) CASE(17) CASE(18)
#undef CASE
    default: break;
    }
    KTLV(6, s);
    KTL(5);
}

// Where the DC-run ranges go in the grid: 0 before every transform range, 1 after the 64- and
// 32-point sizes' ranges, 2 after every transform range. 4K10 bench frame, graph-timed with a
// fresh arena per call: 33.4-33.8 / 34.1-34.4 / 34.6-35.6 us (the banded grid without runs:
// 36.0-36.5 us)
#ifndef MI_ITX_DC_POS
#define MI_ITX_DC_POS 0
#endif

int itx_fill_schedule(ItxArgs &a, const uint32_t *size_start, const uint32_t *band_start, const uint32_t *dc_end) {
    int wg = 0, r = 0;
    a.nbands = band_start ? kItxBands : 1;
    if (band_start)
        for (int s = 0; s < 19; s++)
            for (int q = 0; q < kItxBands; q++)
                a.dc_end[s][q] = (int)(dc_end ? dc_end[s * kItxBands + q] : band_start[s * (kItxBands + 1) + q]);
    // one range: 8 x the largest band's workgroup count (grid index 8m + q serves band q), or the
    // size's count without bands
    auto add = [&](int sz, bool dcr) {
        a.wg_start[r] = wg;
        a.wg_size[r] = sz | (dcr ? kItxDcRange : 0);
        r++;
        const int per_wg = dcr ? itx_dc_blocks(sz) : itx_blocks_per_wg(sz) * itx_rounds(sz);
        if (band_start) {
            const uint32_t *b = band_start + sz * (kItxBands + 1);
            int m = 0;
            for (int q = 0; q < kItxBands; q++) {
                const int lo = dcr ? (int)b[q] : a.dc_end[sz][q], hi = dcr ? a.dc_end[sz][q] : (int)b[q + 1];
                m = std::max(m, (hi - lo + per_wg - 1) / per_wg);
            }
            wg += kItxBands * m;
        } else if (!dcr) {
            const int n = (int)(size_start[sz + 1] - size_start[sz]);
            wg += (n + per_wg - 1) / per_wg;
        }
    };
    auto add_dc = [&]() {
        for (int i = 18; i >= 0; i--) add(kItxLaunchOrder[i], true);
    };
    if (MI_ITX_DC_POS == 0) add_dc();
    for (int i = 0; i < 19; i++) {
        add(kItxLaunchOrder[i], false);
        if (MI_ITX_DC_POS == 1 && i == 9) add_dc();
    }
    if (MI_ITX_DC_POS == 2) add_dc();
    for (int k = r; k < 39; k++) a.wg_start[k] = wg;
    for (int k = 0; k <= 19; k++) a.blk_start[k] = (int)size_start[k];
    if (band_start)
        for (int s = 0; s < 19; s++)
            for (int q = 0; q <= kItxBands; q++) a.band_start[s][q] = (int)band_start[s * (kItxBands + 1) + q];
    return wg;
}

int launch_itx_frame(const ItxArgs &a, int nwg, int bpc, hipStream_t s) {
    if (nwg <= 0) return 0;
    if (bpc == 8) hipLaunchKernelGGL((itx_frame_kernel<uint8_t, int16_t, int16_t, false>), dim3(nwg), dim3(kItxThreads), 0, s, a);
    else if (bpc == 10) hipLaunchKernelGGL((itx_frame_kernel<uint16_t, int32_t, int16_t, false>), dim3(nwg), dim3(kItxThreads), 0, s, a);
    else hipLaunchKernelGGL((itx_frame_kernel<uint16_t, int32_t, int32_t, true>), dim3(nwg), dim3(kItxThreads), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
