// mc.hip — frame-batched motion compensation on gfx950.
//
// Replaces the per-block `mc()` driver and compound dispatch of recon (rav1d src/recon.rs:
// 2025-2203, 3236-3428; C recon_tmpl.c:962-1011, 1836-1921) and the DSP mc[10]/mct[10]
// (8-tap and bilinear put/prep), avg, w_avg, mask, w_mask (src/mc.rs; C mc_tmpl.c).
//
// Work decomposition. Units (one block's rectangle in one plane) arrive bucketed by shape
// class (log2 w, log2 h). Every lane owns one output column and R = min(h, 8) consecutive
// rows. A class whose unit needs at most 64 such lanes packs U = min(64 / lanes, 8) units into
// one wave; a larger unit is cut into 64-lane tiles, one wave each. One wave = one workgroup.
//
// Per item: both references' windows (rows + 7) x (cols + 7) are staged in LDS in one loop
// of 4-sample quads with clamped coordinates (identical to emu_edge's replication, mc_tmpl.c:798-845), then a
// single barrier. Each lane evaluates the horizontal 8-tap for its column on its R + 7 rows
// straight from LDS as five v_dot2_i32_i16 on aligned sample pairs (odd columns use the tap
// set shifted by one), feeds the vertical 8-tap through a register window, and blends the
// two predictions in registers (avg / w_avg / mask / w_mask) before the store.
#include "common.h"
#include <type_traits>

MI_KTL_DEFINE(mc)

namespace mi {

__constant__ __attribute__((aligned(8))) int8_t k_subpel[6][15][8] = {
#include "tables/mc_subpel_filters.inc"
};
__constant__ uint8_t k_obmc[64] = {
#include "tables/obmc_masks.inc"
};

typedef short s16x2 __attribute__((ext_vector_type(2)));

#ifndef MC_MAX_U
#define MC_MAX_U 16
#endif
constexpr int kMaxU = MC_MAX_U;    // units packed per wave
// (5 window loads in flight per lane: the one-grid stage 62.0-62.6 us against 65.2-65.8 for 8,
// 63.8-64.2 for 6, 65.8-66.0 for 7, 67.5-68.6 for 4; 12 and 16 spill; same 92 VGPRs for 4-8.
// Fewer slots of a batch fall past a window's last quad, where they repeat a load:
// profiles/r06_mc_batch.txt)
#ifndef MC_STAGE_BATCH
#define MC_STAGE_BATCH 5
#endif
constexpr int kStageBatch = MC_STAGE_BATCH;   // window loads in flight per lane before their LDS stores
constexpr int kWinElems = 2240;    // window budget (elements), 4x16 units: 8 x 23 x 12 = 2208

// LDS window row stride for a tile TW wide: >= TW + 7 samples, a multiple of 4 (quad stores)
__host__ __device__ __forceinline__ int win_stride(int TW) { return (TW + 11) & ~3; }

// units per wave for a class whose unit needs `lanes` lanes and a (TR+7) x (TW+8) window
__host__ __device__ __forceinline__ int units_per_wave(int lanes, int wn) {
    int u = 64 / lanes;
    u = u < kMaxU ? u : kMaxU;
    return u < kWinElems / wn ? u : kWinElems / wn;
}

// filter2d (Filter2d, horizontal/vertical order) -> subpel filter type (0 regular, 1 smooth, 2 sharp)
__device__ __forceinline__ int f2d_type_h(int f) { return (int)((0x111222000ull >> (4 * f)) & 15); }
__device__ __forceinline__ int f2d_type_v(int f) { return (int)((0x210210210ull >> (4 * f)) & 15); }

__device__ __forceinline__ uint32_t pack2(int lo, int hi) { return (uint32_t)(lo & 0xffff) | ((uint32_t)hi << 16); }

// agent-scope (`sc1`) word access for the in-launch mask hand-off of mi_mc_frame_sync
// (MI355X_MICROARCH.md's hand-off rules cover 4-B stores and loads, not bytes)
typedef __attribute__((address_space(1))) uint32_t *mc_gp32;
__device__ __forceinline__ void st_u32_sc1(uint8_t *q, uint32_t v) {
    __hip_atomic_store((mc_gp32)q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_u8_sc1(const uint8_t *q) {
    const uintptr_t ad = reinterpret_cast<uintptr_t>(q);
    const uint32_t w = __hip_atomic_load((mc_gp32)(ad & ~(uintptr_t)3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (int)((w >> (8 * (ad & 3))) & 0xff);
}

// Shape-class geometry (all wave-uniform).
struct ClassGeom {
    int w, h, TW, R, lanes_u, U, T, TR, ctiles;
};

__device__ __forceinline__ ClassGeom class_geom(int c) {
    ClassGeom g;
    g.w = 1 << (c >> 3);
    g.h = 1 << (c & 7);
    g.TW = min(g.w, 64);
    g.R = min(g.h, 8);
    g.lanes_u = g.TW * (g.h / g.R);
    if (g.lanes_u <= 64) {
        g.T = 1;
        g.TR = g.h;
        g.U = units_per_wave(g.lanes_u, (g.TR + 7) * win_stride(g.TW));
        g.ctiles = 1;
    } else {
        g.U = 1;
        g.TR = (64 / g.TW) * g.R;
        g.ctiles = g.w / g.TW;
        g.T = g.ctiles * (g.h / g.TR);
    }
    return g;
}

// unaligned global reads (gfx950 serves them in one access): 4 x u16, 4 x u8
struct __attribute__((packed, aligned(2))) U2a { uint32_t x, y; };
typedef uint32_t U1a __attribute__((aligned(1)));


// Per-lane view of one reference of its unit.
struct RefSel {
    const uint8_t *base;
    int64_t stride;
    int iw, ih, dx, dy, mx, my;
};

// One reference's prediction for this lane's column and R rows (put: pixels, PREP: the int16
// intermediate of mct). All four cases of put/prep_8tap_c and put/prep_bilin_c (2-D, h only,
// v only, copy) run as the 2-D filter: a missing direction gets the identity tap 1 << SH at
// the centre, and every shift on the identity side is exact, e.g. h only, put:
// ((mid << SH) + 2^(SH+ib-1)) >> (SH+ib) == (mid + 2^(ib-1)) >> ib. No lane diverges.
template <bool PREP, int R>
__device__ __forceinline__ void predict(const McArgs &a, const int16_t *win, int WS, const RefSel &s, int f2d,
                                        int w, int h, int col, int r0, int out[8]) {
    const bool bilin = f2d == 9;
    const int SH = bilin ? 4 : 6, ib = a.ib, one = 1 << SH;
    const int th = f2d_type_h(f2d), tv = f2d_type_v(f2d);
    // the 8 taps of a subpel filter are one aligned 8-byte row of k_subpel: two loads per
    // direction instead of eight byte loads
    const uint2 qh = *reinterpret_cast<const uint2 *>(k_subpel[w > 4 ? th : 3 + (th & 1)][max(s.mx, 1) - 1]);
    const uint2 qv = *reinterpret_cast<const uint2 *>(k_subpel[h > 4 ? tv : 3 + (tv & 1)][max(s.my, 1) - 1]);
    int fh[8], fv[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int id = k == 3 ? one : 0;
        const int bh = k == 3 ? 16 - s.mx : k == 4 ? s.mx : 0;
        const int bv = k == 3 ? 16 - s.my : k == 4 ? s.my : 0;
        const int th8 = (int)(int8_t)(((k < 4 ? qh.x : qh.y) >> (8 * (k & 3))) & 0xff);
        const int tv8 = (int)(int8_t)(((k < 4 ? qv.x : qv.y) >> (8 * (k & 3))) & 0xff);
        fh[k] = bilin ? bh : s.mx ? th8 : id;
        fv[k] = bilin ? bv : s.my ? tv8 : id;
    }
    // horizontal taps as 5 aligned pairs: even column (f0,f1)..(f6,f7),(0,0); odd column
    // starts one sample left: (0,f0),(f1,f2),..,(f7,0)
    const bool odd = col & 1;
    uint32_t hp[5];
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const int lo = odd ? (j ? fh[2 * j - 1] : 0) : (j < 4 ? fh[2 * j] : 0);
        const int hi = odd ? (j < 4 ? fh[2 * j] : 0) : (j < 4 ? fh[2 * j + 1] : 0);
        hp[j] = pack2(lo, hi);
    }
    const uint32_t *wrow = reinterpret_cast<const uint32_t *>(win + r0 * WS + (col & ~1));
    const int WS2 = WS >> 1;
    const int hsh = SH - ib, hrnd = (1 << hsh) >> 1;
    auto hmid = [&](int rr) {
        const uint32_t *p = wrow + rr * WS2;
        int s2 = hrnd;
#pragma unroll
        for (int j = 0; j < 5; j++)
            s2 = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, p[j]), __builtin_bit_cast(s16x2, hp[j]), s2, false);
        return s2 >> hsh;
    };
    const int vsh = PREP ? SH : SH + ib, vrnd = (1 << vsh) >> 1;
    int v[8];
#pragma unroll
    for (int t = 0; t < 7; t++) v[t] = hmid(t);
#pragma unroll
    for (int q = 0; q < 8; q++) {
        if (q < R) {
            v[7] = hmid(q + 7);
            int sum = vrnd;
#pragma unroll
            for (int t = 0; t < 8; t++) sum += __mul24(fv[t], v[t]);   // |tap| < 2^7, |mid| < 2^16
            out[q] = PREP ? (sum >> vsh) - a.bias : min(max(sum >> vsh, 0), a.bdmax);
#pragma unroll
            for (int t = 0; t < 7; t++) v[t] = v[t + 1];
        }
    }
}

// (dispatching the classes largest first was measured slower at 4K10: 83 vs 75 us)
template <typename Px>
// g: 0 / 1 = the waves of plane group 0 / 1; 2 = both groups in one grid (group 0's waves,
// then group 1's; mi_mc_frame_ex with MI_MC_ONE_GRID: no chroma unit reads a mask written
// in the same grid), so the small chroma units fill the luma tail.
// (forcing 6 or 8 waves per SIMD, with or without 4 window loads in flight per lane instead
// of 8, spills and measured 73-147 us against 70 us for the two launches: DESIGN.md §5)
__global__ __launch_bounds__(64, 1) void mc_kernel(McArgs a, int g) {
    __shared__ __attribute__((aligned(16))) int16_t win[kWinElems];
    const int lane = threadIdx.x;
    KTL(0);
    int wave = blockIdx.x;
    if (g == 2) {
        g = wave >= (int)a.first_wave[0][MI_MC_NCLASS];
        if (g) wave -= (int)a.first_wave[0][MI_MC_NCLASS];
    }
    const uint32_t *fw = a.first_wave[g];
    // class of this wave: last class whose first wave <= wave (wave-uniform scan)
    int c = 0;
    for (int k = 1; k < MI_MC_NCLASS; k++)
        if (fw[k] <= (uint32_t)wave) c = k;
    int item = wave - (int)fw[c];
    const ClassGeom G = class_geom(c);
    const uint32_t cls_begin = a.class_start[g * MI_MC_NCLASS + c], cls_end = a.class_start[g * MI_MC_NCLASS + c + 1];
    {
        // the class's waves (padded to a multiple of 8, mc_plan) as 8 contiguous chunks, chunk x
        // on XCD x (grid index mod 8): units are in picture order inside a class, so each XCD
        // predicts one band of the picture and reads the reference rows around it into its L2
        const int chunk = (int)(fw[c + 1] - fw[c]) >> 3;
        item = (item & 7) * chunk + (item >> 3);
        const uint32_t n = cls_end - cls_begin;
        if ((uint32_t)item >= (G.T == 1 ? (n + G.U - 1) / G.U : n * G.T)) return;
    }

    // this lane's unit, tile origin, column and rows
    int uu, tx0 = 0, ty0 = 0, rg, col, tile = 0;
    uint32_t ui;
    if (G.T == 1) {
        uu = lane / G.lanes_u;
        const int li = lane - uu * G.lanes_u;
        rg = li / G.TW;
        col = li - rg * G.TW;
        ui = cls_begin + (uint32_t)item * G.U + uu;
    } else {
        uu = 0;
        tile = item % G.T;
        ui = cls_begin + (uint32_t)(item / G.T);
        tx0 = (tile % G.ctiles) * G.TW;
        ty0 = (tile / G.ctiles) * G.TR;
        rg = lane / G.TW;
        col = lane - rg * G.TW;
    }
    const bool active = uu < G.U && ui < cls_end;
    const MiMcBlock b = a.blocks[active ? ui : cls_begin];
    const int p = b.plane;
    const int ssh = p && a.layout != 3, ssv = p && a.layout == 1;
    const int nref = b.ref[1] >= 0 ? 2 : 1;
    RefSel rs[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int r = b.ref[i] >= 0 ? b.ref[i] : b.ref[0];
        const int mvx = b.mvx[i], mvy = b.mvy[i];
        rs[i].base = a.ref[r][p];
        rs[i].stride = a.ref_stride[r][p ? 1 : 0];
        rs[i].iw = a.ref_w[r][p];
        rs[i].ih = a.ref_h[r][p];
        rs[i].mx = (mvx & (15 >> !ssh)) << !ssh;
        rs[i].my = (mvy & (15 >> !ssv)) << !ssv;
        rs[i].dx = b.x + (mvx >> (3 + ssh)) + tx0 - 3;
        rs[i].dy = b.y + (mvy >> (3 + ssv)) + ty0 - 3;
    }

    // stage the references' windows: rows TR + 7, cols TW + 7 (row stride WS, a multiple of
    // 4), as quads of 4 samples (one unaligned 4- or 8-byte load, one 8-byte LDS store),
    // flattened over the unit's staging lanes, kStageBatch quads in flight per lane before
    // their LDS stores; both references of a compound unit are staged before one barrier. Rows are clamped (emu_edge's replication, mc_tmpl.c:798-845); a window that
    // crosses the left or right picture edge clamps per sample.
    const int WR = G.TR + 7, WS = win_stride(G.TW), WN = WR * WS;
    const int Q = WS >> 2;                          // quads per window row
    const uint32_t inv = (1u << 20) / Q + 1;        // (e * inv) >> 20 == e / Q for e < 2^20 / Q^2
    auto stage = [&](const RefSel &r, int16_t *buf) {
        if (!active) return;
        const int li = G.T == 1 ? lane - uu * G.lanes_u : lane;
        const int nl = G.T == 1 ? G.lanes_u : 64;
        const int NE = WR * Q;
        const bool inside = r.dx >= 0 && r.dx + WS <= r.iw;
        int16_t *wdst = buf + uu * WN;
        for (int e0 = li; e0 < NE; e0 += kStageBatch * nl) {
            uint32_t v0[kStageBatch], v1[kStageBatch];
            int o[kStageBatch];
#pragma unroll
            for (int k = 0; k < kStageBatch; k++) {
                const int e = e0 + k * nl;
                const int ec = e < NE ? e : li;
                const int rr = (int)(((uint32_t)ec * inv) >> 20), qq = ec - rr * Q;
                const int yy = min(max(r.dy + rr, 0), r.ih - 1);
                const int x0 = r.dx + 4 * qq;
                const uint8_t *row = r.base + (uint32_t)__umul24((unsigned)yy, (unsigned)r.stride);
                if (inside) {
                    if (sizeof(Px) == 2) {
                        const U2a q = *reinterpret_cast<const U2a *>(row + 2 * x0);
                        v0[k] = q.x;
                        v1[k] = q.y;
                    } else {
                        const uint32_t q = *reinterpret_cast<const U1a *>(row + x0);
                        v0[k] = (q & 0xffu) | ((q & 0xff00u) << 8);
                        v1[k] = ((q >> 16) & 0xffu) | ((q >> 8) & 0xff0000u);
                    }
                } else {
                    int px[4];
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        px[j] = reinterpret_cast<const Px *>(row)[min(max(x0 + j, 0), r.iw - 1)];
                    v0[k] = pack2(px[0], px[1]);
                    v1[k] = pack2(px[2], px[3]);
                }
                o[k] = e < NE ? rr * WS + 4 * qq : -1;
            }
#pragma unroll
            for (int k = 0; k < kStageBatch; k++)
                if (o[k] >= 0) *reinterpret_cast<uint2 *>(wdst + o[k]) = make_uint2(v0[k], v1[k]);
        }
    };
    // One window buffer: a compound unit's references are staged and filtered one after the
    // other (half the LDS of staging both, so twice the waves fit a CU).
    const bool any2 = __any(active && nref == 2);
    stage(rs[0], win);
    __syncthreads();
    KTL(1);

    // mi_mc_frame_sync: a chroma MASK unit whose mask a SEG unit of this grid writes waits for
    // every tile of that unit (the luma waves precede the chroma ones in the grid, so the waves
    // waited for have started); lanes of the unit poll the tile flags in parallel
    const bool after_seg = a.seg_flags && active && b.comp == MI_MC_MASK && (b.param & MI_MC_AFTER_SEG);
    if (a.seg_flags && __any(after_seg)) {
        int tl = 0;
        if (after_seg) {
            const int lw = b.w << ssh, lh = b.h << ssv;    // the producing (luma) SEG unit
            tl = class_geom(((31 - __clz(lw)) << 3) | (31 - __clz(lh))).T;
        }
        const int li = G.T == 1 ? lane - uu * G.lanes_u : lane, nl = G.T == 1 ? G.lanes_u : 64;
        const size_t f0 = (size_t)(b.mask_off >> 4) * 32;
        // a mask offset past the flag buffer (a caller's mask_bytes too small) is reported,
        // never read out of bounds: the unit then waits for nothing
        if (after_seg && f0 + (size_t)tl > a.seg_nflags) {
            atomicOr(a.err, 2);
            tl = 0;
        }
        const uint32_t *fl = a.seg_flags + f0;
        bool ok = true;
        for (unsigned spins = 0;; spins++) {
            ok = true;
            for (int t = li; t < tl; t += nl)
                ok = ok && __hip_atomic_load(fl + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.seg_epoch;
            if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
            if (spins > (1u << 20)) {
                if (!ok) atomicOr(a.err, 1);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        // No acquire (measured +2.5 us): the mask bytes are read below by `sc1`
        // word loads of the polling wave itself, issued after the poll's loads returned (a
        // wave's vector loads issue in program order and the exit branch waits for the poll's
        // data), so they miss every L1 and see the producer's drained `sc1` stores
        // (MI355X_MICROARCH.md, correctness boundaries: every store of the handed-off bytes
        // `sc1`). This compiler barrier keeps those loads below the loop in the emitted code;
        // tests/test_handoff_isa.py checks the result in the shipped code object.
        asm volatile("" ::: "memory");
    }

    // everything after staging runs with the rows per lane R as a compile-time constant
    // (min(h, 8) is wave-uniform): no per-row exec masking in the filters and epilogues
    auto finish = [&](auto RC) {
        constexpr int R = decltype(RC)::value;
        const int r0 = rg * R;
        int o0[8], o1[8];
        const int64_t ds = a.dst_stride[p ? 1 : 0];
        uint8_t *dst = a.dst[p] + (int64_t)(b.y + ty0 + r0) * ds;
        const int x = b.x + tx0 + col;
        const bool prep0 = nref == 2 || b.comp == MI_MC_PREP;
        if (active) {
            if (prep0) predict<true, R>(a, win + uu * WN, WS, rs[0], b.filter2d, b.w, b.h, col, r0, o0);
            else predict<false, R>(a, win + uu * WN, WS, rs[0], b.filter2d, b.w, b.h, col, r0, o0);
        }
        if (any2) {
            __syncthreads();                 // every lane is done reading reference 0
            if (nref == 2) stage(rs[1], win);
            __syncthreads();
            if (active && nref == 2) predict<true, R>(a, win + uu * WN, WS, rs[1], b.filter2d, b.w, b.h, col, r0, o1);
        }
        if (!active) return;
        if (nref == 1) {
            if (b.comp == MI_MC_PREP) {
                // one side of a compound combined later (mi_mc_combine): the mct intermediate
                int16_t *t = a.tmp + b.mask_off + (ty0 + r0) * b.w + tx0 + col;
    #pragma unroll
                for (int q = 0; q < 8; q++)
                    if (q < R) t[q * b.w] = (int16_t)o0[q];
                return;
            }
            if (b.comp == MI_MC_OBMC_H || b.comp == MI_MC_OBMC_V) {
                // OBMC lap blended into the block's prediction (blend_h / blend_v, mc_tmpl.c:636-660)
                const bool above = b.comp == MI_MC_OBMC_H;
                const int yb = ty0 + r0, xb = tx0 + col;
    #pragma unroll
                for (int q = 0; q < 8; q++) {
                    const int y = yb + q;
                    const bool on = q < R && (above ? y < ((b.param * 3) >> 2) : xb < ((b.w * 3) >> 2));
                    if (on) {
                        const int m = k_obmc[above ? b.param + y : b.w + xb];
                        Px *d = reinterpret_cast<Px *>(dst + (int64_t)q * ds) + x;
                        *d = (Px)((*d * (64 - m) + o0[q] * m + 32) >> 6);
                    }
                }
                return;
            }
    #pragma unroll
            for (int q = 0; q < 8; q++)
                if (q < R) reinterpret_cast<Px *>(dst + (int64_t)q * ds)[x] = (Px)o0[q];
            return;
        }
        const int ib = a.ib, sign = b.param >> 7;
        if (b.comp == MI_MC_SEG) {
            // w_mask (mc_tmpl.c:661-712): per-pixel weight from |t1 - t2|, t1 = tmp[sign]
            const int mask_sh = a.bpc + ib - 4, mask_rnd = 1 << (mask_sh - 5);
            const int sh = ib + 6, rnd = (32 << ib) + a.bias * 64;
            const int msh = a.seg_ss_hor, msv = a.seg_ss_ver, mstride = b.w >> msh;
            const int yb = ty0 + r0, xb = tx0 + col;
            uint8_t *mo = a.masks + b.mask_off;
            int mprev = 0;
    #pragma unroll
            for (int q = 0; q < 8; q++) {
                if (q < R) {
                    const int t1 = sign ? o1[q] : o0[q], t2 = sign ? o0[q] : o1[q];
                    const int m = min(38 + ((abs(t1 - t2) + mask_rnd) >> mask_sh), 64);
                    o0[q] = min(max((t1 * m + t2 * (64 - m) + rnd) >> sh, 0), a.bdmax);
                    // neighbour column (lane ^ 1 holds column ^ 1 of the same rows)
                    const int mn = msh ? __shfl_xor(m, 1) : 0;
                    // this lane's mask byte (-1: none at this row) and where it goes
                    int v = -1, row = 0, cb = 0;
                    if (!msh) {
                        v = m; row = yb + q; cb = xb;
                    } else if (!msv) {
                        if (!(col & 1)) { v = (m + mn + 1 - sign) >> 1; row = yb + q; cb = xb >> 1; }
                    } else if (q & 1) {
                        if (!(col & 1)) { v = (mprev + m + mn + 2 - sign) >> 2; row = (yb + q) >> 1; cb = xb >> 1; }
                    } else {
                        mprev = m + mn;
                    }
                    if (!a.seg_flags) {
                        if (v >= 0) mo[row * mstride + cb] = (uint8_t)v;
                    } else {
                        // in-launch hand-off: four bytes of a row to one lane, one `sc1` word store
                        const int st = msh ? 2 : 1;
                        const int v1 = __shfl_down(v, st), v2 = __shfl_down(v, 2 * st), v3 = __shfl_down(v, 3 * st);
                        if (v >= 0 && !(cb & 3))
                            st_u32_sc1(mo + row * mstride + cb, (uint32_t)v | ((uint32_t)v1 << 8) | ((uint32_t)v2 << 16) |
                                                                    ((uint32_t)v3 << 24));
                    }
                }
            }
        } else {
            const uint8_t *mk = a.masks + b.mask_off;
    #pragma unroll
            for (int q = 0; q < 8; q++) {
                if (q < R) {
                    int v;
                    if (b.comp == MI_MC_AVG) {
                        v = (o0[q] + o1[q] + (1 << ib) + a.bias * 2) >> (ib + 1);
                    } else if (b.comp == MI_MC_WAVG) {
                        const int wt = b.param & 31;
                        v = (o0[q] * wt + o1[q] * (16 - wt) + (8 << ib) + a.bias * 16) >> (ib + 4);
                    } else {
                        const uint8_t *mq = mk + (ty0 + r0 + q) * b.w + tx0 + col;
                        const int m = after_seg ? ld_u8_sc1(mq) : *mq;
                        const int t1 = sign ? o1[q] : o0[q], t2 = sign ? o0[q] : o1[q];
                        v = (t1 * m + t2 * (64 - m) + (32 << ib) + a.bias * 64) >> (ib + 6);
                    }
                    o0[q] = min(max(v, 0), a.bdmax);
                }
            }
        }
    #pragma unroll
        for (int q = 0; q < 8; q++)
            if (q < R) reinterpret_cast<Px *>(dst + (int64_t)q * ds)[x] = (Px)o0[q];

    };
    if (G.R == 8) finish(std::integral_constant<int, 8>{});
    else if (G.R == 4) finish(std::integral_constant<int, 4>{});
    else finish(std::integral_constant<int, 2>{});
    // mi_mc_frame_sync: a SEG unit's tile publishes its mask words (the wave drains its stores,
    // then one lane per unit stores the tile's flag, agent scope)
    const bool seg_unit = a.seg_flags && active && nref == 2 && b.comp == MI_MC_SEG;
    if (a.seg_flags && __any(seg_unit)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int li = G.T == 1 ? lane - uu * G.lanes_u : lane;
        const size_t fi = (size_t)(b.mask_off >> 4) * 32 + tile;
        if (seg_unit && li == 0 && fi >= a.seg_nflags) atomicOr(a.err, 2);
        else if (seg_unit && li == 0)
            __hip_atomic_store(a.seg_flags + fi, a.seg_epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    KTLV(6, c + (any2 ? 64 : 0));
    KTL(5);
}

// Waves per class for one plane group: packed small units or one wave per 64-lane tile.
int mc_plan(McArgs &a, int g) {
    uint32_t waves = 0;
    for (int i = 0; i < MI_MC_NCLASS; i++) {
        const int c = i;
        a.first_wave[g][c] = waves;
        const uint32_t n = a.class_start[g * MI_MC_NCLASS + c + 1] - a.class_start[g * MI_MC_NCLASS + c];
        if (!n) continue;
        const int lw = c >> 3, lh = c & 7;
        if (lw < 1 || lh < 1) return -1;                    // widths/heights are 2..128
        const int w = 1 << lw, h = 1 << lh;
        const int TW = w < 64 ? w : 64, R = h < 8 ? h : 8, lanes = TW * (h / R);
        if (lanes <= 64) {
            const int U = units_per_wave(lanes, (h + 7) * win_stride(TW));
            if (U < 1) return -1;                           // shape outside AV1's (aspect > 8:1)
            waves += (n + U - 1) / U;
        } else {
            const int TR = (64 / TW) * R;
            if ((TR + 7) * win_stride(TW) > kWinElems) return -1;
            waves += n * (uint32_t)((w / TW) * (h / TR));
        }
        waves = (waves + 7) & ~7u;   // whole chunks per XCD (mc_kernel)
    }
    a.first_wave[g][MI_MC_NCLASS] = waves;
    return (int)waves;
}

int launch_mc(const McArgs &a, int g, int waves, hipStream_t s) {
    if (waves <= 0) return 0;
    if (a.bpc == 8) mc_kernel<uint8_t><<<waves, 64, 0, s>>>(a, g);
    else mc_kernel<uint16_t><<<waves, 64, 0, s>>>(a, g);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
