// fg.hip — film-grain synthesis on gfx950 (output-only path).
//
// Replaces rav1d_prep_grain / rav1d_apply_grain_row (rav1d src/fg_apply.rs:14-284) and the DSP
// generate_grain_y/uv, fgy_32x32xn, fguv_32x32xn (src/filmgrain.rs:255-830; C
// filmgrain_tmpl.c).
//
// prep (one workgroup, independent of the pixels, so it can run on a side stream at frame
// start): the 16-bit LFSR is linear over GF(2), so lane i jumps straight to its slice of the
// random sequence with a precomputed matrix power and the grain templates fill in parallel;
// the auto-regressive filter runs as a skewed wavefront (row y lags row y-1 by lag+1
// columns, one LDS barrier per step; the chroma templates trail the luma one by just enough
// steps to see final luma grain); scaling LUTs are filled from their closed form; the
// per-(32-row, 32-col) block offsets are drawn by one lane per block row.
// apply: one wave per 512-pixel row segment, lane-contiguous pixels; grain templates and
// offsets are read through L1/L2 (cache resident), the scaling LUT from LDS.
#include "common.h"

MI_KTL_DEFINE(fg)

namespace mi {

__constant__ int16_t k_gauss[2048] = {
#include "tables/gaussian_sequence.inc"
};
__constant__ uint16_t k_lfsr_jump[256][16];   // M^(24*i) as 16 column vectors

constexpr int kGW = 82, kGH = 73, kDrawsPerLane = 24;
constexpr int kGP = 88;             // pitch of the exported templates (16-byte rows for vector loads)
constexpr int kPrepThreads = 448;   // prep: 7 waves (AR: luma, U, V; scaling LUTs: 4)

__device__ __forceinline__ unsigned lfsr_step(unsigned s) {
    const unsigned bit = (s ^ (s >> 1) ^ (s >> 3) ^ (s >> 12)) & 1;
    return ((s >> 1) | (bit << 15)) & 0xffff;
}
__device__ __forceinline__ int round2i(int x, int sh) { return (x + ((1 << sh) >> 1)) >> sh; }

// Random fill of the grain templates (generate_grain_*: first loop), all planes at once: job j
// is lane `j - first job of its plane` of that plane's draw sequence. The 24 LFSR states of a
// job are stepped first, then the 24 table reads issue back to back.
__device__ void grain_fill_all(int16_t (*lut)[kGH][kGW], unsigned seed, int shift, bool ly, bool uv0, bool uv1,
                               int cw, int chh) {
    const int nl = kGW * kGH, nc = cw * chh;
    const int jl = ly ? (nl + kDrawsPerLane - 1) / kDrawsPerLane : 0, jc = (nc + kDrawsPerLane - 1) / kDrawsPerLane;
    const int jobs = jl + (uv0 ? jc : 0) + (uv1 ? jc : 0);
    for (int j = threadIdx.x; j < jobs; j += kPrepThreads) {
        int pl, lane;
        if (j < jl) pl = 0, lane = j;
        else if (uv0 && j < jl + jc) pl = 1, lane = j - jl;
        else pl = 2, lane = j - jl - (uv0 ? jc : 0);
        const unsigned sd = pl == 0 ? seed : pl == 1 ? seed ^ 0xb524 : seed ^ 0x49d8;
        const int gw = pl ? cw : kGW, n = pl ? nc : nl;
        unsigned st = 0;
#pragma unroll
        for (int b = 0; b < 16; b++)
            if ((sd >> b) & 1) st ^= k_lfsr_jump[lane][b];
        int idx[kDrawsPerLane];
#pragma unroll
        for (int k = 0; k < kDrawsPerLane; k++) {
            st = lfsr_step(st);
            idx[k] = (st >> 5) & 0x7ff;
        }
        int v[kDrawsPerLane];
#pragma unroll
        for (int k = 0; k < kDrawsPerLane; k++) v[k] = k_gauss[idx[k]];
        int16_t *buf = &lut[pl][0][0];
        const int d0 = lane * kDrawsPerLane;
        int r = d0 / gw, c = d0 - r * gw;
#pragma unroll
        for (int k = 0; k < kDrawsPerLane; k++) {
            if (d0 + k < n) buf[r * kGW + c] = (int16_t)round2i(v[k], shift);
            if (++c == gw) c = 0, r++;
        }
    }
}

// Closed form of generate_scaling (fg_apply.rs:14-72) for entry e.
__device__ __forceinline__ int scaling_coarse(const uint8_t (*pts)[2], int num, int k /* coarse index */) {
    if (k < pts[0][0]) return pts[0][1];
    if (k >= pts[num - 1][0]) return pts[num - 1][1];
    int i = 0;
    while (i < num - 2 && k >= pts[i + 1][0]) i++;
    const int bx = pts[i][0], by = pts[i][1], dx = pts[i + 1][0] - bx, dy = pts[i + 1][1] - by;
    const int delta = dy * ((0x10000 + (dx >> 1)) / dx);
    return by + ((0x8000 + (k - bx) * delta) >> 16);
}
__device__ __forceinline__ int scaling_entry(const uint8_t (*pts)[2], int num, int e, int shx) {
    if (num == 0) return 0;
    const int k = e >> shx, n = e & ((1 << shx) - 1);
    const int base = scaling_coarse(pts, num, k);
    if (!n || k < pts[0][0] || k >= pts[num - 1][0]) return base & 0xff;
    const int next = scaling_coarse(pts, num, k + 1);
    const int range = (next & 0xff) - (base & 0xff);
    const int r = ((1 << shx) >> 1) + n * range;
    return ((base & 0xff) + (r >> shx)) & 0xff;
}

// Luma and both chroma templates as three in-register wavefronts, one wave each (wave 0 luma,
// 1 U, 2 V). Lane l owns template rows l and l + 64 (all rows, the three border rows included)
// and runs column X of row y at step t = X + skew y (skew = lag + 1), every column of the row
// from -lag on: border samples pass through (out = fill value), interior ones are filtered.
// Then the samples a step needs from the rows above (column X + lag) were produced one step
// earlier by lane l - 1, which holds them as int16 pairs: its last two outputs and, for the
// rows further up, the pair its own window received lag steps before. One wave_ror:1 DPP per
// window row moves a ready pair, the taps are v_dot2_i32_i16 over the pair rings (a register
// ring per window row, indexed by the step: the step loop is unrolled to the ring period so
// every index is a constant), and no barrier, LDS read or branch sits on the per-step path;
// the step's own fill value (and the chroma's luma average) is read one step ahead. Chroma
// sample (r, c) needs the luma samples under it final: the chroma waves run t0 = 1 + max over
// (r, c) of [last luma step it reads - its own step] steps plus one barrier block behind the
// luma one; the waves meet at one barrier per block of steps. The other waves fill the
// scaling LUTs meanwhile, one entry per lane per block.
__device__ __forceinline__ int dpp_from_prev_lane(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x13C /* wave_ror:1: lane l reads lane l - 1 */, 0xf, 0xf, false);
}
typedef short ar_s2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dot2(int pair, int cpair, int acc) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(ar_s2, pair), __builtin_bit_cast(ar_s2, cpair), acc, false);
}
__device__ __forceinline__ int pk16(int lo, int hi) { return (int)__builtin_amdgcn_perm((unsigned)hi, (unsigned)lo, 0x05040100u); }
constexpr int ar_unroll(int lag) { return lag == 3 ? 12 : 4; }   // lcm(window ring 2 lag, output ring 4)
constexpr int ar_block(int lag) { return lag == 3 ? 24 : 16; }   // steps per barrier, a multiple of the unroll

// AR coefficient i of plane pl (0 luma, 1 U, 2 V), read from the kernel-argument segment (a
// role-indexed access into the by-value FgArgs makes the compiler copy it to scratch)
__device__ __forceinline__ int ar_coef(int pl, int i) {
    constexpr size_t y = offsetof(FgArgs, data) + offsetof(MiFilmGrainData, ar_coeffs_y);
    constexpr size_t uv = offsetof(FgArgs, data) + offsetof(MiFilmGrainData, ar_coeffs_uv);
    if (pl == 0) return i < 24 ? karg_at<int8_t>(y + i) : 0;
    return karg_at<int8_t>(uv + (pl == 2 ? 28 : 0) + i);
}

// scaling LUT entry i of the three planes (closed form of generate_scaling)
__device__ __forceinline__ void scaling_at(const FgArgs &a, const uint8_t (*pts)[2], int i) {
    // pts: the y points (14) then the two uv point sets (10 each), staged in LDS
    const MiFilmGrainData &d = a.data;
    const int bdm8 = a.bpc - 8, size = 1 << a.bpc;
    if (i >= 3 * size) return;
    const int pl = i >> a.bpc, e = i & (size - 1);
    int v = 0;
    if (pl == 0) { if (d.num_y_points || d.chroma_scaling_from_luma) v = scaling_entry(pts, d.num_y_points, e, bdm8); }
    else {
        const int n = pl == 1 ? d.num_uv_points[0] : d.num_uv_points[1];
        if (n) v = scaling_entry(pts + 14 + 10 * (pl - 1), n, e, bdm8);
    }
    a.scaling[pl * 4096 + e] = (uint8_t)v;
}

// average of the luma samples under chroma sample (y, x) (filmgrain.rs generate_grain_uv)
__device__ __forceinline__ int luma_avg(const int16_t *q, int subx, int suby) {
    // four reads whatever the subsampling: (a + a + b + b + 2) >> 2 == (a + b + 1) >> 1
    const int sy = suby * kGW;
    return (q[0] + q[subx] + q[sy] + q[sy + subx] + 2) >> 2;
}

template <int LAG, bool LT>
__device__ __forceinline__ int ar_waves(int16_t (*lut)[kGH][kGW], int16_t *dummy, const uint8_t (*pts)[2], const FgArgs &a, bool ly, bool uv0, bool uv1,
                        int cw, int chh, int gmin, int gmax) {
    const MiFilmGrainData &d = a.data;
    const int subx = a.ss_x, suby = a.ss_y;
    constexpr int NT = 2 * LAG * LAG + 2 * LAG, S = LAG + 1, WC = 2 * LAG + 1;
    const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int shift = (int)d.ar_coeff_shift, rnd = (1 << shift) >> 1;
    {
        constexpr int U = ar_unroll(LAG), B = ar_block(LAG), R = 2 * LAG;
        const int gw = role ? cw : kGW, gh = role ? chh : kGH;
        const bool on = role == 0 ? ly : role == 1 ? uv0 : role == 2 ? uv1 : false;
        const int t0 = 1 + (cw - 7) * ((1 << subx) - 1) + subx + S * ((chh - 4) * ((1 << suby) - 1) + suby);
        const int lend = S * (kGH - 1) + kGW;            // last luma step + 1
        const int cend = S * (chh - 1) + cw;
        const int lagc = ly ? t0 + B : 0;
        // every wave starts U steps early (a row is entered lag steps before its column 0)
        const int total = max(ly ? lend + U : 0, uv0 || uv1 ? lagc + cend + U : 0);
        const int tlag = (role == 1 || role == 2 ? lagc : 0) + U;
        int cg[NT + 1];
#pragma unroll
        for (int i = 0; i <= NT; i++) cg[i] = ar_coef(role, i);
        // packed coefficient pairs: window row r, pair k (columns X - LAG + 2k, + 1) and the
        // newest column X + LAG (high half); own row
        int cpr[LAG][LAG + 1], cown[2];
#pragma unroll
        for (int r = 0; r < LAG; r++) {
#pragma unroll
            for (int k = 0; k < LAG; k++) cpr[r][k] = pk16(cg[r * WC + 2 * k], cg[r * WC + 2 * k + 1]);
            cpr[r][LAG] = pk16(0, cg[r * WC + 2 * LAG]);
        }
        const int *co = cg + LAG * WC;   // own row: columns X - LAG .. X - 1
        if (LAG == 3) { cown[0] = pk16(co[1], co[2]); cown[1] = pk16(0, co[0]); }
        else if (LAG == 2) { cown[0] = pk16(co[0], co[1]); cown[1] = 0; }
        else { cown[0] = pk16(0, co[0]); cown[1] = 0; }
        const int lc = cg[NT];
        int16_t *buf = &lut[role < 3 ? role : 0][0][0];
        const int16_t *luma = &lut[0][0][0];
        // per row of the lane (k = 0: row lane, 1: row lane + 64): the step its second row is
        // entered, the column at step t (t - S y), the LDS offset of (y, X) (t + ro), whether
        // (y, X) is inside the template, and the luma offset of the chroma term
        const int y0 = lane, y1 = lane + 64;
        const int thr = S * y1 - LAG;
        const int ro0 = y0 * kGW - S * y0, ro1 = y1 * kGW - S * y1;
        const int lo0 = (((min(max(y0 - 3, 0), gh - 4)) << suby) + 3) * kGW + 3 - ((S * y0 + 3) << subx);
        const int lo1 = (((min(max(y1 - 3, 0), gh - 4)) << suby) + 3) * kGW + 3 - ((S * y1 + 3) << subx);
        // interior iff (unsigned)(t - xs) < gw - 6 (rows outside 3 .. gh - 1 never)
        const int xs0 = y0 >= 3 && y0 < gh ? S * y0 + 3 : -(1 << 28), xs1 = y1 < gh ? S * y1 + 3 : -(1 << 28);
        const int maxoff = kGH * kGW - 1, lmaxoff = maxoff - subx - suby * kGW;   // (the luma average's reach)
        int win[LAG][R], outp[4], outv = 0;
#pragma unroll
        for (int r = 0; r < LAG; r++)
#pragma unroll
            for (int c = 0; c < R; c++) win[r][c] = 0;
#pragma unroll
        for (int c = 0; c < 4; c++) outp[c] = 0;
        // the LDS reads of step t, issued one step ahead: fill value of (y, X), the four luma
        // samples of the chroma term (summed at the step)
        const int sy = suby * kGW;
        auto fetch = [&](int t, int &p0, int &l0, int &l1, int &l2, int &l3) {
            const bool second = t >= thr;
            p0 = buf[min(max(t + (second ? ro1 : ro0), 0), maxoff)];
            if (LT) {
                const int16_t *q = luma + min(max((t << subx) + (second ? lo1 : lo0), 0), lmaxoff);
                l0 = q[0]; l1 = q[subx]; l2 = q[sy]; l3 = q[sy + subx];
            }
        };
        int p0, l0 = 0, l1 = 0, l2 = 0, l3 = 0;
        fetch(-tlag, p0, l0, l1, l2, l3);
        int nb = 0;
        for (int b0 = 0; b0 < total; b0 += B, nb++) {
            if (on) {
                for (int tb = b0 - tlag; tb < b0 - tlag + B; tb += U) {
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const int t = tb + u;
                        // new window pairs (X + LAG - 1, X + LAG): row y - 1 from lane l - 1's last two
                        // outputs, rows further up from the pair its window row r + 1 got LAG steps ago
                        win[LAG - 1][u % R] = dpp_from_prev_lane(outp[(u + 3) % 4]);
#pragma unroll
                        for (int r = 0; r < LAG - 1; r++) win[r][u % R] = dpp_from_prev_lane(win[r + 1][(u + 3 * R - 1 - LAG) % R]);
                        // taps: pair k of row r is ring slot (u - (2 LAG - 1) + 2k), the newest column
                        // the high half of slot u; own columns X - 2, X - 1 = outp(t - 1), X - 3 the
                        // high half of outp(t - 3)
                        // four reads whatever the subsampling: (a + a + b + b + 2) >> 2 == (a + b + 1) >> 1
                        const int lt = LT ? __mul24((l0 + l1 + l2 + l3 + 2) >> 2, lc) : 0;
                        int acc[4] = { rnd + lt, 0, 0, 0 };
#pragma unroll
                        for (int r = 0; r < LAG; r++) {
#pragma unroll
                            for (int k = 0; k < LAG; k++)
                                acc[(r + k) & 3] = dot2(win[r][(u + 3 * R - (2 * LAG - 1) + 2 * k) % R], cpr[r][k], acc[(r + k) & 3]);
                            acc[(r + LAG) & 3] = dot2(win[r][u % R], cpr[r][LAG], acc[(r + LAG) & 3]);
                        }
                        acc[1] = dot2(outp[(u + 3) % 4], cown[0], acc[1]);
                        if (LAG == 3) acc[2] = dot2(outp[(u + 1) % 4], cown[1], acc[2]);
                        const int sum = (acc[0] + acc[1]) + (acc[2] + acc[3]);
                        const bool second = t >= thr;
                        const bool interior = (unsigned)(t - (second ? xs1 : xs0)) < (unsigned)(gw - 6);
                        const int g = interior ? min(max(p0 + (sum >> shift), gmin), gmax) : p0;
                        outp[u % 4] = pk16(outv, g);
                        outv = g;
                        int16_t *dst = interior ? buf + t + (second ? ro1 : ro0) : dummy + lane;
                        *dst = (int16_t)g;
                        fetch(t + 1, p0, l0, l1, l2, l3);
                    }
                }
            } else if (role >= 3) {
                scaling_at(a, pts, (int)threadIdx.x - 192 + 256 * nb);
            }
            __syncthreads();
        }
        return nb;
    }
}

template <int LAG>
__device__ int grain_ar_all(int16_t (*lut)[kGH][kGW], int16_t *dummy, const uint8_t (*pts)[2], const FgArgs &a, bool ly, bool uv0, bool uv1,
                            int cw, int chh, int gmin, int gmax) {
    const MiFilmGrainData &d = a.data;
    const int subx = a.ss_x, suby = a.ss_y;
    constexpr int NT = 2 * LAG * LAG + 2 * LAG, S = LAG + 1, WC = 2 * LAG + 1;
    const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int shift = (int)d.ar_coeff_shift, rnd = (1 << shift) >> 1;
    if constexpr (LAG == 0) {
        // no neighbours: samples are independent (luma first: chroma reads it)
        for (int ph = 0; ph < 2; ph++) {
            const bool on = ph == 0 ? role == 0 && ly : (role == 1 && uv0) || (role == 2 && uv1);
            if (on) {
                const int gw = role ? cw : kGW, gh = role ? chh : kGH;
                const int lc = ar_coef(role, 0);
                const bool lterm = role && d.num_y_points;
                int16_t *buf = &lut[role][0][0];
                for (int e = lane; e < (gh - 3) * (gw - 6); e += 64) {
                    const int i = e / (gw - 6), x = e - i * (gw - 6);
                    int16_t *q = buf + (3 + i) * kGW + 3 + x;
                    const int lt = lterm ? __mul24(luma_avg(&lut[0][(i << suby) + 3][(x << subx) + 3], subx, suby), lc) : 0;
                    *q = (int16_t)min(max(*q + ((lt + rnd) >> shift), gmin), gmax);
                }
            }
            __syncthreads();
        }
        return 0;
    } else {
        const bool lterm = (role == 1 || role == 2) && d.num_y_points;
        return lterm ? ar_waves<LAG, true>(lut, dummy, pts, a, ly, uv0, uv1, cw, chh, gmin, gmax)
                     : ar_waves<LAG, false>(lut, dummy, pts, a, ly, uv0, uv1, cw, chh, gmin, gmax);
    }
}

__global__ __launch_bounds__(kPrepThreads) void fg_prep_kernel(FgArgs a) {
    __shared__ int16_t lut[3][kGH][kGW];
    const MiFilmGrainData &d = a.data;
    const int bdm8 = a.bpc - 8;
    const int shift = 4 - bdm8 + d.grain_scale_shift;
    const int gctr = 128 << bdm8;
    // per-call generate_grain_uv: one chroma template over the caller's luma template
    const bool ly = !a.lut_y;
    const bool uv0 = ly ? a.layout && (d.num_uv_points[0] || d.chroma_scaling_from_luma) : a.uv_only == 1;
    const bool uv1 = ly ? a.layout && (d.num_uv_points[1] || d.chroma_scaling_from_luma) : a.uv_only == 2;
    const int cw = a.ss_x ? 44 : kGW, chh = a.ss_y ? 38 : kGH;

    KTL(0);
    // scaling points staged in LDS (y 14, u 10, v 10 pairs), read before the first barrier
    __shared__ uint8_t pts[34][2];
    {
        constexpr size_t yo = offsetof(FgArgs, data) + offsetof(MiFilmGrainData, y_points);
        constexpr size_t uvo = offsetof(FgArgs, data) + offsetof(MiFilmGrainData, uv_points);
        const int i = threadIdx.x;
        if (i < 28) (&pts[0][0])[i] = karg_at<uint8_t>(yo + i);
        else if (i < 68) (&pts[0][0])[i] = karg_at<uint8_t>(uvo + i - 28);
    }
    grain_fill_all(lut, d.seed, shift, ly, uv0, uv1, cw, chh);
    if (!ly)
        for (int i = threadIdx.x; i < kGH * kGW; i += kPrepThreads) (&lut[0][0][0])[i] = a.lut_y[i];
    __syncthreads();
    KTL(1);
    __shared__ int16_t dummy[64];
    int nb;
    switch (d.ar_coeff_lag) {
    case 0: nb = grain_ar_all<0>(lut, dummy, pts, a, ly, uv0, uv1, cw, chh, -gctr, gctr - 1); break;
    case 1: nb = grain_ar_all<1>(lut, dummy, pts, a, ly, uv0, uv1, cw, chh, -gctr, gctr - 1); break;
    case 2: nb = grain_ar_all<2>(lut, dummy, pts, a, ly, uv0, uv1, cw, chh, -gctr, gctr - 1); break;
    default: nb = grain_ar_all<3>(lut, dummy, pts, a, ly, uv0, uv1, cw, chh, -gctr, gctr - 1); break;
    }
    KTL(2);
    // export templates
    for (int i = threadIdx.x; i < 3 * kGH * kGP; i += kPrepThreads) {
        const int r = i / kGP, c = i - r * kGP;
        a.lut[i] = c < kGW ? (&lut[0][0][0])[r * kGW + c] : 0;
    }
    KTL(3);
    // scaling LUT entries the AR blocks left (waves 3-6 fill 256 per block)
    for (int i = 256 * nb + threadIdx.x; i < 3 << a.bpc; i += kPrepThreads) scaling_at(a, pts, i);
    KTL(4);
}

// Per-block offsets (filmgrain.rs row_seed + one 8-bit draw per 32-wide block along the row):
// one lane per (block row, block). Draw b of a row is the LFSR state after b + 1 steps from
// the row seed: jump by M^(24 q) (k_lfsr_jump) then at most 23 single steps.
__global__ __launch_bounds__(256) void fg_offsets_kernel(FgArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.nrows * a.nblocks) return;
    const int b = i % a.nblocks, row = i / a.nblocks + a.row0;
    unsigned s = a.data.seed;
    s ^= (unsigned)(((row * 37 + 178) & 0xFF) << 8);
    s ^= (unsigned)((row * 173 + 105) & 0xFF);
    s &= 0xffff;
    const int n = b + 1, q = n / kDrawsPerLane, r = n - q * kDrawsPerLane;
    unsigned t = 0;
#pragma unroll
    for (int j = 0; j < 16; j++)
        if ((s >> j) & 1) t ^= k_lfsr_jump[q][j];
    for (int k = 0; k < r; k++) t = lfsr_step(t);
    a.offsets[i] = (uint8_t)((t >> 8) & 0xff);
}

__device__ __forceinline__ int lut_at(const int16_t *lut, int rv, int subx, int suby, int bx, int by, int x, int y) {
    const int ox = 3 + (2 >> subx) * (3 + (rv >> 4));
    const int oy = 3 + (2 >> suby) * (3 + (rv & 0xF));
    return lut[(oy + y + (32 >> suby) * by) * kGP + ox + x + (32 >> subx) * bx];
}

__device__ __forceinline__ int blend(int a, int b, int wa, int wb, int gmin, int gmax) {
    return min(max(round2i(__mul24(a, wa) + __mul24(b, wb), 5), gmin), gmax);
}

// Position of one 8-pixel chunk inside its grain block and the block offsets it needs.
struct GrainPos {
    int sx, sy, yy, xx0, bi;
    int rc, rl, rt, rtl;        // offsets: own block, left, top, top-left
    bool hx, vy;                // inside the horizontal / vertical overlap band
};

// 8 grain samples of template `lut` for a chunk (filmgrain.rs fgy/fguv inner loops, with the
// overlap blends), `g` out. Template loads: three aligned 8-byte loads + a funnel shift.
__device__ __forceinline__ void grain8(const int16_t *lut, const GrainPos &q, int gmin, int gmax, int g[8]) {
    {
        const int ox = 3 + (2 >> q.sx) * (3 + (q.rc >> 4));
        const int oy = 3 + (2 >> q.sy) * (3 + (q.rc & 0xF));
        const int s0 = (oy + q.yy) * kGP + ox + q.xx0, sh = s0 & 3;
        const uint2 *v = reinterpret_cast<const uint2 *>(lut + (s0 - sh));
        const uint2 q0 = v[0], q1 = v[1], q2 = v[2];
        const uint32_t w[6] = { q0.x, q0.y, q1.x, q1.y, q2.x, q2.y };
        uint32_t u[5], o[4];
#pragma unroll
        for (int i = 0; i < 5; i++) u[i] = sh & 2 ? w[i + 1] : w[i];
#pragma unroll
        for (int i = 0; i < 4; i++) o[i] = sh & 1 ? __builtin_amdgcn_alignbyte(u[i + 1], u[i], 2) : u[i];
#pragma unroll
        for (int j = 0; j < 8; j++) g[j] = (int)(int16_t)(o[j >> 1] >> (16 * (j & 1)));
    }
    if (!(q.hx || q.vy)) return;
    const int sx = q.sx, sy = q.sy, yy = q.yy, xx0 = q.xx0;
    const int xstart = q.hx ? 2 >> sx : 0;
    const int wy0 = sy ? 23 : (yy & 1 ? 17 : 27), wy1 = sy ? 22 : (yy & 1 ? 27 : 17);
    int left[2] = { 0, 0 }, top[8], tl[2] = { 0, 0 };
    if (q.hx) {
#pragma unroll
        for (int j = 0; j < 2; j++) left[j] = lut_at(lut, q.rl, sx, sy, 1, 0, xx0 + j, yy);
    }
    if (q.vy) {
#pragma unroll
        for (int j = 0; j < 8; j++) top[j] = lut_at(lut, q.rt, sx, sy, 0, 1, xx0 + j, yy);
        if (q.hx) {
#pragma unroll
            for (int j = 0; j < 2; j++) tl[j] = lut_at(lut, q.rtl, sx, sy, 1, 1, xx0 + j, yy);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const bool inx = j < xstart;
        const int xx = xx0 + j;
        const int wx0 = sx ? 23 : (xx & 1 ? 17 : 27), wx1 = sx ? 22 : (xx & 1 ? 27 : 17);
        if (inx && !q.vy) {
            g[j] = blend(left[j & 1], g[j], wx0, wx1, gmin, gmax);
        } else if (!inx && q.vy) {
            g[j] = blend(top[j], g[j], wy0, wy1, gmin, gmax);
        } else if (inx && q.vy) {
            const int tp = blend(tl[j & 1], top[j], wx0, wx1, gmin, gmax);
            const int gg = blend(left[j & 1], g[j], wx0, wx1, gmin, gmax);
            g[j] = blend(tp, gg, wy0, wy1, gmin, gmax);
        }
    }
}

// 8 pixels <-> one 8-byte (u8) or 16-byte (u16) vector, unpacked to / packed from ints.
__device__ __forceinline__ void unpack8(const uint2 v, int e[8]) {
#pragma unroll
    for (int j = 0; j < 4; j++) { e[j] = (v.x >> (8 * j)) & 0xff; e[4 + j] = (v.y >> (8 * j)) & 0xff; }
}
__device__ __forceinline__ void unpack8(const uint4 v, int e[8]) {
    const uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll
    for (int j = 0; j < 4; j++) { e[2 * j] = w[j] & 0xffff; e[2 * j + 1] = w[j] >> 16; }
}
template <typename Px> struct Vec8;
template <> struct Vec8<uint8_t> {
    using T = uint2;
    static __device__ __forceinline__ T pack(const int e[8]) {
        T v;
        v.x = (uint32_t)e[0] | (uint32_t)e[1] << 8 | (uint32_t)e[2] << 16 | (uint32_t)e[3] << 24;
        v.y = (uint32_t)e[4] | (uint32_t)e[5] << 8 | (uint32_t)e[6] << 16 | (uint32_t)e[7] << 24;
        return v;
    }
};
template <> struct Vec8<uint16_t> {
    using T = uint4;
    static __device__ __forceinline__ T pack(const int e[8]) {
        T v;
        v.x = (uint32_t)e[0] | (uint32_t)e[1] << 16;
        v.y = (uint32_t)e[2] | (uint32_t)e[3] << 16;
        v.z = (uint32_t)e[4] | (uint32_t)e[5] << 16;
        v.w = (uint32_t)e[6] | (uint32_t)e[7] << 16;
        return v;
    }
};

template <typename Px>
__device__ __forceinline__ void load8(int e[8], const Px *src, int n) {
    if (n == 8) {
        unpack8(*reinterpret_cast<const typename Vec8<Px>::T *>(src), e);
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) e[j] = j < n ? src[j] : 0;
    }
}

template <typename Px>
__device__ __forceinline__ void store8(Px *dst, const int e[8], int n) {
    if (n == 8) {
        *reinterpret_cast<typename Vec8<Px>::T *>(dst) = Vec8<Px>::pack(e);
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (j < n) dst[j] = (Px)e[j];
    }
}

// One lane per 8-pixel chunk of a plane row, one wave per 512-pixel row segment (fgy_32x32xn /
// fguv_32x32xn, filmgrain.rs:404-830, re-cut by output chunk). A chunk never straddles a grain
// block (32 wide, 16 when subsampled), so the block offset and the column inside the block are
// per chunk; overlap blending touches only the first 2 (1) columns and rows of a block, and its
// loads are issued together inside one branch. The scaling LUT is staged in LDS while the pixel
// loads are in flight.
template <typename Px>
__global__ __launch_bounds__(256) void fg_apply_kernel(FgArgs a) {
    __shared__ uint32_t scl32[1024];
    const uint8_t *scl = reinterpret_cast<const uint8_t *>(scl32);
    const int b = blockIdx.x;
    const int p = b < a.blk_start[1] ? 0 : b < a.blk_start[2] ? 1 : 2;
    const MiFilmGrainData &d = a.data;
    const bool grain = a.grain[p];
    const int wpr = a.chunks[p];   // waves per plane row
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pw = a.pw[p], ph = a.ph[p];
    const int64_t st = a.stride[p];
    const int sx = p ? a.ss_x : 0, sy = p ? a.ss_y : 0;
    const int bdm8 = a.bpc - 8, bdmax = (1 << a.bpc) - 1;
    const int gctr = 128 << bdm8, gmin = -gctr, gmax = gctr - 1;
    int minv = 0, maxv = bdmax;
    if (d.clip_to_restricted_range) {
        minv = 16 << bdm8;
        maxv = (p == 0 || a.is_id ? 235 : 240) << bdm8;
    }

    // the scaling LUT (1 << bpc entries) staged once per workgroup, for kFgItems wave-items
    // per wave (a workgroup per single row segment spent as many loads on the LUT as on pixels)
    if (grain) {
        const int nw = (1 << a.bpc) >> 2;
        const uint32_t *g = reinterpret_cast<const uint32_t *>(
            a.scaling + (p && !d.chroma_scaling_from_luma ? p : 0) * 4096);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int i = threadIdx.x + 256 * k;
            if (i < nw) scl32[i] = g[i];
        }
        __syncthreads();
    }

    for (int it = 0; it < kFgItems; it++) {
        const int t = ((b - a.blk_start[p]) * kFgItems + it) * 4 + wave;
        const int y = t / wpr, seg = t - y * wpr;
        const int x0 = (seg * 64 + (threadIdx.x & 63)) * 8;
        const bool active = y < ph && x0 < pw;
        if (!__builtin_amdgcn_readfirstlane((int)(y < ph))) break;    // past the plane: wave-uniform
        const int n = active ? min(8, pw - x0) : 0;
        const Px *src = reinterpret_cast<const Px *>(a.src[p] + (int64_t)y * st) + x0;
        Px *dst = reinterpret_cast<Px *>(a.dst[p] + (int64_t)y * st) + x0;
        if (!grain) {   // uniform per workgroup: plain copy
            if (active) {
                int e[8];
                load8(e, src, n);
                store8(dst, e, n);
            }
            continue;
        }
        if (!active) continue;
        int sv[8];
        load8(sv, src, n);

        // co-located luma (chroma planes): 8 << sx samples from x0 << sx, clamped at w - 1
        int lum[8];
        if (p) {
            const int lx0 = x0 << sx;
            const Px *luma = reinterpret_cast<const Px *>(a.src[0] + (int64_t)(y << sy) * a.stride[0]);
            if (sx) {
                int l0[8], l1[8];
                if (lx0 + 16 <= a.w) {
                    load8(l0, luma + lx0, 8);
                    load8(l1, luma + lx0 + 8, 8);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        l0[j] = luma[min(lx0 + j, a.w - 1)];
                        l1[j] = luma[min(lx0 + 8 + j, a.w - 1)];
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    lum[j] = (l0[2 * j] + l0[2 * j + 1] + 1) >> 1;
                    lum[4 + j] = (l1[2 * j] + l1[2 * j + 1] + 1) >> 1;
                }
            } else if (n == 8) {
                load8(lum, luma + lx0, 8);
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++) lum[j] = luma[min(lx0 + j, a.w - 1)];
            }
        }

        // grain samples of this chunk's block
        int g[8];
        {
            GrainPos q;
            q.sx = sx; q.sy = sy;
            const int bsh = 32 >> sy, bsw = 32 >> sx;
            const int lrow = y >> (5 - sy), row = lrow + a.row_off;
            q.yy = y & (bsh - 1);
            q.bi = x0 >> (5 - sx);
            q.xx0 = x0 & (bsw - 1);
            const uint8_t *offr = a.offsets + row * a.nblocks;
            const uint8_t *offp = row ? offr - a.nblocks : offr;
            q.rc = offr[q.bi];
            q.hx = q.vy = false;
            q.rl = q.rt = q.rtl = 0;
            if (d.overlap_flag) {
                const int bh = p ? (min(a.h - lrow * 32, 32) + sy) >> sy : min(a.h - lrow * 32, 32);
                const int ystart = row ? min(2 >> sy, bh) : 0;
                q.hx = q.bi > 0 && q.xx0 == 0;     // blocks are >= 1 px wide: xstart > 0 iff bi > 0
                q.vy = q.yy < ystart;
                if (q.hx) q.rl = offr[q.bi - 1];
                if (q.vy) q.rt = offp[q.bi];
                if (q.hx && q.vy) q.rtl = offp[q.bi - 1];
            }
            grain8(a.lut + p * kGH * kGP, q, gmin, gmax, g);
        }

        int ov[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            int val = sv[j];
            if (p) {
                val = lum[j];
                if (!d.chroma_scaling_from_luma) {
                    const int comb = __mul24(lum[j], (int)d.uv_luma_mult[p - 1]) + __mul24(sv[j], (int)d.uv_mult[p - 1]);
                    val = min(max((comb >> 6) + d.uv_offset[p - 1] * (1 << bdm8), 0), bdmax);
                }
            }
            const int noise = round2i(__mul24((int)scl[val], g[j]), d.scaling_shift);
            ov[j] = min(max(sv[j] + noise, minv), maxv);
        }
        store8(dst, ov, n);
    }
}

int init_fg_tables() {
    // columns of the LFSR step matrix M, then M^(24 i) by repeated multiplication
    uint16_t m[16], p[16], host[256][16];
    auto step = [](unsigned s) {
        const unsigned bit = (s ^ (s >> 1) ^ (s >> 3) ^ (s >> 12)) & 1;
        return (uint16_t)(((s >> 1) | (bit << 15)) & 0xffff);
    };
    auto apply = [](const uint16_t *mat, unsigned v) {
        unsigned r = 0;
        for (int j = 0; j < 16; j++)
            if ((v >> j) & 1) r ^= mat[j];
        return (uint16_t)r;
    };
    for (int j = 0; j < 16; j++) m[j] = step(1u << j);
    uint16_t m24[16];
    for (int j = 0; j < 16; j++) {
        unsigned v = 1u << j;
        for (int k = 0; k < kDrawsPerLane; k++) v = apply(m, v);
        m24[j] = (uint16_t)v;
    }
    for (int j = 0; j < 16; j++) p[j] = (uint16_t)(1u << j);   // identity
    for (int i = 0; i < 256; i++) {
        for (int j = 0; j < 16; j++) host[i][j] = p[j];
        uint16_t q[16];
        for (int j = 0; j < 16; j++) q[j] = apply(m24, p[j]);
        for (int j = 0; j < 16; j++) p[j] = q[j];
    }
    return hipMemcpyToSymbol(HIP_SYMBOL(k_lfsr_jump), host, sizeof(host)) == hipSuccess ? 0 : -5;
}

int launch_fg(const FgArgs &a, hipStream_t s, bool prep, bool apply) {
    if (prep) {
        hipLaunchKernelGGL(fg_prep_kernel, dim3(1), dim3(kPrepThreads), 0, s, a);
        const int nb = a.nrows * a.nblocks;
        if (nb > 0) hipLaunchKernelGGL(fg_offsets_kernel, dim3((nb + 255) / 256), dim3(256), 0, s, a);
    }
    if (apply && a.blk_start[3] > 0) {
        if (a.bpc == 8) fg_apply_kernel<uint8_t><<<a.blk_start[3], 256, 0, s>>>(a);
        else fg_apply_kernel<uint16_t><<<a.blk_start[3], 256, 0, s>>>(a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// per-call fgy / fguv_32x32xn: the caller's templates and scaling are already in a.lut /
// a.scaling; draw the block offsets of this row (and the one above) and apply
int launch_fg_call(const FgArgs &a, hipStream_t s) {
    const int nb = a.nrows * a.nblocks;
    if (nb > 0) hipLaunchKernelGGL(fg_offsets_kernel, dim3((nb + 255) / 256), dim3(256), 0, s, a);
    if (a.blk_start[3] > 0) {
        if (a.bpc == 8) fg_apply_kernel<uint8_t><<<a.blk_start[3], 256, 0, s>>>(a);
        else fg_apply_kernel<uint16_t><<<a.blk_start[3], 256, 0, s>>>(a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
