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

namespace mi {

__constant__ int16_t k_gauss[2048] = {
#include "tables/gaussian_sequence.inc"
};
__constant__ uint16_t k_lfsr_jump[256][16];   // M^(24*i) as 16 column vectors

constexpr int kGW = 82, kGH = 73, kDrawsPerLane = 24;
constexpr int kGP = 88;             // pitch of the exported templates (16-byte rows for vector loads)
constexpr int kPrepThreads = 384;   // prep: 3 x 128 lanes (luma, U, V template rows)

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

// Luma and both chroma templates in one skewed wavefront: threads 0-127 own luma rows,
// 128-255 U rows, 256-383 V rows. Chroma sample (r, c) needs the luma samples under it final;
// luma (Y, X) is final after step (X - 3) + skew (Y - 3), so the chroma wavefront can start
// t0 = 1 + max over (r, c) of [last luma step it reads - its own step] steps after the luma
// one, instead of after the whole luma template (8K10 4:2:0, lag 3: 353 steps, not 526).
template <int LAG>
__device__ void grain_ar_all(int16_t (*lut)[kGH][kGW], const MiFilmGrainData &d, bool ly, bool uv0, bool uv1,
                             int cw, int chh, int subx, int suby, int gmin, int gmax) {
    constexpr int NT = 2 * LAG * LAG + 2 * LAG, skew = LAG + 1;
    const int role = threadIdx.x >> 7, lane = threadIdx.x & 127;   // role: wave-uniform
    const int8_t *cg = role == 0 ? d.ar_coeffs_y : d.ar_coeffs_uv[role - 1];
    int coef[NT + 1];
#pragma unroll
    for (int i = 0; i <= NT; i++) coef[i] = cg[i];
    const int gw = role ? cw : kGW, gh = role ? chh : kGH;
    const bool on = role == 0 ? ly : role == 1 ? uv0 : uv1;
    const bool own = on && lane < gh - 3;
    const bool lterm = role && d.num_y_points;
    const int shift = (int)d.ar_coeff_shift;
    const int cmax = cw - 7, rmax = chh - 4;
    const int t0 = 1 + cmax * ((1 << subx) - 1) + subx + skew * (rmax * ((1 << suby) - 1) + suby);
    const int lsteps = (kGW - 6) + skew * (kGH - 4);
    const int csteps = (cw - 6) + skew * (chh - 4);
    const int steps = max(lsteps, uv0 || uv1 ? t0 + csteps : 0);
    const int tstart = role ? t0 : 0;
    int16_t *buf = &lut[role][0][0];
    const int y = 3 + lane;
    // The lane's neighbourhood slides one column per step: rows y-LAG .. y-1 over columns
    // x-LAG .. x+LAG and its own row's last LAG outputs live in registers, so a step reads
    // only the new column x+LAG of the rows above (final: those rows run skew = LAG+1 columns
    // ahead) instead of all NT neighbours.
    constexpr int WA = LAG ? LAG : 1, WC = 2 * LAG + 1;
    int wv[WA][WC], cv[WA];
    bool primed = false;
    for (int t = 0; t < steps; t++) {
        const int x = 3 + (t - tstart) - skew * lane;
        if (own && x >= 3 && x < gw - 3) {
            const int16_t *p = buf + y * kGW + x;
            if constexpr (LAG > 0) {
                if (!primed) {
#pragma unroll
                    for (int r = 0; r < LAG; r++)
#pragma unroll
                        for (int c = 0; c < WC; c++) wv[r][c] = p[(r - LAG) * kGW + c - LAG];
#pragma unroll
                    for (int c = 0; c < LAG; c++) cv[c] = p[c - LAG];
                    primed = true;
                } else {
#pragma unroll
                    for (int r = 0; r < LAG; r++) {
#pragma unroll
                        for (int c = 0; c < WC - 1; c++) wv[r][c] = wv[r][c + 1];
                        wv[r][WC - 1] = p[(r - LAG) * kGW + LAG];
                    }
                }
            }
            // four partial sums: the step's critical path is the multiply-add chain, so it is
            // cut from NT dependent adds to NT / 4 + 2
            int part[4] = { 0, 0, 0, 0 }, ci = 0;
#pragma unroll
            for (int dy = -LAG; dy <= 0; dy++)
#pragma unroll
                for (int dx = -LAG; dx <= LAG; dx++) {
                    if (dy == 0 && dx == 0) break;
                    part[ci & 3] += coef[ci] * (dy < 0 ? wv[dy + LAG][dx + LAG] : cv[dx + LAG]);
                    ci++;
                }
            int sum = (part[0] + part[1]) + (part[2] + part[3]);
            if (lterm) {
                const int lx = ((x - 3) << subx) + 3, ly = ((y - 3) << suby) + 3;
                const int16_t *q = &lut[0][ly][lx];
                int l = q[0];
                if (subx) l += q[1];
                if (suby) { l += q[kGW]; if (subx) l += q[kGW + 1]; }
                sum += round2i(l, subx + suby) * coef[NT];
            }
            const int g = min(max(p[0] + round2i(sum, shift), gmin), gmax);
            buf[y * kGW + x] = (int16_t)g;
            if constexpr (LAG > 0) {
#pragma unroll
                for (int c = 0; c < LAG - 1; c++) cv[c] = cv[c + 1];
                cv[LAG - 1] = g;
            }
        }
        __syncthreads();
    }
}

// Closed form of generate_scaling (fg_apply.rs:14-72) for entry e.
__device__ int scaling_coarse(const uint8_t (*pts)[2], int num, int k /* coarse index */) {
    if (k < pts[0][0]) return pts[0][1];
    if (k >= pts[num - 1][0]) return pts[num - 1][1];
    int i = 0;
    while (i < num - 2 && k >= pts[i + 1][0]) i++;
    const int bx = pts[i][0], by = pts[i][1], dx = pts[i + 1][0] - bx, dy = pts[i + 1][1] - by;
    const int delta = dy * ((0x10000 + (dx >> 1)) / dx);
    return by + ((0x8000 + (k - bx) * delta) >> 16);
}
__device__ int scaling_entry(const uint8_t (*pts)[2], int num, int e, int shx) {
    if (num == 0) return 0;
    const int k = e >> shx, n = e & ((1 << shx) - 1);
    const int base = scaling_coarse(pts, num, k);
    if (!n || k < pts[0][0] || k >= pts[num - 1][0]) return base & 0xff;
    const int next = scaling_coarse(pts, num, k + 1);
    const int range = (next & 0xff) - (base & 0xff);
    const int r = ((1 << shx) >> 1) + n * range;
    return ((base & 0xff) + (r >> shx)) & 0xff;
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

    grain_fill_all(lut, d.seed, shift, ly, uv0, uv1, cw, chh);
    if (!ly)
        for (int i = threadIdx.x; i < kGH * kGW; i += kPrepThreads) (&lut[0][0][0])[i] = a.lut_y[i];
    __syncthreads();
    switch (d.ar_coeff_lag) {
    case 0: grain_ar_all<0>(lut, d, ly, uv0, uv1, cw, chh, a.ss_x, a.ss_y, -gctr, gctr - 1); break;
    case 1: grain_ar_all<1>(lut, d, ly, uv0, uv1, cw, chh, a.ss_x, a.ss_y, -gctr, gctr - 1); break;
    case 2: grain_ar_all<2>(lut, d, ly, uv0, uv1, cw, chh, a.ss_x, a.ss_y, -gctr, gctr - 1); break;
    default: grain_ar_all<3>(lut, d, ly, uv0, uv1, cw, chh, a.ss_x, a.ss_y, -gctr, gctr - 1); break;
    }
    // export templates
    for (int i = threadIdx.x; i < 3 * kGH * kGP; i += kPrepThreads) {
        const int r = i / kGP, c = i - r * kGP;
        a.lut[i] = c < kGW ? (&lut[0][0][0])[r * kGW + c] : 0;
    }

    // scaling LUTs
    const int size = 1 << a.bpc;
    for (int i = threadIdx.x; i < 3 * size; i += kPrepThreads) {
        const int pl = i / size, e = i % size;
        int v = 0;
        if (pl == 0) { if (d.num_y_points || d.chroma_scaling_from_luma) v = scaling_entry(d.y_points, d.num_y_points, e, bdm8); }
        else if (d.num_uv_points[pl - 1]) v = scaling_entry(d.uv_points[pl - 1], d.num_uv_points[pl - 1], e, bdm8);
        a.scaling[pl * 4096 + e] = (uint8_t)v;
    }
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
    return min(max(round2i(a * wa + b * wb, 5), gmin), gmax);
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
                    const int comb = lum[j] * d.uv_luma_mult[p - 1] + sv[j] * d.uv_mult[p - 1];
                    val = min(max((comb >> 6) + d.uv_offset[p - 1] * (1 << bdm8), 0), bdmax);
                }
            }
            const int noise = round2i(scl[val] * g[j], d.scaling_shift);
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
