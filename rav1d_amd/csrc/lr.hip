// lr.hip — whole-frame loop restoration (Wiener / self-guided) on gfx950.
//
// Replaces rav1d_lr_sbrow / lr_sbrow / lr_stripe (rav1d src/lr_apply.rs:28-329) and the DSP
// lr.wiener[2] / lr.sgr[3] (src/looprestoration.rs:139-912; C looprestoration_tmpl.c).
//
// The reference works in place, unit by unit, keeping the pre-LR left columns of the previous
// unit and a line buffer of deblocked rows around every stripe boundary. Reading the CDEF output
// C (immutable) inside the stripe and the deblocked picture D for the rows beyond a stripe edge
// gives exactly the samples it sees, so every (stripe, 32/64-px column tile) is independent:
// one 512-lane workgroup each (8 waves, so 4 resident tiles fill a CU), the (h+6) x (w+6)
// window staged once in LDS, both filter passes
// (or the box sums and the A/B maps of the self-guided filter) computed from LDS, and the
// output streamed to a separate picture O.
#include "common.h"

MI_KTL_DEFINE(lr)

namespace mi {

constexpr int kLrWin = 80;             // LDS window row stride (int16): columns x0-8 .. x0+71
constexpr int kWX = 8;                 // window column of x0 (8-px aligned halo: vector staging)
constexpr int kLrAB = 68;              // A/B row stride
constexpr int kNY = 8;                 // waves (row groups) per workgroup
constexpr int kNR = 64 / kNY;          // output rows per lane
constexpr int kNT = 64 * kNY;          // lanes per workgroup
constexpr int kWL = (70 + kNY - 1) / kNY;   // window rows loaded per lane

__constant__ uint16_t k_sgr_params[16][2] = {
    { 140, 3236 }, { 112, 2158 }, { 93, 1618 }, { 80, 1438 }, { 70, 1295 }, { 58, 1177 },
    { 47, 1079 },  { 37, 996 },   { 30, 925 },  { 25, 863 },  { 0, 2589 },  { 0, 1618 },
    { 0, 1177 },   { 0, 925 },    { 56, 0 },    { 22, 0 },
};

__device__ __forceinline__ unsigned sgr_x_by_x(unsigned z) {
    // round(256 / (z + 1)), pinned to 255 at z = 0 and 0 at z = 255 (dav1d_sgr_x_by_x)
    if (z == 0) return 255;
    if (z >= 255) return 0;
    return (256 + ((z + 1) >> 1)) / (z + 1);
}

template <typename Px>
__device__ __forceinline__ int ld_px(const uint8_t *base, int64_t stride, int y, int x) {
    return reinterpret_cast<const Px *>(base + (int64_t)y * stride)[x];
}

// Self-guided A/B maps (looprestoration.rs selfguided_filter, first half) by column pairs:
// lane (g, cp) owns positions x = 2cp - 2 and x + 1 (x even, so
// the six window samples x-2 .. x+3 are three aligned 32-bit LDS reads per row serving both
// columns' horizontal sums, instead of 2 x (2R+1) 16-bit reads). 34 pairs x 15 row groups.
template <int R>
__device__ void sgr_ab(const int16_t *win, int *A, int16_t *B, int sh, int tw, unsigned s, int bdm8,
                        const uint8_t *xbyx) {
    constexpr int n = (2 * R + 1) * (2 * R + 1);
    constexpr unsigned one_by_x = n == 25 ? 164 : 455;
    constexpr int NP = 34, G = kNT / NP;
    const int g = threadIdx.x / NP, cp = threadIdx.x - g * NP;
    const int x = 2 * cp - 2;                          // positions x, x + 1 (valid: -1 .. tw)
    if (g >= G || x > tw) return;
    const int nrows = sh + 2;
    // R = 2 keeps A/B on odd rows only: an even row count per group starts every group on an
    // odd row, so the row parity test below is the same for all lanes (no divergent halves)
    const int per = R == 2 ? (((nrows + G - 1) / G) + 1) & ~1 : (nrows + G - 1) / G;
    const int y0 = -1 + g * per, y1 = min(-1 + (g + 1) * per, sh + 1);
    if (y0 >= y1) return;
    const uint32_t *col = reinterpret_cast<const uint32_t *>(win + x - 2 + kWX);
    constexpr int W2 = kLrWin / 2;
    auto hsum = [&](int yy, int &s0, int &q0, int &s1, int &q1) {
        const uint32_t *r = col + (yy + 3) * W2;
        const uint32_t w0 = r[0], w1 = r[1], w2 = r[2];
        const int v0 = w0 & 0xffff, v1 = w0 >> 16, v2 = w1 & 0xffff, v3 = w1 >> 16, v4 = w2 & 0xffff, v5 = w2 >> 16;
        if (R == 2) {
            const int m = v1 + v2 + v3 + v4, mq = v1 * v1 + v2 * v2 + v3 * v3 + v4 * v4;
            s0 = m + v0; q0 = mq + v0 * v0; s1 = m + v5; q1 = mq + v5 * v5;
        } else {
            const int m = v2 + v3, mq = v2 * v2 + v3 * v3;
            s0 = m + v1; q0 = mq + v1 * v1; s1 = m + v4; q1 = mq + v4 * v4;
        }
    };
    int rs0[2 * R + 1], rq0[2 * R + 1], rs1[2 * R + 1], rq1[2 * R + 1];
#pragma unroll
    for (int k = 0; k < 2 * R; k++) hsum(y0 - R + k, rs0[k], rq0[k], rs1[k], rq1[k]);
    const bool c0 = x >= -1, c1 = x + 1 <= tw;
    for (int y = y0; y < y1; y++) {
        hsum(y + R, rs0[2 * R], rq0[2 * R], rs1[2 * R], rq1[2 * R]);
        if (R == 1 || !((y + 1) & 1)) {
            int sum0 = 0, sq0 = 0, sum1 = 0, sq1 = 0;
#pragma unroll
            for (int k = 0; k <= 2 * R; k++) { sum0 += rs0[k]; sq0 += rq0[k]; sum1 += rs1[k]; sq1 += rq1[k]; }
            const int sums[2] = { sum0, sum1 }, sqs[2] = { sq0, sq1 };
            const bool on[2] = { c0, c1 };
#pragma unroll
            for (int e = 0; e < 2; e++) {
                // a, b < 2^21 (25 squares of 8-bit-scaled samples) and xv * one_by_x < 2^17, sums
                // < 2^17: 24-bit multiplies (full rate) except p * s, which wraps in u32 as the
                // reference's does
                const int a = (sqs[e] + ((1 << (2 * bdm8)) >> 1)) >> (2 * bdm8);
                const int b = (sums[e] + ((1 << bdm8) >> 1)) >> bdm8;
                const unsigned p = (unsigned)max((int)__umul24((unsigned)a, (unsigned)n) - (int)__umul24((unsigned)b, (unsigned)b), 0);
                const unsigned z = (p * s + (1u << 19)) >> 20;
                const unsigned xv = xbyx[min(z, 255u)];
                if (on[e]) {
                    A[(y + 1) * kLrAB + x + e + 1] = (int)((__umul24(__umul24(xv, one_by_x), (unsigned)sums[e]) + (1u << 11)) >> 12);
                    B[(y + 1) * kLrAB + x + e + 1] = (int16_t)xv;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 2 * R; k++) { rs0[k] = rs0[k + 1]; rq0[k] = rq0[k + 1]; rs1[k] = rs1[k + 1]; rq1[k] = rq1[k + 1]; }
    }
}

// Self-guided output terms for rows r0..r0+kNR-1 of column i (looprestoration.rs selfguided_filter
// tail). The lane walks down its column keeping, per A/B row, the centre value c and the sum of
// its two horizontal neighbours s in registers: 3 A + 3 B LDS reads per row instead of 9 + 9.
template <int R>
__device__ __forceinline__ void sgr_px(const int *A, const int16_t *B, int r0, int r1, int i,
                                       const int16_t *win, int w, int acc[kNR]) {
    const int *a0 = A + i + 1;
    const int16_t *b0 = B + i + 1;
    auto ld = [&](int y, int &ca, int &sa, int &cb, int &sb) {
        const int *ar = a0 + (y + 1) * kLrAB;
        const int16_t *br = b0 + (y + 1) * kLrAB;
        ca = ar[0]; sa = ar[-1] + ar[1];
        cb = br[0]; sb = br[-1] + br[1];
    };
    if (R == 1) {
        int ca0, sa0, cb0, sb0, ca1, sa1, cb1, sb1, ca2, sa2, cb2, sb2;
        ld(r0 - 1, ca0, sa0, cb0, sb0);
        ld(r0, ca1, sa1, cb1, sb1);
#pragma unroll
        for (int q = 0; q < kNR; q++) {
            ld(r0 + q + 1, ca2, sa2, cb2, sb2);
            if (r0 + q < r1) {
                const int src = win[(r0 + q + 3) * kLrWin + i + kWX];
                const int a = (cb1 + sb1 + cb0 + cb2) * 4 + (sb0 + sb2) * 3;
                const int b = (ca1 + sa1 + ca0 + ca2) * 4 + (sa0 + sa2) * 3;
                acc[q] += w * ((b - a * src + (1 << 8)) >> 9);
            }
            ca0 = ca1; sa0 = sa1; cb0 = cb1; sb0 = sb1;
            ca1 = ca2; sa1 = sa2; cb1 = cb2; sb1 = sb2;
        }
    } else {
        // A/B exist on odd rows: even j uses rows j-1 and j+1, odd j uses row j (r0 is even)
        int cau, sau, cbu, sbu, cad, sad, cbd, sbd;
        ld(r0 - 1, cau, sau, cbu, sbu);
#pragma unroll
        for (int q = 0; q < kNR; q += 2) {
            ld(r0 + q + 1, cad, sad, cbd, sbd);
            if (r0 + q < r1) {
                const int src = win[(r0 + q + 3) * kLrWin + i + kWX];
                const int a = (cbu + cbd) * 6 + (sbu + sbd) * 5;
                const int b = (cau + cad) * 6 + (sau + sad) * 5;
                acc[q] += w * ((b - a * src + (1 << 8)) >> 9);
            }
            if (r0 + q + 1 < r1) {
                const int src = win[(r0 + q + 4) * kLrWin + i + kWX];
                const int a = cbd * 6 + sbd * 5;
                const int b = cad * 6 + sad * 5;
                acc[q + 1] += w * ((b - a * src + (1 << 7)) >> 8);
            }
            cau = cad; sau = sad; cbu = cbd; sbu = sbd;
        }
    }
}

// Wiener horizontal pass (looprestoration.rs:299-335) by column pairs: lane (rg, cp) filters
// columns 2cp and 2cp + 1 of rows rg, rg + 16, ...: the ten samples x-4 .. x+5 are five aligned
// 32-bit LDS reads (2.5 per output instead of 7) and the pair is one 32-bit store.
__device__ __forceinline__ void wiener_hor(const int16_t *win, int16_t *hor, int wr, int tw, const int (&fh)[7],
                                           int bd, int rbh, int clip_h) {
    const int cp = threadIdx.x & 31, rg = threadIdx.x >> 5, x = 2 * cp;
    if (x >= tw) return;
    for (int rr = rg; rr < wr; rr += kNT / 32) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(win + rr * kLrWin + x + kWX - 4);
        int v[10];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const uint32_t q = w[k];
            v[2 * k] = (int)(int16_t)(q & 0xffffu);
            v[2 * k + 1] = (int)(int16_t)(q >> 16);
        }
        int s0 = 1 << (bd + 6), s1 = s0;
#pragma unroll
        for (int t = 0; t < 7; t++) { s0 += v[t + 1] * fh[t]; s1 += v[t + 2] * fh[t]; }
        const int h0 = min(max((s0 + (1 << (rbh - 1))) >> rbh, 0), clip_h);
        const int h1 = min(max((s1 + (1 << (rbh - 1))) >> rbh, 0), clip_h);
        *reinterpret_cast<uint32_t *>(hor + rr * 64 + x) = (uint32_t)(h0 & 0xffff) | ((uint32_t)h1 << 16);
    }
}

// Self-guided filter tail by column pairs (looprestoration.rs:566-912): lane (rg, cp) owns
// columns 2cp, 2cp + 1 and rows 4rg .. 4rg + 3. Per A/B row the four entries x-1 .. x+2 are two
// 32-bit reads of each map (A int, B int16: 3 reads) for both columns instead of 6 per column.
// Runs both radii as the frame has them and leaves the finished tile in B (row stride 64).
__device__ __forceinline__ void sgr_pairs(int *A, int16_t *B, const int16_t *win, int sh, int tw, int bdm8, int s0,
                                          int s1, int w0, int w1, const uint8_t *xbyx, int bdmax) {
    const int cp = threadIdx.x & 31, rg = threadIdx.x >> 5, x = 2 * cp;
    const int r0 = rg * 4, r1 = min(r0 + 4, sh);
    int acc[2][4] = {};
    // c: centre, s: left + right neighbours, for columns x (e = 0) and x + 1 (e = 1)
    auto ld = [&](int y, int (&ca)[2], int (&sa)[2], int (&cb)[2], int (&sb)[2]) {
        const int *ar = A + (y + 1) * kLrAB + x;            // entries x-1 .. x+2 at ar[0..3]
        const int16_t *br = B + (y + 1) * kLrAB + x;
        const int2 a01 = *reinterpret_cast<const int2 *>(ar), a23 = *reinterpret_cast<const int2 *>(ar + 2);
        const uint32_t b01 = *reinterpret_cast<const uint32_t *>(br), b23 = *reinterpret_cast<const uint32_t *>(br + 2);
        const int bv0 = (int16_t)(b01 & 0xffff), bv1 = (int16_t)(b01 >> 16), bv2 = (int16_t)(b23 & 0xffff),
                  bv3 = (int16_t)(b23 >> 16);
        ca[0] = a01.y; sa[0] = a01.x + a23.x; ca[1] = a23.x; sa[1] = a01.y + a23.y;
        cb[0] = bv1; sb[0] = bv0 + bv2; cb[1] = bv2; sb[1] = bv1 + bv3;
    };
    auto src2 = [&](int j, int (&v)[2]) {
        const uint32_t q = *reinterpret_cast<const uint32_t *>(win + (j + 3) * kLrWin + x + kWX);
        v[0] = (int16_t)(q & 0xffff); v[1] = (int16_t)(q >> 16);
    };
    const bool act = x < tw && r0 < r1;
    if (s0) {
        sgr_ab<2>(win, A, B, sh, tw, (unsigned)s0, bdm8, xbyx);
        __syncthreads();
        KTL(2);
        if (act) {
            // A/B on odd rows: even j uses rows j-1 and j+1, odd j row j (r0 is even)
            int cau[2], sau[2], cbu[2], sbu[2], cad[2], sad[2], cbd[2], sbd[2];
            ld(r0 - 1, cau, sau, cbu, sbu);
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                ld(r0 + q + 1, cad, sad, cbd, sbd);
                int v[2];
                if (r0 + q < r1) {
                    src2(r0 + q, v);
#pragma unroll
                    for (int e = 0; e < 2; e++) {
                        const int a = (cbu[e] + cbd[e]) * 6 + (sbu[e] + sbd[e]) * 5;
                        const int b = (cau[e] + cad[e]) * 6 + (sau[e] + sad[e]) * 5;
                        acc[e][q] += __mul24(w0, (b - __mul24(a, v[e]) + (1 << 8)) >> 9);
                    }
                }
                if (r0 + q + 1 < r1) {
                    src2(r0 + q + 1, v);
#pragma unroll
                    for (int e = 0; e < 2; e++) {
                        const int a = cbd[e] * 6 + sbd[e] * 5;
                        const int b = cad[e] * 6 + sad[e] * 5;
                        acc[e][q + 1] += __mul24(w0, (b - __mul24(a, v[e]) + (1 << 7)) >> 8);
                    }
                }
#pragma unroll
                for (int e = 0; e < 2; e++) { cau[e] = cad[e]; sau[e] = sad[e]; cbu[e] = cbd[e]; sbu[e] = sbd[e]; }
            }
        }
        __syncthreads();
        KTL(3);
    }
    if (s1) {
        sgr_ab<1>(win, A, B, sh, tw, (unsigned)s1, bdm8, xbyx);
        __syncthreads();
        KTL(4);
        if (act) {
            int c0[2], t0[2], d0[2], u0[2], c1[2], t1[2], d1[2], u1[2], c2[2], t2[2], d2[2], u2[2];
            ld(r0 - 1, c0, t0, d0, u0);
            ld(r0, c1, t1, d1, u1);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                ld(r0 + q + 1, c2, t2, d2, u2);
                if (r0 + q < r1) {
                    int v[2];
                    src2(r0 + q, v);
#pragma unroll
                    for (int e = 0; e < 2; e++) {
                        const int a = (d1[e] + u1[e] + d0[e] + d2[e]) * 4 + (u0[e] + u2[e]) * 3;
                        const int b = (c1[e] + t1[e] + c0[e] + c2[e]) * 4 + (t0[e] + t2[e]) * 3;
                        acc[e][q] += __mul24(w1, (b - __mul24(a, v[e]) + (1 << 8)) >> 9);
                    }
                }
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    c0[e] = c1[e]; t0[e] = t1[e]; d0[e] = d1[e]; u0[e] = u1[e];
                    c1[e] = c2[e]; t1[e] = t2[e]; d1[e] = d2[e]; u1[e] = u2[e];
                }
            }
        }
    }
    __syncthreads();   // B (the A/B map) is free: it becomes the output tile
    if (act) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (r0 + q < r1) {
                int v[2];
                src2(r0 + q, v);
                const int o0 = min(max(v[0] + ((acc[0][q] + (1 << 10)) >> 11), 0), bdmax);
                const int o1 = min(max(v[1] + ((acc[1][q] + (1 << 10)) >> 11), 0), bdmax);
                *reinterpret_cast<uint32_t *>(B + (r0 + q) * 64 + x) = (uint32_t)(o0 & 0xffff) | ((uint32_t)o1 << 16);
            }
        }
    }
}

// Wiener vertical pass (looprestoration.rs:337-370) by column pairs: lane (rg, cp) filters
// columns 2cp, 2cp + 1 of rows 4rg .. 4rg + 3 from ten 32-bit reads of the horizontal output
// (one per row, both columns) and stores each output pair as one 32-bit word.
__device__ __forceinline__ void wiener_ver(const int16_t *hor, int16_t *B, int wr, int sh, int tw, const int (&fv)[7],
                                           int bd, int rbv, int bdmax) {
    const int cp = threadIdx.x & 31, rg = threadIdx.x >> 5, x = 2 * cp;
    const int r0 = rg * 4, r1 = min(r0 + 4, sh);
    if (x >= tw || r0 >= r1) return;
    const int off = 1 << (bd + rbv - 1);
    int h0[10], h1[10];
#pragma unroll
    for (int q = 0; q < 10; q++) {
        const uint32_t w = r0 + q < wr ? *reinterpret_cast<const uint32_t *>(hor + (r0 + q) * 64 + x) : 0u;
        h0[q] = (int)(w & 0xffffu);
        h1[q] = (int)(w >> 16);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (r0 + q < r1) {
            int s0 = -off, s1 = -off;
#pragma unroll
            for (int t = 0; t < 7; t++) { s0 += h0[q + t] * fv[t]; s1 += h1[q + t] * fv[t]; }
            const int o0 = min(max((s0 + (1 << (rbv - 1))) >> rbv, 0), bdmax);
            const int o1 = min(max((s1 + (1 << (rbv - 1))) >> rbv, 0), bdmax);
            *reinterpret_cast<uint32_t *>(B + (r0 + q) * 64 + x) = (uint32_t)(o0 & 0xffff) | ((uint32_t)o1 << 16);
        }
    }
}

// 8 pixels as int16 pairs in a uint4 (u16: one 16-B load; u8: one 8-B load widened)
__device__ __forceinline__ uint32_t pk2(int lo, int hi) { return (uint32_t)(lo & 0xffff) | ((uint32_t)hi << 16); }
template <typename Px>
__device__ __forceinline__ uint4 load8(const Px *p) {
    if constexpr (sizeof(Px) == 2) {
        return *reinterpret_cast<const uint4 *>(p);
    } else {
        const uint2 d = *reinterpret_cast<const uint2 *>(p);
        return make_uint4((d.x & 0xff) | ((d.x & 0xff00) << 8), ((d.x >> 16) & 0xff) | ((d.x >> 8) & 0xff0000),
                          (d.y & 0xff) | ((d.y & 0xff00) << 8), ((d.y >> 16) & 0xff) | ((d.y >> 8) & 0xff0000));
    }
}
template <typename Px>
__device__ __forceinline__ void store8(Px *p, const uint4 &u) {
    if constexpr (sizeof(Px) == 2) {
        *reinterpret_cast<uint4 *>(p) = u;
    } else {
        uint2 d;
        d.x = (u.x & 0xff) | ((u.x >> 8) & 0xff00) | ((u.y & 0xff) << 16) | ((u.y & 0xff0000) << 8);
        d.y = (u.z & 0xff) | ((u.z >> 8) & 0xff00) | ((u.w & 0xff) << 16) | ((u.w & 0xff0000) << 8);
        *reinterpret_cast<uint2 *>(p) = d;
    }
}
// byte offset of plane row y: rows < 2^24 and strides < 2^24 with a product below 4 GB (an 8K
// 16-bit plane is 70 MB), so one 24-bit multiply instead of a 64-bit one
__device__ __forceinline__ size_t row_off(int y, int64_t st) { return (size_t)__umul24((unsigned)y, (unsigned)st); }
// the finished sh x tw output tile (int16, row stride 64, in LDS) -> O with 8-pixel stores
template <typename Px>
__device__ __forceinline__ void store_tile(const int16_t *t, uint8_t *O, int64_t st, int S, int sh, int x0, int tw) {
    for (int i = threadIdx.x; i < sh * 8; i += kNT) {
        const int r = i >> 3, c = 8 * (i & 7);
        if (c >= tw) continue;
        Px *dp = reinterpret_cast<Px *>(O + row_off(S + r, st)) + x0 + c;
        if (c + 8 <= tw) store8<Px>(dp, *reinterpret_cast<const uint4 *>(t + r * 64 + c));
        else for (int j = 0; j < tw - c; j++) dp[j] = (Px)t[r * 64 + c + j];
    }
}

// Stripe (64 luma rows, offset 8 up; first stripe 56) -> plane rows.
__device__ __forceinline__ int stripe_start(int k, int ssv) { return k ? (64 * k - 8) >> ssv : 0; }

// Filter the staged window (sh + 6 rows, window column kWX = tile column 0) of one tile of at
// most 64 x 64 into the output tile B (int16, row stride 64): Wiener (looprestoration.rs:
// 299-370) or self-guided (:566-912). Shared by the frame kernel and the per-call entries;
// two functions so that each branch of the frame kernel keeps only its own parameters live.
__device__ __forceinline__ void lr_wiener_tile(const int (&fh)[7], const int (&fv)[7], int16_t *win, int16_t *B,
                                               int16_t *hor, int sh, int tw, int bd) {
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int r0 = ty * kNR, r1 = min(r0 + kNR, sh);
    const int wr = sh + 6, bdmax = (1 << bd) - 1;
    {
        const int rbh = bd == 12 ? 5 : 3, rbv = bd == 12 ? 9 : 11;
        const int clip_h = (1 << (bd + 1 + 7 - rbh)) - 1;
        wiener_hor(win, hor, wr, tw, fh, bd, rbh, clip_h);
        __syncthreads();
        wiener_ver(hor, B, wr, sh, tw, fv, bd, rbv, bdmax);
        __syncthreads();
    }
}
__device__ __forceinline__ void lr_sgr_tile(int s0, int s1, int w0, int w1, int16_t *win, int *A, int16_t *B, int sh,
                                            int tw, int bd, uint8_t *xbyx /* LDS [256] */) {
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int r0 = ty * kNR, r1 = min(r0 + kNR, sh);
    const int bdmax = (1 << bd) - 1;
    if (threadIdx.x < 256) xbyx[threadIdx.x] = (uint8_t)sgr_x_by_x(threadIdx.x);
    __syncthreads();
    const int bdm8 = bd - 8;
    sgr_pairs(A, B, win, sh, tw, bdm8, s0, s1, w0, w1, xbyx, bdmax);
    __syncthreads();
}

// amdgpu_waves_per_eu(8): 64 VGPRs, four 512-lane workgroups per CU (the LDS allows four)
template <typename Px>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(8))) void lr_kernel(LrArgs a) {
    __shared__ __attribute__((aligned(16))) int16_t win[70 * kLrWin];
    __shared__ __attribute__((aligned(16))) int A[66 * kLrAB];
    __shared__ __attribute__((aligned(16))) int16_t B[66 * kLrAB];
    int16_t *hor = reinterpret_cast<int16_t *>(A);    // Wiener: [70][64] aliases A

    KTL(0);
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    // (hardware round robin: XCD-local orders of the tiles cut LR's HBM reads from 70 to 28 MB
    // but ran 1.3-5.9 us slower)
    int blk = blockIdx.x;
    if (a.order) {
        // the caller's order (mi_lr_tile_order): longest tiles first
        blk = a.order[blk];
        if ((unsigned)blk >= (unsigned)a.blk_start[3]) return;
    }
    const int p = blk < a.blk_start[1] ? 0 : blk < a.blk_start[2] ? 1 : 2;
    const int lb = blk - a.blk_start[p];
    const int tiles = a.tiles_x[p];
    const int k = lb / tiles, ti = lb - k * tiles;
    const int ssv = p ? a.ss_ver : 0, ssh = p ? a.ss_hor : 0;
    const int pw = a.pw[p], ph = a.ph[p];
    const int x0 = ti * a.tw[p];
    const int tw = min(a.tw[p], pw - x0);
    const int S = stripe_start(k, ssv);
    const int E = min(stripe_start(k + 1, ssv), ph);
    const int sh = E - S;
    const uint8_t *C = a.src[p];
    const uint8_t *D = a.lpf[p];
    uint8_t *O = a.dst[p];
    const int64_t st = a.stride[p];
    // lane (tx, ty) owns output column tx, rows [ty*kNR, ty*kNR+kNR)
    const int r0 = ty * kNR, r1 = min(r0 + kNR, sh);

    // restoration unit of this tile (lr_apply.rs:151-259 indexing)
    int type = 0;
    const MiAv1RestorationUnit *u = nullptr;
    if (a.restore & (1 << p)) {
        const int us = 1 << a.unit_log2[p ? 1 : 0];
        const int nu = max(1, (pw + (us >> 1)) / us);
        const int uc = min(x0 / us, nu - 1);
        const int xu = uc * us;
        int ay = ((64 * k) >> ssv) & ~(us - 1);
        if (ay && ay + (us >> 1) > ph) ay -= us;
        ay <<= ssv;
        const int sbi = (ay >> 7) * a.sb128w + (xu >> (7 - ssh));
        const int ui = (((ay >> 6) & 1) << 1) + ((xu >> (6 - ssh)) & 1);
        u = &a.lr_mask[sbi].lr[p][ui];
        type = u->type;
    }
    if (type == 0) {   // RESTORATION_NONE: O = C, 8-pixel vectors
        for (int i = threadIdx.x; i < sh * 8; i += kNT) {
            const int r = i >> 3, x = x0 + 8 * (i & 7);
            if (x >= x0 + tw) continue;
            const Px *sp = reinterpret_cast<const Px *>(C + row_off(S + r, st)) + x;
            Px *dp = reinterpret_cast<Px *>(O + row_off(S + r, st)) + x;
            if (x + 8 <= x0 + tw) store8<Px>(dp, load8<Px>(sp));   // O = C
            else for (int j = 0; j < x0 + tw - x; j++) dp[j] = sp[j];
        }
        KTLV(6, 0);
        KTL(5);
        return;
    }
    KTLV(6, type);

    // ---- stage the (sh+6)-row window, columns x0-8 .. x0+71 (C inside the stripe, D across
    // its edges) as 8-pixel vectors; columns outside the plane replicate the edge pixel ----
    const bool have_top = k > 0, have_bottom = E < ph;
    const int wr = sh + 6;
    constexpr int kNV = kLrWin / 8;                   // vectors per window row
    constexpr int kSV = (70 * kNV + kNT - 1) / kNT;   // vectors per lane
    uint4 sv[kSV];
#pragma unroll
    for (int q = 0; q < kSV; q++) {
        sv[q] = make_uint4(0, 0, 0, 0);
        const int i = threadIdx.x + q * kNT;
        const int rr = i / kNV, x = x0 - 8 + 8 * (i % kNV), r = rr - 3;
        if (rr < wr) {
            int yy;
            const uint8_t *src;
            if (r >= 0 && r < sh) { src = C; yy = S + r; }
            else if (r < 0) { src = have_top ? D : C; yy = have_top ? S - 2 + (r == -1) : S; }
            else { src = have_bottom ? D : C; yy = have_bottom ? min(E + (r > sh), ph - 1) : E - 1; }
            const Px *row = reinterpret_cast<const Px *>(src + row_off(yy, st));
            if (x >= 0 && x + 8 <= pw) sv[q] = load8<Px>(row + x);
            else {
                int e[8];
#pragma unroll
                for (int j = 0; j < 8; j++) e[j] = row[min(max(x + j, 0), pw - 1)];
                sv[q] = make_uint4(pk2(e[0], e[1]), pk2(e[2], e[3]), pk2(e[4], e[5]), pk2(e[6], e[7]));
            }
        }
    }
#pragma unroll
    for (int q = 0; q < kSV; q++) {
        const int i = threadIdx.x + q * kNT;
        const int rr = i / kNV;
        if (rr < wr) *reinterpret_cast<uint4 *>(&win[rr * kLrWin + 8 * (i % kNV)]) = sv[q];
    }
    __syncthreads();
    KTL(1);

    // (the tile filter is written out here rather than through lr_wiener_tile / lr_sgr_tile:
    //  that form measured 70.5 vs 63 us at 4K10 with the same registers and LDS size, most
    //  likely because its function-scope __shared__ table, used by two kernels, is reached
    //  through the per-kernel LDS lookup that LLVM emits for such variables)
    const int bd = a.bd, bdmax = (1 << bd) - 1;
    if (type == 2) {
        // ---- Wiener (looprestoration.rs:299-370) ----
        int fh[7], fv[7];
        fh[0] = fh[6] = u->filter_h[0]; fh[1] = fh[5] = u->filter_h[1]; fh[2] = fh[4] = u->filter_h[2];
        fh[3] = 128 - 2 * (fh[0] + fh[1] + fh[2]);
        fv[0] = fv[6] = u->filter_v[0]; fv[1] = fv[5] = u->filter_v[1]; fv[2] = fv[4] = u->filter_v[2];
        fv[3] = 128 - 2 * (fv[0] + fv[1] + fv[2]);
        const int rbh = bd == 12 ? 5 : 3, rbv = bd == 12 ? 9 : 11;
        const int clip_h = (1 << (bd + 1 + 7 - rbh)) - 1;
        wiener_hor(win, hor, wr, tw, fh, bd, rbh, clip_h);
        __syncthreads();
        KTL(2);
        wiener_ver(hor, B, wr, sh, tw, fv, bd, rbv, bdmax);
        __syncthreads();
        KTL(3);
        store_tile<Px>(B, O, st, S, sh, x0, tw);
        KTL(5);
        return;
    }

    // ---- self-guided (looprestoration.rs:566-912) ----
    __shared__ uint8_t xbyx[256];
    if (threadIdx.x < 256) xbyx[threadIdx.x] = (uint8_t)sgr_x_by_x(threadIdx.x);
    __syncthreads();
    const int sidx = type - 3;
    const int s0 = k_sgr_params[sidx][0], s1 = k_sgr_params[sidx][1];
    const int w0 = u->sgr_weights[0];
    const int w1 = 128 - (u->sgr_weights[0] + u->sgr_weights[1]);
    const int bdm8 = bd - 8;
    sgr_pairs(A, B, win, sh, tw, bdm8, s0, s1, w0, w1, xbyx, bdmax);
    __syncthreads();
    store_tile<Px>(B, O, st, S, sh, x0, tw);
    KTL(5);
}

// ---- per-call lr.wiener / lr.sgr (looprestoration.rs:91-107, 139-912) ----
// One 512-lane workgroup per 64-column tile of the unit (w <= 384, h <= 64). The window is
// the reference's `padding` (looprestoration.rs:139-268) built in LDS from the staged inputs:
// the unit's pixels (with 3 columns either side where HAVE_LEFT / HAVE_RIGHT), left[h][4],
// and the lpf rows 0, 1 (above) and 6, 7 (below); missing sides replicate.
template <typename Px>
__global__ __launch_bounds__(kNT) void lr_call_kernel(LrCallArgs a) {
    __shared__ __attribute__((aligned(16))) int16_t win[70 * kLrWin];
    __shared__ __attribute__((aligned(16))) int A[66 * kLrAB];
    __shared__ __attribute__((aligned(16))) int16_t B[66 * kLrAB];
    int16_t *hor = reinterpret_cast<int16_t *>(A);
    const int x0 = blockIdx.x * 64, tw = min(64, a.w - x0), h = a.h;
    const bool hl = a.edges & 1, hr = a.edges & 2, ht = a.edges & 4, hb = a.edges & 8;
    const Px *p = reinterpret_cast<const Px *>(a.p), *lpf = reinterpret_cast<const Px *>(a.lpf);
    const Px *left = reinterpret_cast<const Px *>(a.left);
    for (int i = threadIdx.x; i < (h + 6) * kLrWin; i += kNT) {
        const int rr = i / kLrWin, c = i % kLrWin;
        int x = x0 - kWX + c;
        int v = 0;
        if (x >= -3 && x < a.w + 3) {
            if (!hr && x >= a.w) x = a.w - 1;
            if (!hl && x < 0) x = 0;
            const int j = rr - 3;
            if (rr < 3 && ht) v = lpf[(rr < 2 ? 0 : 1) * a.ps + x];
            else if (j >= h && hb) v = lpf[(j == h ? 6 : 7) * a.ps + x];
            else {
                const int jj = min(max(j, 0), h - 1);   // rows above / below replicate when absent
                v = x < 0 ? left[jj * 4 + 1 + (x + 3)] : p[jj * a.ps + x];
            }
        }
        win[i] = (int16_t)v;
    }
    __syncthreads();
    if (a.tp.wiener) lr_wiener_tile(a.tp.fh, a.tp.fv, win, B, hor, h, tw, a.bd);
    else {
        __shared__ uint8_t xbyx[256];
        lr_sgr_tile(a.tp.s0, a.tp.s1, a.tp.w0, a.tp.w1, win, A, B, h, tw, a.bd, xbyx);
    }
    // output tile -> the packed w x h result
    for (int i = threadIdx.x; i < h * 64; i += kNT) {
        const int r = i >> 6, c = i & 63;
        if (c < tw) reinterpret_cast<Px *>(a.out)[r * a.w + x0 + c] = (Px)B[r * 64 + c];
    }
}

int launch_lr_call(const LrCallArgs &a, int bpc, hipStream_t s) {
    const int n = (a.w + 63) / 64;
    if (bpc == 8) hipLaunchKernelGGL(lr_call_kernel<uint8_t>, dim3(n), dim3(kNT), 0, s, a);
    else hipLaunchKernelGGL(lr_call_kernel<uint16_t>, dim3(n), dim3(kNT), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_lr(const LrArgs &a, int bpc, hipStream_t s) {
    const int n = a.blk_start[3];
    if (n <= 0) return 0;
    if (bpc == 8) hipLaunchKernelGGL(lr_kernel<uint8_t>, dim3(n), dim3(kNT), 0, s, a);
    else hipLaunchKernelGGL(lr_kernel<uint16_t>, dim3(n), dim3(kNT), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
