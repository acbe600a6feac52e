// cdef.hip — whole-frame CDEF on gfx950, out of place (deblocked D -> C).
//
// Replaces rav1d_cdef_brow (rav1d src/cdef_apply.rs:159-507) and the DSP cdef.dir/cdef.fb[3]
// (src/cdef.rs:545-1031; C src/cdef_tmpl.c). The reference filters in place and keeps line and
// column backups so every block reads deblocked (pre-CDEF) samples only; reading an immutable
// D and writing C gives the same result without backups.
//
// One 256-lane workgroup per 64x64 luma unit (the granularity of cdef_idx, so strengths are
// workgroup-uniform) plus its co-located chroma. The tile and a 2-px halo are staged in LDS as
// int16 with i16::MIN where the reference's padding marks samples unavailable (frame edges,
// cdef.rs:567-665). Phase 1: 64 lanes find the 8x8 directions; phase 2: every lane filters
// pixels straight out of LDS and streams C back with coalesced stores.
#include "common.h"

MI_KTL_DEFINE(cdef)

namespace mi {


// Tap offsets (dy, dx) per direction and distance (dav1d_cdef_directions, src/tables.rs:698),
// packed as 4-bit (value + 2) nibbles indexed by direction so that a per-lane direction
// selects its offsets with shifts instead of a divergent table load.
//   dir:        0   1   2   3   4   5   6   7
//   k=0 dy:    -1   0   0   0   1   1   1   1      dx: 1 1 1 1 1 0 0 0
//   k=1 dy:    -2  -1   0   1   2   2   2   2      dx: 2 2 2 2 2 1 0 -1
__device__ __forceinline__ int nib(unsigned packed, int dir) { return (int)((packed >> (4 * dir)) & 15) - 2; }
__device__ __forceinline__ int dir_off(int dir, int k, int ts) {
    constexpr unsigned DY0 = 0x33332221u, DX0 = 0x22233333u, DY1 = 0x44443210u, DX1 = 0x12344444u;
    return k == 0 ? nib(DY0, dir) * ts + nib(DX0, dir) : nib(DY1, dir) * ts + nib(DX1, dir);
}

// Luma tile: 68 rows (2-row halo) x 88 int16 (frame columns x0-8 .. x0+79; interior at column 8).
// 88 = 44 dwords per row: a 32-lane group's 8 rows x 4 dwords fall on 32 distinct banks, and
// every 8-px block row is 16-B aligned for ds_read_b128.
constexpr int kTY = 68, kTS = 88;

__device__ __forceinline__ int constrain(int diff, int thr, int shift) {
    const int ad = abs(diff);
    const int v = min(ad, max(0, thr - (ad >> shift)));
    return diff < 0 ? -v : v;
}

__device__ __forceinline__ int ulog2i(unsigned v) { return 31 - __clz(v); }

__device__ __forceinline__ int adjust_strength(int strength, unsigned var) {
    if (!var) return 0;
    const int i = (var >> 6) ? min(ulog2i(var >> 6), 12) : 0;
    return (strength * (4 + i) + 8) >> 4;
}

// 8x8 direction search on an LDS tile (cdef.rs:921-1031).
__device__ int find_dir(const int16_t *t, int ts, int bdm8, unsigned *var) {
    int hv0[8] = {}, hv1[8] = {}, dg0[15] = {}, dg1[15] = {}, al[4][11] = {};
#pragma unroll
    for (int y = 0; y < 8; y++) {
#pragma unroll
        for (int x = 0; x < 8; x++) {
            const int p = ((int)t[y * ts + x] >> bdm8) - 128;
            dg0[y + x] += p;
            al[0][y + (x >> 1)] += p;
            hv0[y] += p;
            al[1][3 + y - (x >> 1)] += p;
            dg1[7 + y - x] += p;
            al[2][3 - (y >> 1) + x] += p;
            hv1[x] += p;
            al[3][(y >> 1) + x] += p;
        }
    }
    const unsigned dv[7] = { 840, 420, 280, 210, 168, 140, 120 };
    unsigned cost[8] = {};
#pragma unroll
    for (int n = 0; n < 8; n++) {
        cost[2] += (unsigned)(hv0[n] * hv0[n]);
        cost[6] += (unsigned)(hv1[n] * hv1[n]);
    }
    cost[2] *= 105;
    cost[6] *= 105;
#pragma unroll
    for (int n = 0; n < 7; n++) {
        cost[0] += (unsigned)(dg0[n] * dg0[n] + dg0[14 - n] * dg0[14 - n]) * dv[n];
        cost[4] += (unsigned)(dg1[n] * dg1[n] + dg1[14 - n] * dg1[14 - n]) * dv[n];
    }
    cost[0] += (unsigned)(dg0[7] * dg0[7]) * 105;
    cost[4] += (unsigned)(dg1[7] * dg1[7]) * 105;
#pragma unroll
    for (int n = 0; n < 4; n++) {
        unsigned c = 0;
#pragma unroll
        for (int m = 0; m < 5; m++) c += (unsigned)(al[n][3 + m] * al[n][3 + m]);
        c *= 105;
#pragma unroll
        for (int m = 0; m < 3; m++)
            c += (unsigned)(al[n][m] * al[n][m] + al[n][10 - m] * al[n][10 - m]) * dv[2 * m + 1];
        cost[2 * n + 1] = c;
    }
    int best = 0;
    unsigned bc = cost[0];
#pragma unroll
    for (int n = 1; n < 8; n++)
        if (cost[n] > bc) { bc = cost[n]; best = n; }
    *var = (bc - cost[best ^ 4]) >> 10;
    return best;
}

// find_dir split by direction pair over the workgroup's four waves (cdef.rs:921-1031): wave
// PAIR takes directions 2 PAIR and 2 PAIR + 1 of the 64 blocks (lane = block), so each lane
// keeps two partial-sum arrays instead of eight and all four waves share the search.
template <int PAIR>
__device__ __forceinline__ void dir_costs(const int16_t *t, int ts, int bdm8, unsigned &ca, unsigned &cb) {
    constexpr int NA = PAIR == 1 || PAIR == 3 ? 8 : 15;
    int a[NA] = {}, b[11] = {};
#pragma unroll
    for (int y = 0; y < 8; y++) {
#pragma unroll
        for (int x = 0; x < 8; x += 2) {
            const uint32_t pr = *reinterpret_cast<const uint32_t *>(t + y * ts + x);
            const int p0 = ((int)(int16_t)(pr & 0xffffu) >> bdm8) - 128, p1 = ((int)(int16_t)(pr >> 16) >> bdm8) - 128;
            const int pp[2] = { p0, p1 };
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int xx = x + e, p = pp[e];
                if (PAIR == 0) { a[y + xx] += p; b[y + (xx >> 1)] += p; }
                if (PAIR == 1) { a[y] += p; b[3 + y - (xx >> 1)] += p; }
                if (PAIR == 2) { a[7 + y - xx] += p; b[3 - (y >> 1) + xx] += p; }
                if (PAIR == 3) { a[xx] += p; b[(y >> 1) + xx] += p; }
            }
        }
    }
    const unsigned dv[7] = { 840, 420, 280, 210, 168, 140, 120 };
    unsigned c = 0;
    if (NA == 8) {
#pragma unroll
        for (int n = 0; n < 8; n++) c += (unsigned)(a[n] * a[n]);
        c *= 105;
    } else {
#pragma unroll
        for (int n = 0; n < 7; n++) c += (unsigned)(a[n] * a[n] + a[14 - n] * a[14 - n]) * dv[n];
        c += (unsigned)(a[7] * a[7]) * 105;
    }
    ca = c;
    c = 0;
#pragma unroll
    for (int m = 0; m < 5; m++) c += (unsigned)(b[3 + m] * b[3 + m]);
    c *= 105;
#pragma unroll
    for (int m = 0; m < 3; m++) c += (unsigned)(b[m] * b[m] + b[10 - m] * b[10 - m]) * dv[2 * m + 1];
    cb = c;
}

// find_dir's cost of one direction D for the 8x8 block at t (cdef.rs:921-1031): the partial
// sums of that direction only (index didx<D>), the pixel bias of -128 folded into their start
// values. One wave per direction, lane = block.
template <int D> __device__ __host__ constexpr int didx(int y, int x) {
    return D == 0 ? y + x : D == 1 ? y + (x >> 1) : D == 2 ? y : D == 3 ? 3 + y - (x >> 1)
         : D == 4 ? 7 + y - x : D == 5 ? 3 - (y >> 1) + x : D == 6 ? x : (y >> 1) + x;
}
template <int D> __device__ __host__ constexpr int dcount(int k) {
    int n = 0;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) n += didx<D>(y, x) == k;
    return n;
}
template <int D>
__device__ __forceinline__ unsigned dir_cost1(const int16_t *t, int ts, int bdm8) {
    constexpr int NA = D == 2 || D == 6 ? 8 : (D & 1) ? 11 : 15;
    int a[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) a[k] = -128 * dcount<D>(k);
#pragma unroll
    for (int y = 0; y < 8; y++) {
        const uint4 v = *reinterpret_cast<const uint4 *>(t + y * ts);   // one 8-px row, ds_read_b128
        const uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll
        for (int x = 0; x < 8; x += 2) {
            a[didx<D>(y, x)] += (int)(int16_t)(w[x >> 1] & 0xffffu) >> bdm8;
            a[didx<D>(y, x + 1)] += (int)(int16_t)(w[x >> 1] >> 16) >> bdm8;
        }
    }
    const unsigned dv[7] = { 840, 420, 280, 210, 168, 140, 120 };
    unsigned c = 0;
    if constexpr (NA == 8) {
#pragma unroll
        for (int n = 0; n < 8; n++) c += (unsigned)(a[n] * a[n]);
        c *= 105;
    } else if constexpr (NA == 15) {
#pragma unroll
        for (int n = 0; n < 7; n++) c += (unsigned)(a[n] * a[n] + a[14 - n] * a[14 - n]) * dv[n];
        c += (unsigned)(a[7] * a[7]) * 105;
    } else {
#pragma unroll
        for (int m = 0; m < 5; m++) c += (unsigned)(a[3 + m] * a[3 + m]);
        c *= 105;
#pragma unroll
        for (int m = 0; m < 3; m++) c += (unsigned)(a[m] * a[m] + a[10 - m] * a[10 - m]) * dv[2 * m + 1];
    }
    return c;
}

// Filter one pixel at LDS position (x, y); c = centre sample. Returns the new value.
__device__ __forceinline__ int cdef_px(const int16_t *t, int ts, int x, int y, int pri, int sec,
                                       int dir, int damping, int bdm8) {
    const int c = t[y * ts + x];
    int sum = 0, mx = c;
    unsigned mn = (unsigned)c & 0xffff;   // i16 sentinel compares as unsigned 0x8000+ (large)
    if (pri) {
        const int shift = max(0, damping - ulog2i(pri));
        int tap = 4 - ((pri >> bdm8) & 1);
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int o = dir_off(dir, k, ts);
            const int a = t[y * ts + x + o], b = t[y * ts + x - o];
            sum += tap * (constrain(a - c, pri, shift) + constrain(b - c, pri, shift));
            tap = (tap & 3) | 2;
            mn = min(mn, (unsigned)a & 0xffff); mx = max(mx, a);
            mn = min(mn, (unsigned)b & 0xffff); mx = max(mx, b);
        }
    }
    if (sec) {
        const int shift = damping - ulog2i(sec);
        const int d2 = (dir + 2) & 7, d6 = (dir + 6) & 7;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int o2 = dir_off(d2, k, ts);
            const int o3 = dir_off(d6, k, ts);
            const int s0 = t[y * ts + x + o2], s1 = t[y * ts + x - o2];
            const int s2 = t[y * ts + x + o3], s3 = t[y * ts + x - o3];
            sum += (2 - k) * (constrain(s0 - c, sec, shift) + constrain(s1 - c, sec, shift) +
                              constrain(s2 - c, sec, shift) + constrain(s3 - c, sec, shift));
            mn = min(mn, (unsigned)s0 & 0xffff); mx = max(mx, s0);
            mn = min(mn, (unsigned)s1 & 0xffff); mx = max(mx, s1);
            mn = min(mn, (unsigned)s2 & 0xffff); mx = max(mx, s2);
            mn = min(mn, (unsigned)s3 & 0xffff); mx = max(mx, s3);
        }
    }
    int v = c + ((sum - (sum < 0) + 8) >> 4);
    if (pri && sec) v = min(max(v, (int)mn), mx);
    return v;
}

// Tile loader: the (ROWS x COLS) window at (x0-2, y0-2) as int16, i16::MIN outside the frame,
// written twice: T[r][c] and T1[r][c-1] (T shifted left by one sample), so that any horizontal
// sample pair (c, c+1) is one aligned 32-bit LDS word in T (c even) or T1 (c odd). Each row of
// the window is read as 8-sample aligned vectors from
// x0 - 8 (one 16-B load at 16 bits, 8-B at 8 bits; per-sample checks only for a vector that
// straddles the frame edge) and written to T as 4 aligned pairs and to T1 (shifted by one) as
// 3 pairs plus the two end samples: 10 vectors per luma row instead of 68 scalar loads.
template <typename Px, int ROWS, int COLS, int NTH>
struct VecTileLoad {
    static constexpr int NV = (COLS + 6 + 7) / 8, N = ROWS * NV, IT = (N + NTH - 1) / NTH;
    uint32_t w[IT][4];
    __device__ __forceinline__ void fetch(const uint8_t *src, int64_t stride, int x0, int y0, int fw, int fh) {
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const int i = threadIdx.x + NTH * k;
            const int r = i / NV, j = i - r * NV;
            const int y = y0 - 2 + r, xs = x0 - 8 + 8 * j;
#pragma unroll
            for (int q = 0; q < 4; q++) w[k][q] = 0x80008000u;
            if (i < N && y >= 0 && y < fh) {
                const Px *row = reinterpret_cast<const Px *>(src + (int64_t)y * stride);
                if (xs >= 0 && xs + 8 <= fw) {
                    if constexpr (sizeof(Px) == 2) {
                        const uint4 v = *reinterpret_cast<const uint4 *>(row + xs);
                        w[k][0] = v.x; w[k][1] = v.y; w[k][2] = v.z; w[k][3] = v.w;
                    } else {
                        const uint2 v = *reinterpret_cast<const uint2 *>(row + xs);
                        w[k][0] = (v.x & 0xffu) | ((v.x & 0xff00u) << 8);
                        w[k][1] = ((v.x >> 16) & 0xffu) | ((v.x >> 8) & 0xff0000u);
                        w[k][2] = (v.y & 0xffu) | ((v.y & 0xff00u) << 8);
                        w[k][3] = ((v.y >> 16) & 0xffu) | ((v.y >> 8) & 0xff0000u);
                    }
                } else if (xs + 8 > 0 && xs < fw) {
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const int x = xs + e;
                        const uint32_t v = x >= 0 && x < fw ? (uint32_t)row[x] : 0x8000u;
                        w[k][e >> 1] = (w[k][e >> 1] & (e & 1 ? 0xffffu : 0xffff0000u)) | (v << (16 * (e & 1)));
                    }
                }
            }
        }
    }
    // T column c holds frame column x0 - 8 + c, so vector j lands 16-B aligned at column 8j
    // (one ds_write_b128) and the tile interior starts at column 8. T1[c] = T[c + 1]: samples
    // (1,2) (3,4) (5,6) as one 12-B store at column 8j, samples 0 and 7 alone.
    __device__ __forceinline__ void store(int16_t *t, int16_t *t1, int ts) const {
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const int i = threadIdx.x + NTH * k;
            if (i >= N) continue;
            const int r = i / NV, j = i - r * NV;
            int16_t *tr = t + r * ts + 8 * j, *t1r = t1 + r * ts + 8 * j;
            *reinterpret_cast<uint4 *>(tr) = make_uint4(w[k][0], w[k][1], w[k][2], w[k][3]);
            *reinterpret_cast<uint3 *>(t1r) = make_uint3((w[k][0] >> 16) | (w[k][1] << 16),
                                                         (w[k][1] >> 16) | (w[k][2] << 16),
                                                         (w[k][2] >> 16) | (w[k][3] << 16));
            if (j) t1r[-1] = (int16_t)(w[k][0] & 0xffffu);
            t1r[6] = (int16_t)(w[k][3] >> 16);
        }
    }
};

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// constrain() (cdef.rs:545) on two samples at once. d = sat(p - c): a sentinel tap gives
// d = -32768 and |d| = 32767 (saturated), so its contribution is 0 exactly as in 32-bit.
__device__ __forceinline__ s16x2 constrain2(s16x2 d, u16x2 thr, u16x2 shift) {
    const s16x2 zero = { 0, 0 };
    const s16x2 ad = __builtin_elementwise_max(d, __builtin_elementwise_sub_sat(zero, d));
    // max(0, thr - (|d| >> shift)) as one unsigned saturating subtract
    const s16x2 m = __builtin_bit_cast(s16x2, __builtin_elementwise_sub_sat(thr, __builtin_bit_cast(u16x2, ad) >> shift));
    return __builtin_elementwise_max(__builtin_elementwise_min(d, m), zero - m);
}

// byte offset of tap (dy, dx) from a pair's base in T: pairs at odd dx come from T1
template <int TS, int T1OFF>
__device__ __forceinline__ int tap_delta(int dy, int dx) {
    return dy * TS * 2 + (dx - (dx & 1)) * 2 + (dx & 1) * T1OFF;
}

struct PairTaps {
    int pri[4], sec[8];      // byte deltas: pri (k0+, k0-, k1+, k1-), sec (d2 k0 +-, d6 k0 +-, d2 k1 +-, d6 k1 +-)
};

template <int TS, int T1OFF>
__device__ __forceinline__ void make_taps(PairTaps &t, int dir) {
    constexpr unsigned DY0 = 0x33332221u, DX0 = 0x22233333u, DY1 = 0x44443210u, DX1 = 0x12344444u;
    const int d2 = (dir + 2) & 7, d6 = (dir + 6) & 7;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const unsigned DY = k ? DY1 : DY0, DX = k ? DX1 : DX0;
        const int py = nib(DY, dir), px = nib(DX, dir);
        t.pri[2 * k] = tap_delta<TS, T1OFF>(py, px);
        t.pri[2 * k + 1] = tap_delta<TS, T1OFF>(-py, -px);
        const int ay = nib(DY, d2), ax = nib(DX, d2), by = nib(DY, d6), bx = nib(DX, d6);
        t.sec[4 * k] = tap_delta<TS, T1OFF>(ay, ax);
        t.sec[4 * k + 1] = tap_delta<TS, T1OFF>(-ay, -ax);
        t.sec[4 * k + 2] = tap_delta<TS, T1OFF>(by, bx);
        t.sec[4 * k + 3] = tap_delta<TS, T1OFF>(-by, -bx);
    }
}

__device__ __forceinline__ s16x2 ld2(const char *p) { return *reinterpret_cast<const s16x2 *>(p); }

// cdef_filter_block_c inner loop (cdef.rs:668-790) for the pixel pair whose base is P.
__device__ __forceinline__ s16x2 cdef_pair(const char *P, const PairTaps &t, int pri, int sec,
                                           int damping, int bdm8) {
    const s16x2 c = ld2(P);
    s16x2 sum = { 0, 0 }, mx = c;
    u16x2 mn = __builtin_bit_cast(u16x2, c);
    if (pri) {
        const unsigned short sh = (unsigned short)max(0, damping - ulog2i(pri));
        const u16x2 thr = { (unsigned short)pri, (unsigned short)pri }, shv = { sh, sh };
        const short tap0 = (short)(4 - ((pri >> bdm8) & 1)), tap1 = (short)((tap0 & 3) | 2);
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const s16x2 a = ld2(P + t.pri[2 * k]), b = ld2(P + t.pri[2 * k + 1]);
            const s16x2 v = constrain2(__builtin_elementwise_sub_sat(a, c), thr, shv) +
                            constrain2(__builtin_elementwise_sub_sat(b, c), thr, shv);
            const short tp = k ? tap1 : tap0;
            const s16x2 tpv = { tp, tp };
            sum += tpv * v;
            mn = __builtin_elementwise_min(mn, __builtin_bit_cast(u16x2, a));
            mn = __builtin_elementwise_min(mn, __builtin_bit_cast(u16x2, b));
            mx = __builtin_elementwise_max(mx, a);
            mx = __builtin_elementwise_max(mx, b);
        }
    }
    if (sec) {
        const unsigned short sh = (unsigned short)(damping - ulog2i(sec));
        const u16x2 thr = { (unsigned short)sec, (unsigned short)sec }, shv = { sh, sh };
#pragma unroll
        for (int k = 0; k < 2; k++) {
            s16x2 v = { 0, 0 };
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const s16x2 a = ld2(P + t.sec[4 * k + j]);
                v += constrain2(__builtin_elementwise_sub_sat(a, c), thr, shv);
                mn = __builtin_elementwise_min(mn, __builtin_bit_cast(u16x2, a));
                mx = __builtin_elementwise_max(mx, a);
            }
            sum += k ? v : v + v;
        }
    }
    const s16x2 one5 = { 15, 15 }, eight = { 8, 8 }, four = { 4, 4 };
    s16x2 v = c + ((sum + (sum >> one5) + eight) >> four);
    if (pri && sec) v = __builtin_elementwise_min(__builtin_elementwise_max(v, __builtin_bit_cast(s16x2, mn)), mx);
    return v;
}

template <typename Px> __device__ __forceinline__ void store_pair(Px *d, s16x2 v);
template <> __device__ __forceinline__ void store_pair<uint16_t>(uint16_t *d, s16x2 v) {
    *reinterpret_cast<s16x2 *>(d) = v;
}
template <> __device__ __forceinline__ void store_pair<uint8_t>(uint8_t *d, s16x2 v) {
    *reinterpret_cast<uint16_t *>(d) = (uint16_t)((v.x & 0xff) | (v.y << 8));
}
template <typename Px> __device__ __forceinline__ void copy_pair(Px *d, const Px *s);
template <> __device__ __forceinline__ void copy_pair<uint16_t>(uint16_t *d, const uint16_t *s) {
    *reinterpret_cast<uint32_t *>(d) = *reinterpret_cast<const uint32_t *>(s);
}
template <> __device__ __forceinline__ void copy_pair<uint8_t>(uint8_t *d, const uint8_t *s) {
    *reinterpret_cast<uint16_t *>(d) = *reinterpret_cast<const uint16_t *>(s);
}

// Filter (or copy) one plane of the unit as pixel pairs. W x H plane pixels, BW x BH pixels per
// direction block; LP lanes (lane index `lane`) each own one pair column and NR consecutive rows.
template <typename Px, int W, int H, int BW, int BH, int LP, int TS, int T1OFF, int MASK, bool TILE_COPY>
__device__ __forceinline__ void filter_plane(const int16_t *T, int lane, const int8_t *bdir,
                                             const int8_t *bflag, const int16_t *bpri, bool adj_pri,
                                             int pri_lvl, int sec, int damping, int bdm8, bool remap422,
                                             const uint8_t *src, uint8_t *dst, int64_t stride,
                                             int gx0, int gy0, int fw, int fh) {
    constexpr int PW = W / 2, NR = H * PW / LP, RB = NR < BH ? NR : BH;
    const int pc = lane % PW, rg = lane / PW, x = 2 * pc;
#pragma unroll
    for (int bb = 0; bb < NR / RB; bb++) {
        const int r0 = rg * NR + bb * RB;
        const int b = (r0 / BH) * 8 + x / BW;
        const int flag = bflag[b];
        const int gx = gx0 + x;
        if (flag & MASK) {
            const int pri = adj_pri ? bpri[b] : pri_lvl;
            int dir = pri_lvl ? bdir[b] : 0;
            if (remap422 && pri_lvl) dir = nib(0x66654207u, dir) + 2;   // {7,0,2,4,5,6,6,6}
            PairTaps t;
            make_taps<TS, T1OFF>(t, dir);
#pragma unroll
            for (int i = 0; i < RB; i++) {
                const int r = r0 + i;
                const char *P = reinterpret_cast<const char *>(T + (r + 2) * TS + x + 8);
                const s16x2 v = cdef_pair(P, t, pri, sec, damping, bdm8);
                store_pair<Px>(reinterpret_cast<Px *>(dst + (int64_t)(gy0 + r) * stride) + gx, v);
            }
        } else {
#pragma unroll
            for (int i = 0; i < RB; i++) {
                const int r = r0 + i, gy = gy0 + r;
                Px *dp = reinterpret_cast<Px *>(dst + (int64_t)gy * stride) + gx;
                if (TILE_COPY && gx < fw && gy < fh) store_pair<Px>(dp, ld2(reinterpret_cast<const char *>(T + (r + 2) * TS + x + 8)));
                else copy_pair<Px>(dp, reinterpret_cast<const Px *>(src + (int64_t)gy * stride) + gx);
            }
        }
    }
}

// 4:2:0 chroma of one unit (32x32 per plane, 64 4x4 blocks): lanes 0..255 U, 256..511 V. A
// 32-lane group takes four horizontally adjacent blocks at a time (lane: block l / 8, row
// (l % 8) / 2, pair column l % 2), so a tap read of the group touches four directions instead of
// the eight of a row-major mapping (half the bank conflicts), and the direction's tap deltas
// are three broadcast-per-block LDS reads (table built once per unit) instead of a per-lane
// decode of the direction nibbles.
template <typename Px, int TS>
__device__ __forceinline__ void filter_chroma420(const int16_t *T, const int4 (*taps)[3], const int8_t *bdir,
                                                 const int8_t *bflag, int pri, int sec, int damping, int bdm8,
                                                 const uint8_t *src, uint8_t *dst, int64_t stride, int gx0, int gy0) {
    const int ln = threadIdx.x & 255, gq = ln >> 5, l = ln & 31;
    const int j = l >> 3, rr = (l & 7) >> 1, e = l & 1;
#pragma unroll
    for (int it = 0; it < 2; it++) {
        const int b = it * 32 + gq * 4 + j, by = b >> 3, bx = b & 7;
        const int r = by * 4 + rr, x = bx * 4 + 2 * e;
        Px *dp = reinterpret_cast<Px *>(dst + (int64_t)(gy0 + r) * stride) + gx0 + x;
        if (bflag[b] & 2) {
            const int dir = pri ? bdir[b] : 0;
            PairTaps t;
            const int4 q0 = taps[dir][0], q1 = taps[dir][1], q2 = taps[dir][2];
            t.pri[0] = q0.x; t.pri[1] = q0.y; t.pri[2] = q0.z; t.pri[3] = q0.w;
            t.sec[0] = q1.x; t.sec[1] = q1.y; t.sec[2] = q1.z; t.sec[3] = q1.w;
            t.sec[4] = q2.x; t.sec[5] = q2.y; t.sec[6] = q2.z; t.sec[7] = q2.w;
            const char *P = reinterpret_cast<const char *>(T + (r + 2) * TS + x + 8);
            store_pair<Px>(dp, cdef_pair(P, t, pri, sec, damping, bdm8));
        } else {
            copy_pair<Px>(dp, reinterpret_cast<const Px *>(src + (int64_t)(gy0 + r) * stride) + gx0 + x);
        }
    }
}

// Luma of one 64x64 unit, one 8x8 block per 32-lane group at a time: lane l of group g takes
// row g*8 + l/4 and pair column l%4 of the blocks (g, 0..7) in turn. Every lane of a group then
// shares the block's direction, so a tap read touches 8 rows x 4 consecutive dwords: with the
// 36-dword row stride those are 32 distinct banks (no bank conflicts for any direction), where a
// row-major mapping mixed eight directions per group. Per-block state is one broadcast LDS word
// (flag | dir << 8 | pri << 16) and the direction's tap deltas three broadcast 16-B reads.
template <typename Px, int TS>
__device__ __forceinline__ void filter_luma(const int16_t *T, const int4 (*taps)[3], const int *bstate,
                                            int sec, int damping, int bdm8, const uint8_t *src, uint8_t *dst,
                                            int64_t stride, int gx0, int gy0, int fw, int fh) {
    const int g = threadIdx.x >> 5, l = threadIdx.x & 31;     // 16 groups: block row g / 2, columns 4 (g & 1) ..
    const int r = (g >> 1) * 8 + (l >> 2), gy = gy0 + r, c0 = (g & 1) * 4;
    const char *prow = reinterpret_cast<const char *>(T + (r + 2) * TS + 2 * (l & 3) + 8);
    Px *drow = reinterpret_cast<Px *>(dst + (int64_t)gy * stride) + gx0 + 2 * (l & 3);
    const Px *srow = reinterpret_cast<const Px *>(src + (int64_t)gy * stride) + gx0 + 2 * (l & 3);
#pragma unroll
    for (int i = c0; i < c0 + 4; i++) {
        const int st = bstate[(g >> 1) * 8 + i];
        const char *P = prow + 16 * i;
        if (st & 1) {
            const int dir = (st >> 8) & 7, pri = st >> 16;
            PairTaps t;
            const int4 q0 = taps[dir][0], q1 = taps[dir][1], q2 = taps[dir][2];
            t.pri[0] = q0.x; t.pri[1] = q0.y; t.pri[2] = q0.z; t.pri[3] = q0.w;
            t.sec[0] = q1.x; t.sec[1] = q1.y; t.sec[2] = q1.z; t.sec[3] = q1.w;
            t.sec[4] = q2.x; t.sec[5] = q2.y; t.sec[6] = q2.z; t.sec[7] = q2.w;
            store_pair<Px>(drow + 8 * i, cdef_pair(P, t, pri, sec, damping, bdm8));
        } else if (gx0 + 8 * i + 2 * (l & 3) < fw && gy < fh) {
            store_pair<Px>(drow + 8 * i, ld2(P));
        } else {
            copy_pair<Px>(drow + 8 * i, srow + 8 * i);
        }
    }
}

// One 64x64 luma unit (+ co-located chroma) per 512-lane workgroup (eight waves: one per
// direction in the search, 34 KB of LDS for four workgroups = 32 waves per CU). L = layout (0 I400,
// 1 I420, 2 I422, 3 I444), compile-time so every tile index is a shift or a constant divide.
template <typename Px, int L>
__global__ __launch_bounds__(512, 8) void cdef_kernel(CdefArgs a) {
    constexpr int NTH = 512;
    constexpr int SSH = L == 1 || L == 2, SSV = L == 1;
    constexpr int CW = 64 >> SSH, CH = 64 >> SSV, CTS = CW == 64 ? 88 : 48;   // 24-dword rows: two rows 2 apart are 16 banks apart
    constexpr int UVW = 8 >> SSH, UVH = 8 >> SSV;
    constexpr int YN = kTY * kTS, CN = L ? (CH + 4) * CTS : 2;
    constexpr int NT = 2;
    __shared__ __align__(16) int16_t ty[NT * YN];              // T, T1
    __shared__ __align__(16) int16_t tuv[2][NT * CN];          // per chroma plane: T, T1
    __shared__ int8_t bdir[64];
    __shared__ int8_t bflag[64];          // bit0 luma filtered, bit1 chroma filtered
    __shared__ unsigned dcost[8][64];     // find_dir costs per direction and block
    __shared__ int bstate[64];            // luma: filtered | dir << 8 | adjusted pri << 16
    __shared__ int4 ytaps[8][3];          // luma tap byte deltas per direction (PairTaps order)
    __shared__ int4 ctaps[8][3];          // 4:2:0 chroma tap byte deltas per direction
    KTL(0);

    int bid = xcd_block(blockIdx.x, gridDim.x);
    if (a.order) {
        // the caller's order (mi_cdef_tile_order): the costliest units first
        bid = a.order[blockIdx.x];
        if ((unsigned)bid >= gridDim.x) return;
    }
    const int tx = bid % a.tiles_x, tyy = bid / a.tiles_x;
    const int x0 = tx * 64, y0 = tyy * 64;
    const MiAv1Filter *lf = &a.masks[(tyy >> 1) * a.sb128w + (tx >> 1)];
    const int cdef_idx = lf->cdef_idx[(tyy & 1) * 2 + (tx & 1)];
    const int y_lvl = cdef_idx >= 0 ? a.y_strength[cdef_idx] : 0;
    const int uv_lvl = cdef_idx >= 0 && L ? a.uv_strength[cdef_idx] : 0;
    const int fwy = a.bw4 * 4, fhy = a.bh4 * 4;
    const int fwc = fwy >> SSH, fhc = fhy >> SSV;

    if (!y_lvl && !uv_lvl) {
        // untouched 64x64 unit: C = D, 8 bytes per lane
        constexpr int PX8 = 8 / sizeof(Px);
#pragma unroll
        for (int p = 0; p < (L ? 3 : 1); p++) {
            const int pw = p ? CW : 64, ph = p ? CH : 64;
            const int px0 = p ? x0 >> SSH : x0, py0 = p ? y0 >> SSV : y0;
            const int cpr = pw / PX8;   // 8-byte chunks per row
            for (int i = threadIdx.x; i < cpr * ph; i += NTH) {
                const int r = i / cpr, c = i - r * cpr;
                const int64_t off = (int64_t)(py0 + r) * a.stride[p] + (int64_t)(px0 + c * PX8) * sizeof(Px);
                *reinterpret_cast<uint2 *>(a.dst[p] + off) = *reinterpret_cast<const uint2 *>(a.src[p] + off);
            }
        }
        KTL(5);
        return;
    }

    const int bdm8 = a.bdm8;
    const int y_pri = (y_lvl >> 2) << bdm8;
    int y_sec = y_lvl & 3; y_sec += y_sec == 3; y_sec <<= bdm8;
    const int uv_pri = (uv_lvl >> 2) << bdm8;
    int uv_sec = uv_lvl & 3; uv_sec += uv_sec == 3; uv_sec <<= bdm8;

    if (threadIdx.x < 8) {
        PairTaps t;
        make_taps<kTS, YN * 2>(t, threadIdx.x);
        ytaps[threadIdx.x][0] = make_int4(t.pri[0], t.pri[1], t.pri[2], t.pri[3]);
        ytaps[threadIdx.x][1] = make_int4(t.sec[0], t.sec[1], t.sec[2], t.sec[3]);
        ytaps[threadIdx.x][2] = make_int4(t.sec[4], t.sec[5], t.sec[6], t.sec[7]);
    } else if (L == 1 && threadIdx.x < 16) {
        PairTaps t;
        make_taps<CTS, CN * 2>(t, threadIdx.x - 8);
        ctaps[threadIdx.x - 8][0] = make_int4(t.pri[0], t.pri[1], t.pri[2], t.pri[3]);
        ctaps[threadIdx.x - 8][1] = make_int4(t.sec[0], t.sec[1], t.sec[2], t.sec[3]);
        ctaps[threadIdx.x - 8][2] = make_int4(t.sec[4], t.sec[5], t.sec[6], t.sec[7]);
    }
    {
        VecTileLoad<Px, 68, 68, NTH> ly;
        VecTileLoad<Px, CH + 4, CW + 4, NTH> lu, lv;
        ly.fetch(a.src[0], a.stride[0], x0, y0, fwy, fhy);
        if (L && uv_lvl) {
            lu.fetch(a.src[1], a.stride[1], x0 >> SSH, y0 >> SSV, fwc, fhc);
            lv.fetch(a.src[2], a.stride[2], x0 >> SSH, y0 >> SSV, fwc, fhc);
        }
        ly.store(ty, ty + YN, kTS);
        if (L && uv_lvl) {
            lu.store(tuv[0], tuv[0] + CN, CTS);
            lv.store(tuv[1], tuv[1] + CN, CTS);
        }
    }
    __syncthreads();
    KTL(1);

    if (y_pri || uv_pri) {
        const int b = threadIdx.x & 63, w = threadIdx.x >> 6;   // wave-uniform direction
        const int16_t *tb = ty + ((b >> 3) * 8 + 2) * kTS + (b & 7) * 8 + 8;
        unsigned c;
        switch (w) {
        case 0: c = dir_cost1<0>(tb, kTS, bdm8); break;
        case 1: c = dir_cost1<1>(tb, kTS, bdm8); break;
        case 2: c = dir_cost1<2>(tb, kTS, bdm8); break;
        case 3: c = dir_cost1<3>(tb, kTS, bdm8); break;
        case 4: c = dir_cost1<4>(tb, kTS, bdm8); break;
        case 5: c = dir_cost1<5>(tb, kTS, bdm8); break;
        case 6: c = dir_cost1<6>(tb, kTS, bdm8); break;
        default: c = dir_cost1<7>(tb, kTS, bdm8); break;
        }
        dcost[w][b] = c;
        __syncthreads();
    }
    KTL(2);

    if (threadIdx.x < 64) {
        const int b = threadIdx.x, bxl = b & 7, byl = b >> 3;
        const int bx = (x0 >> 2) + bxl * 2, by = (y0 >> 2) + byl * 2;   // 4-px units
        int flag = 0, dir = 0, pri = 0;
        if (bx < a.bw4 && by < a.bh4) {
            const int by_idx = (by & 30) >> 1;
            const unsigned noskip = (unsigned)lf->noskip_mask[by_idx][1] << 16 | lf->noskip_mask[by_idx][0];
            if (noskip & (3u << (bx & 30))) {
                unsigned var = 0;
                if (y_pri || uv_pri) {
                    unsigned bc = dcost[0][b];
#pragma unroll
                    for (int n = 1; n < 8; n++)
                        if (dcost[n][b] > bc) { bc = dcost[n][b]; dir = n; }
                    var = (bc - dcost[dir ^ 4][b]) >> 10;
                }
                if (y_pri) {
                    pri = adjust_strength(y_pri, var);
                    if (pri || y_sec) flag |= 1;
                } else if (y_sec) {
                    flag |= 1;
                }
                if (uv_lvl) flag |= 2;
            }
        }
        bdir[b] = (int8_t)dir;
        bflag[b] = (int8_t)flag;
        bstate[b] = (flag & 1) | (y_pri ? dir : 0) << 8 | (y_pri ? pri : 0) << 16;
    }
    __syncthreads();
    KTL(3);

    // luma: 2048 pairs, one 8x8 block per 32-lane group at a time
    filter_luma<Px, kTS>(ty, ytaps, bstate, y_sec, a.damping, bdm8, a.src[0], a.dst[0], a.stride[0],
                             x0, y0, fwy, fhy);
    KTL(4);
    if (L) {
        // chroma: lanes 0..255 U, 256..511 V (damping - 1, cdef_apply.rs)
        const int p = 1 + (threadIdx.x >> 8);
        // (the chroma tile is only staged when uv_lvl != 0: unfiltered chroma copies from D)
        if constexpr (L == 1)
            filter_chroma420<Px, CTS>(tuv[p - 1], ctaps, bdir, bflag, uv_pri, uv_sec, a.damping - 1, bdm8,
                                      a.src[p], a.dst[p], a.stride[p], x0 >> SSH, y0 >> SSV);
        else
            filter_plane<Px, CW, CH, UVW, UVH, 256, CTS, CN * 2, 2, false>(
                tuv[p - 1], threadIdx.x & 255, bdir, bflag, nullptr, false, uv_pri, uv_sec, a.damping - 1, bdm8,
                L == 2, a.src[p], a.dst[p], a.stride[p], x0 >> SSH, y0 >> SSV, fwc, fhc);
    }
    KTL(5);
}

// ---- per-call cdef.fb[] / cdef.dir (cdef.rs:567-1031) ----
// One block (8x8, 4x8 or 4x4): the padded i16 tile is built in LDS as the reference's
// `padding` does (the block from dst, 2 columns from left, 2 rows above from top and below
// from bottom, i16::MIN where `edges` says the neighbour is missing), then one lane per pixel.
constexpr int kCallTs = 12;
template <typename Px>
__global__ __launch_bounds__(64) void cdef_call_kernel(CdefCallArgs a) {
    __shared__ int16_t tb[kCallTs * kCallTs];
    int16_t *t = tb + 2 * kCallTs + 2;
    const int lane = threadIdx.x, w = a.w, h = a.h;
    const int64_t ps = a.stride / (int64_t)sizeof(Px);
    const Px *dst = reinterpret_cast<const Px *>(a.dst), *top = reinterpret_cast<const Px *>(a.top);
    const Px *bot = reinterpret_cast<const Px *>(a.bottom), *left = reinterpret_cast<const Px *>(a.left);
    for (int i = lane; i < kCallTs * kCallTs; i += 64) {
        const int y = i / kCallTs - 2, x = i % kCallTs - 2;
        int v = INT16_MIN;
        if (y < h + 2 && x < w + 2) {
            const bool in_x = x >= 0 ? (x < w || (a.edges & 2)) : (a.edges & 1);   // HAVE_RIGHT 2, HAVE_LEFT 1
            const bool in_y = y >= 0 ? (y < h || (a.edges & 8)) : (a.edges & 4);   // HAVE_BOTTOM 8, HAVE_TOP 4
            if (in_x && in_y) {
                if (y < 0) v = top[(y + 2) * ps + x];
                else if (y >= h) v = bot[(y - h) * ps + x];
                else if (x < 0) v = left[y * 2 + 2 + x];
                else v = dst[y * ps + x];
            }
        }
        tb[i] = (int16_t)v;
    }
    __syncthreads();
    if (lane < w * h) {
        const int y = lane / w, x = lane % w;
        const int v = cdef_px(t, kCallTs, x, y, a.pri, a.sec, a.dir, a.damping, a.bdm8);
        reinterpret_cast<Px *>(a.out)[y * w + x] = (Px)v;
    }
}

template <typename Px>
__global__ __launch_bounds__(64) void cdef_dir_call_kernel(CdefCallArgs a) {
    __shared__ int16_t t[64];
    const int64_t ps = a.stride / (int64_t)sizeof(Px);
    const int lane = threadIdx.x;
    t[lane] = (int16_t)reinterpret_cast<const Px *>(a.dst)[(lane >> 3) * ps + (lane & 7)];
    __syncthreads();
    if (lane == 0) {
        unsigned var;
        const int d = find_dir(t, 8, a.bdm8, &var);
        reinterpret_cast<int *>(a.out)[0] = d;
        reinterpret_cast<unsigned *>(a.out)[1] = var;
    }
}

int launch_cdef_call(const CdefCallArgs &a, int bpc, bool dir, hipStream_t s) {
    if (dir) {
        if (bpc == 8) cdef_dir_call_kernel<uint8_t><<<1, 64, 0, s>>>(a);
        else cdef_dir_call_kernel<uint16_t><<<1, 64, 0, s>>>(a);
    } else {
        if (bpc == 8) cdef_call_kernel<uint8_t><<<1, 64, 0, s>>>(a);
        else cdef_call_kernel<uint16_t><<<1, 64, 0, s>>>(a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_cdef(const CdefArgs &a, int tiles, int bpc, hipStream_t s) {
    if (tiles <= 0) return 0;
#define MI_CDEF_LAUNCH(L)                                                                            \
    do {                                                                                             \
        if (bpc == 8) cdef_kernel<uint8_t, L><<<tiles, 512, 0, s>>>(a);                               \
        else cdef_kernel<uint16_t, L><<<tiles, 512, 0, s>>>(a);                                       \
    } while (0)
    switch (a.layout) {
    case 0: MI_CDEF_LAUNCH(0); break;
    case 1: MI_CDEF_LAUNCH(1); break;
    case 2: MI_CDEF_LAUNCH(2); break;
    default: MI_CDEF_LAUNCH(3); break;
    }
#undef MI_CDEF_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
