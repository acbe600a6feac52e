// itx_1d.h — gfx950 device 1-D inverse transforms (one lane runs one whole 1-D transform
// in VGPRs; the 2-D driver in itx.hip feeds rows/columns through LDS).
//
// Semantics follow rav1d src/itx_1d.rs:5-1140 (C twin src/itx_1d.c:66-1034): the same
// butterfly network, the same CLIP points and output negations. Rotations are evaluated as
// the exact value (a*ca + b*cb + 2048) >> 12 — the reference's "(c - 4096)" rewrite is
// value-identical and exists only to avoid 32-bit overflow on 12-bit streams. For 8/10 bpc
// every product and pair-sum fits in 32 bits (|in| <= 2^17, |c| < 2^12); the 12-bit
// instantiation (Wide = true) evaluates products in 64 bits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi {

template <bool Wide>
struct Ar {
    __device__ static __forceinline__ int r12(int a, int ca, int b, int cb) {
        if constexpr (Wide)
            return (int)(((int64_t)a * ca + (int64_t)b * cb + 2048) >> 12);
        else
            return (a * ca + b * cb + 2048) >> 12;
    }
    __device__ static __forceinline__ int s12(int a, int ca) {
        if constexpr (Wide) return (int)(((int64_t)a * ca + 2048) >> 12);
        else return (a * ca + 2048) >> 12;
    }
    __device__ static __forceinline__ int h181(int x) {
        if constexpr (Wide) return (int)(((int64_t)x * 181 + 128) >> 8);
        else return (x * 181 + 128) >> 8;
    }
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

// c[i*S] addressing on a register array; S, N compile-time so everything stays in VGPRs.
#define E(i) c[(i) * S]

template <bool W, int S>
__device__ __forceinline__ void idct4(int *c, int lo, int hi, bool half) {
    using A = Ar<W>;
    int e0, e1, o0, o1;
    if (half) {
        e0 = e1 = A::h181(E(0));
        o0 = A::s12(E(1), 1567);
        o1 = A::s12(E(1), 3784);
    } else {
        e0 = A::h181(E(0) + E(2));
        e1 = A::h181(E(0) - E(2));
        o0 = A::r12(E(1), 1567, E(3), -3784);
        o1 = A::r12(E(1), 3784, E(3), 1567);
    }
    E(0) = clampi(e0 + o1, lo, hi);
    E(1) = clampi(e1 + o0, lo, hi);
    E(2) = clampi(e1 - o0, lo, hi);
    E(3) = clampi(e0 - o1, lo, hi);
}

// Combine the even half (already transformed in place at even slots) with the odd half o[]:
// out[i] = even[i] + o[n/2-1-i], out[n-1-i] = even[i] - o[n/2-1-i].
template <int N, int S>
__device__ __forceinline__ void dct_merge(int *c, const int *o, int lo, int hi) {
    int ev[N / 2];
#pragma unroll
    for (int i = 0; i < N / 2; i++) ev[i] = E(2 * i);
#pragma unroll
    for (int i = 0; i < N / 2; i++) {
        E(i) = clampi(ev[i] + o[N / 2 - 1 - i], lo, hi);
        E(N - 1 - i) = clampi(ev[i] - o[N / 2 - 1 - i], lo, hi);
    }
}

template <bool W, int S>
__device__ __forceinline__ void idct8(int *c, int lo, int hi, bool half) {
    using A = Ar<W>;
    idct4<W, 2 * S>(c, lo, hi, half);
    int a4, a5, a6, a7;
    if (half) {
        a4 = A::s12(E(1), 799);
        a5 = A::s12(E(3), -2276);
        a6 = A::s12(E(3), 3406);
        a7 = A::s12(E(1), 4017);
    } else {
        a4 = A::r12(E(1), 799, E(7), -4017);
        a5 = A::r12(E(5), 3406, E(3), -2276);
        a6 = A::r12(E(5), 2276, E(3), 3406);
        a7 = A::r12(E(1), 4017, E(7), 799);
    }
    const int b4 = clampi(a4 + a5, lo, hi), b5 = clampi(a4 - a5, lo, hi);
    const int b7 = clampi(a7 + a6, lo, hi), b6 = clampi(a7 - a6, lo, hi);
    const int o[4] = { b4, A::h181(b6 - b5), A::h181(b6 + b5), b7 };
    dct_merge<8, S>(c, o, lo, hi);
}

template <bool W, int S>
__device__ __forceinline__ void idct16(int *c, int lo, int hi, bool half) {
    using A = Ar<W>;
    idct8<W, 2 * S>(c, lo, hi, half);
    int t[16];
    if (half) {
        t[8] = A::s12(E(1), 401);   t[9] = A::s12(E(7), -2598);
        t[10] = A::s12(E(5), 1931); t[11] = A::s12(E(3), -1189);
        t[12] = A::s12(E(3), 3920); t[13] = A::s12(E(5), 3612);
        t[14] = A::s12(E(7), 3166); t[15] = A::s12(E(1), 4076);
    } else {
        t[8] = A::r12(E(1), 401, E(15), -4076);
        t[9] = A::r12(E(9), 3166, E(7), -2598);
        t[10] = A::r12(E(5), 1931, E(11), -3612);
        t[11] = A::r12(E(13), 3920, E(3), -1189);
        t[12] = A::r12(E(13), 1189, E(3), 3920);
        t[13] = A::r12(E(5), 3612, E(11), 1931);
        t[14] = A::r12(E(9), 2598, E(7), 3166);
        t[15] = A::r12(E(1), 4076, E(15), 401);
    }
    // butterflies: (8,9) sum/diff; (11,10) sum/diff reversed; ...
    int u8 = clampi(t[8] + t[9], lo, hi), u9 = clampi(t[8] - t[9], lo, hi);
    int u10 = clampi(t[11] - t[10], lo, hi), u11 = clampi(t[11] + t[10], lo, hi);
    int u12 = clampi(t[12] + t[13], lo, hi), u13 = clampi(t[12] - t[13], lo, hi);
    int u14 = clampi(t[15] - t[14], lo, hi), u15 = clampi(t[15] + t[14], lo, hi);
    const int v9 = A::r12(u14, 1567, u9, -3784);
    const int v14 = A::r12(u14, 3784, u9, 1567);
    const int v10 = A::r12(u13, -3784, u10, -1567);
    const int v13 = A::r12(u13, 1567, u10, -3784);
    const int w8 = clampi(u8 + u11, lo, hi), w11 = clampi(u8 - u11, lo, hi);
    const int w9 = clampi(v9 + v10, lo, hi), w10 = clampi(v9 - v10, lo, hi);
    const int w12 = clampi(u15 - u12, lo, hi), w15 = clampi(u15 + u12, lo, hi);
    const int w13 = clampi(v14 - v13, lo, hi), w14 = clampi(v14 + v13, lo, hi);
    const int o[8] = { w8, w9, A::h181(w13 - w10), A::h181(w12 - w11),
                       A::h181(w12 + w11), A::h181(w13 + w10), w14, w15 };
    dct_merge<16, S>(c, o, lo, hi);
}

template <bool W, int S>
__device__ __forceinline__ void idct32(int *c, int lo, int hi, bool half) {
    using A = Ar<W>;
    idct16<W, 2 * S>(c, lo, hi, half);
    int t[32];
    if (half) {
        t[16] = A::s12(E(1), 201);   t[17] = A::s12(E(15), -2751);
        t[18] = A::s12(E(9), 1751);  t[19] = A::s12(E(7), -1380);
        t[20] = A::s12(E(5), 995);   t[21] = A::s12(E(11), -2106);
        t[22] = A::s12(E(13), 2440); t[23] = A::s12(E(3), -601);
        t[24] = A::s12(E(3), 4052);  t[25] = A::s12(E(13), 3290);
        t[26] = A::s12(E(11), 3513); t[27] = A::s12(E(5), 3973);
        t[28] = A::s12(E(7), 3857);  t[29] = A::s12(E(9), 3703);
        t[30] = A::s12(E(15), 3035); t[31] = A::s12(E(1), 4091);
    } else {
        t[16] = A::r12(E(1), 201, E(31), -4091);
        t[17] = A::r12(E(17), 3035, E(15), -2751);
        t[18] = A::r12(E(9), 1751, E(23), -3703);
        t[19] = A::r12(E(25), 3857, E(7), -1380);
        t[20] = A::r12(E(5), 995, E(27), -3973);
        t[21] = A::r12(E(21), 3513, E(11), -2106);
        t[22] = A::r12(E(13), 2440, E(19), -3290);
        t[23] = A::r12(E(29), 4052, E(3), -601);
        t[24] = A::r12(E(29), 601, E(3), 4052);
        t[25] = A::r12(E(13), 3290, E(19), 2440);
        t[26] = A::r12(E(21), 2106, E(11), 3513);
        t[27] = A::r12(E(5), 3973, E(27), 995);
        t[28] = A::r12(E(25), 1380, E(7), 3857);
        t[29] = A::r12(E(9), 3703, E(23), 1751);
        t[30] = A::r12(E(17), 2751, E(15), 3035);
        t[31] = A::r12(E(1), 4091, E(31), 201);
    }
    int u[32];
    // groups of four: (+,-,-rev,+rev)
#pragma unroll
    for (int g = 16; g < 32; g += 4) {
        u[g] = clampi(t[g] + t[g + 1], lo, hi);
        u[g + 1] = clampi(t[g] - t[g + 1], lo, hi);
        u[g + 2] = clampi(t[g + 3] - t[g + 2], lo, hi);
        u[g + 3] = clampi(t[g + 3] + t[g + 2], lo, hi);
    }
    {
        const int r17 = A::r12(u[30], 799, u[17], -4017);
        const int r30 = A::r12(u[30], 4017, u[17], 799);
        const int r18 = A::r12(u[29], -4017, u[18], -799);
        const int r29 = A::r12(u[29], 799, u[18], -4017);
        const int r21 = A::r12(u[26], 3406, u[21], -2276);
        const int r26 = A::r12(u[26], 2276, u[21], 3406);
        const int r22 = A::r12(u[25], -2276, u[22], -3406);
        const int r25 = A::r12(u[25], 3406, u[22], -2276);
        u[17] = r17; u[30] = r30; u[18] = r18; u[29] = r29;
        u[21] = r21; u[26] = r26; u[22] = r22; u[25] = r25;
    }
    int v[32];
#pragma unroll
    for (int g = 16; g < 32; g += 8) {
        v[g] = clampi(u[g] + u[g + 3], lo, hi);
        v[g + 1] = clampi(u[g + 1] + u[g + 2], lo, hi);
        v[g + 2] = clampi(u[g + 1] - u[g + 2], lo, hi);
        v[g + 3] = clampi(u[g] - u[g + 3], lo, hi);
        v[g + 4] = clampi(u[g + 7] - u[g + 4], lo, hi);
        v[g + 5] = clampi(u[g + 6] - u[g + 5], lo, hi);
        v[g + 6] = clampi(u[g + 6] + u[g + 5], lo, hi);
        v[g + 7] = clampi(u[g + 7] + u[g + 4], lo, hi);
    }
    {
        const int s18 = A::r12(v[29], 1567, v[18], -3784);
        const int s29 = A::r12(v[29], 3784, v[18], 1567);
        const int s19 = A::r12(v[28], 1567, v[19], -3784);
        const int s28 = A::r12(v[28], 3784, v[19], 1567);
        const int s20 = A::r12(v[27], -3784, v[20], -1567);
        const int s27 = A::r12(v[27], 1567, v[20], -3784);
        const int s21 = A::r12(v[26], -3784, v[21], -1567);
        const int s26 = A::r12(v[26], 1567, v[21], -3784);
        v[18] = s18; v[29] = s29; v[19] = s19; v[28] = s28;
        v[20] = s20; v[27] = s27; v[21] = s21; v[26] = s26;
    }
    int w[32];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        w[16 + k] = clampi(v[16 + k] + v[23 - k], lo, hi);
        w[23 - k] = clampi(v[16 + k] - v[23 - k], lo, hi);
        w[24 + k] = clampi(v[31 - k] - v[24 + k], lo, hi);
        w[31 - k] = clampi(v[31 - k] + v[24 + k], lo, hi);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int l = 20 + k, h = 27 - k;
        const int wl = w[l], wh = w[h];
        w[l] = A::h181(wh - wl);
        w[h] = A::h181(wh + wl);
    }
    int o[16];
#pragma unroll
    for (int i = 0; i < 16; i++) o[i] = w[16 + i];
    dct_merge<32, S>(c, o, lo, hi);
}

// 64-point: only inputs 0..31 can be nonzero (the reference's tx64 path).
template <bool W, int S>
__device__ __forceinline__ void idct64(int *c, int lo, int hi) {
    using A = Ar<W>;
    idct32<W, 2 * S>(c, lo, hi, true);
    int t[64];
    // input scales: (input index, constant) for t32..t63
    t[32] = A::s12(E(1), 101);   t[33] = A::s12(E(31), -2824);
    t[34] = A::s12(E(17), 1660); t[35] = A::s12(E(15), -1474);
    t[36] = A::s12(E(9), 897);   t[37] = A::s12(E(23), -2191);
    t[38] = A::s12(E(25), 2359); t[39] = A::s12(E(7), -700);
    t[40] = A::s12(E(5), 501);   t[41] = A::s12(E(27), -2520);
    t[42] = A::s12(E(21), 2019); t[43] = A::s12(E(11), -1092);
    t[44] = A::s12(E(13), 1285); t[45] = A::s12(E(19), -1842);
    t[46] = A::s12(E(29), 2675); t[47] = A::s12(E(3), -301);
    t[48] = A::s12(E(3), 4085);  t[49] = A::s12(E(29), 3102);
    t[50] = A::s12(E(19), 3659); t[51] = A::s12(E(13), 3889);
    t[52] = A::s12(E(11), 3948); t[53] = A::s12(E(21), 3564);
    t[54] = A::s12(E(27), 3229); t[55] = A::s12(E(5), 4065);
    t[56] = A::s12(E(7), 4036);  t[57] = A::s12(E(25), 3349);
    t[58] = A::s12(E(23), 3461); t[59] = A::s12(E(9), 3996);
    t[60] = A::s12(E(15), 3822); t[61] = A::s12(E(17), 3745);
    t[62] = A::s12(E(31), 2967); t[63] = A::s12(E(1), 4095);
    int u[64];
#pragma unroll
    for (int g = 32; g < 64; g += 4) {
        u[g] = clampi(t[g] + t[g + 1], lo, hi);
        u[g + 1] = clampi(t[g] - t[g + 1], lo, hi);
        u[g + 2] = clampi(t[g + 3] - t[g + 2], lo, hi);
        u[g + 3] = clampi(t[g + 3] + t[g + 2], lo, hi);
    }
    {
        // stage-1 rotation pairs (lo index, hi index, k0, k1): rotated as
        //   lo' = r(lo*-k1 + hi*k0) , hi' = r(lo*k0 + hi*k1) for the "upper" pairs
        const int a33 = A::r12(u[33], -4076, u[62], 401);
        const int a62 = A::r12(u[33], 401, u[62], 4076);
        const int a34 = A::r12(u[34], -401, u[61], -4076);
        const int a61 = A::r12(u[34], -4076, u[61], 401);
        const int a37 = A::r12(u[37], -2598, u[58], 3166);
        const int a58 = A::r12(u[37], 3166, u[58], 2598);
        const int a38 = A::r12(u[38], -3166, u[57], -2598);
        const int a57 = A::r12(u[38], -2598, u[57], 3166);
        const int a41 = A::r12(u[41], -3612, u[54], 1931);
        const int a54 = A::r12(u[41], 1931, u[54], 3612);
        const int a42 = A::r12(u[42], -1931, u[53], -3612);
        const int a53 = A::r12(u[42], -3612, u[53], 1931);
        const int a45 = A::r12(u[45], -1189, u[50], 3920);
        const int a50 = A::r12(u[45], 3920, u[50], 1189);
        const int a46 = A::r12(u[46], -3920, u[49], -1189);
        const int a49 = A::r12(u[46], -1189, u[49], 3920);
        u[33] = a33; u[62] = a62; u[34] = a34; u[61] = a61;
        u[37] = a37; u[58] = a58; u[38] = a38; u[57] = a57;
        u[41] = a41; u[54] = a54; u[42] = a42; u[53] = a53;
        u[45] = a45; u[50] = a50; u[46] = a46; u[49] = a49;
    }
    int v[64];
#pragma unroll
    for (int g = 32; g < 64; g += 8) {
        v[g] = clampi(u[g] + u[g + 3], lo, hi);
        v[g + 1] = clampi(u[g + 1] + u[g + 2], lo, hi);
        v[g + 2] = clampi(u[g + 1] - u[g + 2], lo, hi);
        v[g + 3] = clampi(u[g] - u[g + 3], lo, hi);
        v[g + 4] = clampi(u[g + 7] - u[g + 4], lo, hi);
        v[g + 5] = clampi(u[g + 6] - u[g + 5], lo, hi);
        v[g + 6] = clampi(u[g + 6] + u[g + 5], lo, hi);
        v[g + 7] = clampi(u[g + 7] + u[g + 4], lo, hi);
    }
    {
        const int b34 = A::r12(v[34], -4017, v[61], 799);
        const int b61 = A::r12(v[34], 799, v[61], 4017);
        const int b35 = A::r12(v[35], -4017, v[60], 799);
        const int b60 = A::r12(v[35], 799, v[60], 4017);
        const int b36 = A::r12(v[36], -799, v[59], -4017);
        const int b59 = A::r12(v[36], -4017, v[59], 799);
        const int b37 = A::r12(v[37], -799, v[58], -4017);
        const int b58 = A::r12(v[37], -4017, v[58], 799);
        const int b42 = A::r12(v[42], -2276, v[53], 3406);
        const int b53 = A::r12(v[42], 3406, v[53], 2276);
        const int b43 = A::r12(v[43], -2276, v[52], 3406);
        const int b52 = A::r12(v[43], 3406, v[52], 2276);
        const int b44 = A::r12(v[44], -3406, v[51], -2276);
        const int b51 = A::r12(v[44], -2276, v[51], 3406);
        const int b45 = A::r12(v[45], -3406, v[50], -2276);
        const int b50 = A::r12(v[45], -2276, v[50], 3406);
        v[34] = b34; v[61] = b61; v[35] = b35; v[60] = b60;
        v[36] = b36; v[59] = b59; v[37] = b37; v[58] = b58;
        v[42] = b42; v[53] = b53; v[43] = b43; v[52] = b52;
        v[44] = b44; v[51] = b51; v[45] = b45; v[50] = b50;
    }
    int w[64];
#pragma unroll
    for (int g = 32; g < 64; g += 16) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            w[g + k] = clampi(v[g + k] + v[g + 7 - k], lo, hi);
            w[g + 7 - k] = clampi(v[g + k] - v[g + 7 - k], lo, hi);
            w[g + 8 + k] = clampi(v[g + 15 - k] - v[g + 8 + k], lo, hi);
            w[g + 15 - k] = clampi(v[g + 15 - k] + v[g + 8 + k], lo, hi);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int p = 36 + k, q = 59 - k;
        const int wp = w[p], wq = w[q];
        w[p] = A::r12(wp, -3784, wq, 1567);
        w[q] = A::r12(wp, 1567, wq, 3784);
        const int r = 40 + k, s = 55 - k;
        const int wr = w[r], ws = w[s];
        w[r] = A::r12(wr, -1567, ws, -3784);
        w[s] = A::r12(wr, -3784, ws, 1567);
    }
    int x[64];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        x[32 + k] = clampi(w[32 + k] + w[47 - k], lo, hi);
        x[47 - k] = clampi(w[32 + k] - w[47 - k], lo, hi);
        x[48 + k] = clampi(w[63 - k] - w[48 + k], lo, hi);
        x[63 - k] = clampi(w[63 - k] + w[48 + k], lo, hi);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int l = 40 + k, h = 55 - k;
        const int xl = x[l], xh = x[h];
        x[l] = A::h181(xh - xl);
        x[h] = A::h181(xh + xl);
    }
    int o[32];
#pragma unroll
    for (int i = 0; i < 32; i++) o[i] = x[32 + i];
    dct_merge<64, S>(c, o, lo, hi);
}

// The 64-point DCT over a lane pair (the even and the odd lane of an aligned pair), so that no
// lane holds more than 32 values: idct64 is its even half (a 32-point DCT of inputs 0, 2, ..,
// 30) merged with its odd half (the t32..t63 network of inputs 1, 3, .., 31). In: y[k] = input
// 2k (even lane) or 2k + 1 (odd lane), k < 16 (inputs >= 32 are zero, as in idct64). Out: the
// even lane's y[i] = output i, the odd lane's y[i] = output 63 - i. The merge trades each
// lane's half with its partner by DPP (quad_perm [1,0,3,2]); both lanes run both halves'
// code paths masked, so a wave stays converged.
__device__ __forceinline__ int pair_swap(int v) {
    return __builtin_amdgcn_mov_dpp(v, 0xb1, 0xf, 0xf, false);
}
#define OD(i) y[((i) - 1) >> 1]
template <bool W>
__device__ __forceinline__ void idct64_odd(int *y, int lo, int hi) {
    using A = Ar<W>;
    int t[64];
    t[32] = A::s12(OD(1), 101);   t[33] = A::s12(OD(31), -2824);
    t[34] = A::s12(OD(17), 1660); t[35] = A::s12(OD(15), -1474);
    t[36] = A::s12(OD(9), 897);   t[37] = A::s12(OD(23), -2191);
    t[38] = A::s12(OD(25), 2359); t[39] = A::s12(OD(7), -700);
    t[40] = A::s12(OD(5), 501);   t[41] = A::s12(OD(27), -2520);
    t[42] = A::s12(OD(21), 2019); t[43] = A::s12(OD(11), -1092);
    t[44] = A::s12(OD(13), 1285); t[45] = A::s12(OD(19), -1842);
    t[46] = A::s12(OD(29), 2675); t[47] = A::s12(OD(3), -301);
    t[48] = A::s12(OD(3), 4085);  t[49] = A::s12(OD(29), 3102);
    t[50] = A::s12(OD(19), 3659); t[51] = A::s12(OD(13), 3889);
    t[52] = A::s12(OD(11), 3948); t[53] = A::s12(OD(21), 3564);
    t[54] = A::s12(OD(27), 3229); t[55] = A::s12(OD(5), 4065);
    t[56] = A::s12(OD(7), 4036);  t[57] = A::s12(OD(25), 3349);
    t[58] = A::s12(OD(23), 3461); t[59] = A::s12(OD(9), 3996);
    t[60] = A::s12(OD(15), 3822); t[61] = A::s12(OD(17), 3745);
    t[62] = A::s12(OD(31), 2967); t[63] = A::s12(OD(1), 4095);
    int u[64];
#pragma unroll
    for (int g = 32; g < 64; g += 4) {
        u[g] = clampi(t[g] + t[g + 1], lo, hi);
        u[g + 1] = clampi(t[g] - t[g + 1], lo, hi);
        u[g + 2] = clampi(t[g + 3] - t[g + 2], lo, hi);
        u[g + 3] = clampi(t[g + 3] + t[g + 2], lo, hi);
    }
    {
        const int a33 = A::r12(u[33], -4076, u[62], 401);
        const int a62 = A::r12(u[33], 401, u[62], 4076);
        const int a34 = A::r12(u[34], -401, u[61], -4076);
        const int a61 = A::r12(u[34], -4076, u[61], 401);
        const int a37 = A::r12(u[37], -2598, u[58], 3166);
        const int a58 = A::r12(u[37], 3166, u[58], 2598);
        const int a38 = A::r12(u[38], -3166, u[57], -2598);
        const int a57 = A::r12(u[38], -2598, u[57], 3166);
        const int a41 = A::r12(u[41], -3612, u[54], 1931);
        const int a54 = A::r12(u[41], 1931, u[54], 3612);
        const int a42 = A::r12(u[42], -1931, u[53], -3612);
        const int a53 = A::r12(u[42], -3612, u[53], 1931);
        const int a45 = A::r12(u[45], -1189, u[50], 3920);
        const int a50 = A::r12(u[45], 3920, u[50], 1189);
        const int a46 = A::r12(u[46], -3920, u[49], -1189);
        const int a49 = A::r12(u[46], -1189, u[49], 3920);
        u[33] = a33; u[62] = a62; u[34] = a34; u[61] = a61;
        u[37] = a37; u[58] = a58; u[38] = a38; u[57] = a57;
        u[41] = a41; u[54] = a54; u[42] = a42; u[53] = a53;
        u[45] = a45; u[50] = a50; u[46] = a46; u[49] = a49;
    }
    int v[64];
#pragma unroll
    for (int g = 32; g < 64; g += 8) {
        v[g] = clampi(u[g] + u[g + 3], lo, hi);
        v[g + 1] = clampi(u[g + 1] + u[g + 2], lo, hi);
        v[g + 2] = clampi(u[g + 1] - u[g + 2], lo, hi);
        v[g + 3] = clampi(u[g] - u[g + 3], lo, hi);
        v[g + 4] = clampi(u[g + 7] - u[g + 4], lo, hi);
        v[g + 5] = clampi(u[g + 6] - u[g + 5], lo, hi);
        v[g + 6] = clampi(u[g + 6] + u[g + 5], lo, hi);
        v[g + 7] = clampi(u[g + 7] + u[g + 4], lo, hi);
    }
    {
        const int b34 = A::r12(v[34], -4017, v[61], 799);
        const int b61 = A::r12(v[34], 799, v[61], 4017);
        const int b35 = A::r12(v[35], -4017, v[60], 799);
        const int b60 = A::r12(v[35], 799, v[60], 4017);
        const int b36 = A::r12(v[36], -799, v[59], -4017);
        const int b59 = A::r12(v[36], -4017, v[59], 799);
        const int b37 = A::r12(v[37], -799, v[58], -4017);
        const int b58 = A::r12(v[37], -4017, v[58], 799);
        const int b42 = A::r12(v[42], -2276, v[53], 3406);
        const int b53 = A::r12(v[42], 3406, v[53], 2276);
        const int b43 = A::r12(v[43], -2276, v[52], 3406);
        const int b52 = A::r12(v[43], 3406, v[52], 2276);
        const int b44 = A::r12(v[44], -3406, v[51], -2276);
        const int b51 = A::r12(v[44], -2276, v[51], 3406);
        const int b45 = A::r12(v[45], -3406, v[50], -2276);
        const int b50 = A::r12(v[45], -2276, v[50], 3406);
        v[34] = b34; v[61] = b61; v[35] = b35; v[60] = b60;
        v[36] = b36; v[59] = b59; v[37] = b37; v[58] = b58;
        v[42] = b42; v[53] = b53; v[43] = b43; v[52] = b52;
        v[44] = b44; v[51] = b51; v[45] = b45; v[50] = b50;
    }
    int w[64];
#pragma unroll
    for (int g = 32; g < 64; g += 16) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            w[g + k] = clampi(v[g + k] + v[g + 7 - k], lo, hi);
            w[g + 7 - k] = clampi(v[g + k] - v[g + 7 - k], lo, hi);
            w[g + 8 + k] = clampi(v[g + 15 - k] - v[g + 8 + k], lo, hi);
            w[g + 15 - k] = clampi(v[g + 15 - k] + v[g + 8 + k], lo, hi);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int p = 36 + k, q = 59 - k;
        const int wp = w[p], wq = w[q];
        w[p] = A::r12(wp, -3784, wq, 1567);
        w[q] = A::r12(wp, 1567, wq, 3784);
        const int r = 40 + k, s = 55 - k;
        const int wr = w[r], ws = w[s];
        w[r] = A::r12(wr, -1567, ws, -3784);
        w[s] = A::r12(wr, -3784, ws, 1567);
    }
    int x[64];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        x[32 + k] = clampi(w[32 + k] + w[47 - k], lo, hi);
        x[47 - k] = clampi(w[32 + k] - w[47 - k], lo, hi);
        x[48 + k] = clampi(w[63 - k] - w[48 + k], lo, hi);
        x[63 - k] = clampi(w[63 - k] + w[48 + k], lo, hi);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int l = 40 + k, h = 55 - k;
        const int xl = x[l], xh = x[h];
        x[l] = A::h181(xh - xl);
        x[h] = A::h181(xh + xl);
    }
#pragma unroll
    for (int i = 0; i < 32; i++) y[i] = x[32 + i];
}
#undef OD

template <bool W>
__device__ __forceinline__ void idct64_pair(int *y, bool odd, int lo, int hi) {
    if (!odd) {
#pragma unroll
        for (int i = 16; i < 32; i++) y[i] = 0;
        idct32<W, 1>(y, lo, hi, true);
    } else {
        idct64_odd<W>(y, lo, hi);
    }
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int a = y[i], b = y[31 - i];
        const int sa = pair_swap(a), sb = pair_swap(b);
        y[i] = odd ? clampi(sa - b, lo, hi) : clampi(a + sb, lo, hi);
        y[31 - i] = odd ? clampi(sb - a, lo, hi) : clampi(b + sa, lo, hi);
    }
}

// ---- ADST: outputs written in natural order into `out` (flip handled by the caller) ----

template <bool W>
__device__ __forceinline__ void iadst4(const int *x, int *out) {
    if constexpr (W) {
        const int64_t a = x[0], b = x[1], d = x[2], e = x[3];
        out[0] = (int)((1321 * a + 3344 * b + 3803 * d + 2482 * e + 2048) >> 12);
        out[1] = (int)((2482 * a + 3344 * b - 1321 * d - 3803 * e + 2048) >> 12);
        out[2] = (int)((209 * (a - d + e) + 128) >> 8);
        out[3] = (int)((3803 * a - 3344 * b + 2482 * d - 1321 * e + 2048) >> 12);
    } else {
        const int a = x[0], b = x[1], d = x[2], e = x[3];
        out[0] = (1321 * a + 3344 * b + 3803 * d + 2482 * e + 2048) >> 12;
        out[1] = (2482 * a + 3344 * b - 1321 * d - 3803 * e + 2048) >> 12;
        out[2] = (209 * (a - d + e) + 128) >> 8;
        out[3] = (3803 * a - 3344 * b + 2482 * d - 1321 * e + 2048) >> 12;
    }
}

template <bool W>
__device__ __forceinline__ void iadst8(const int *x, int *out, int lo, int hi) {
    using A = Ar<W>;
    const int p0 = A::r12(x[7], 4076, x[0], 401), p1 = A::r12(x[7], 401, x[0], -4076);
    const int p2 = A::r12(x[5], 3612, x[2], 1931), p3 = A::r12(x[5], 1931, x[2], -3612);
    const int p4 = A::r12(x[3], 2598, x[4], 3166), p5 = A::r12(x[3], 3166, x[4], -2598);
    const int p6 = A::r12(x[1], 1189, x[6], 3920), p7 = A::r12(x[1], 3920, x[6], -1189);
    const int q0 = clampi(p0 + p4, lo, hi), q4 = clampi(p0 - p4, lo, hi);
    const int q1 = clampi(p1 + p5, lo, hi), q5 = clampi(p1 - p5, lo, hi);
    const int q2 = clampi(p2 + p6, lo, hi), q6 = clampi(p2 - p6, lo, hi);
    const int q3 = clampi(p3 + p7, lo, hi), q7 = clampi(p3 - p7, lo, hi);
    const int r4 = A::r12(q4, 3784, q5, 1567), r5 = A::r12(q4, 1567, q5, -3784);
    const int r6 = A::r12(q7, 3784, q6, -1567), r7 = A::r12(q7, 1567, q6, 3784);
    out[0] = clampi(q0 + q2, lo, hi);
    out[7] = -clampi(q1 + q3, lo, hi);
    const int s2 = clampi(q0 - q2, lo, hi), s3 = clampi(q1 - q3, lo, hi);
    out[1] = -clampi(r4 + r6, lo, hi);
    out[6] = clampi(r5 + r7, lo, hi);
    const int s6 = clampi(r4 - r6, lo, hi), s7 = clampi(r5 - r7, lo, hi);
    out[3] = -A::h181(s2 + s3);
    out[4] = A::h181(s2 - s3);
    out[2] = A::h181(s6 + s7);
    out[5] = -A::h181(s6 - s7);
}

template <bool W>
__device__ __forceinline__ void iadst16(const int *x, int *out, int lo, int hi) {
    using A = Ar<W>;
    int p[16];
    p[0] = A::r12(x[15], 4091, x[0], 201);   p[1] = A::r12(x[15], 201, x[0], -4091);
    p[2] = A::r12(x[13], 3973, x[2], 995);   p[3] = A::r12(x[13], 995, x[2], -3973);
    p[4] = A::r12(x[11], 3703, x[4], 1751);  p[5] = A::r12(x[11], 1751, x[4], -3703);
    p[6] = A::r12(x[9], 3290, x[6], 2440);   p[7] = A::r12(x[9], 2440, x[6], -3290);
    p[8] = A::r12(x[7], 2751, x[8], 3035);   p[9] = A::r12(x[7], 3035, x[8], -2751);
    p[10] = A::r12(x[5], 2106, x[10], 3513); p[11] = A::r12(x[5], 3513, x[10], -2106);
    p[12] = A::r12(x[3], 1380, x[12], 3857); p[13] = A::r12(x[3], 3857, x[12], -1380);
    p[14] = A::r12(x[1], 601, x[14], 4052);  p[15] = A::r12(x[1], 4052, x[14], -601);
    int q[16];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        q[k] = clampi(p[k] + p[k + 8], lo, hi);
        q[k + 8] = clampi(p[k] - p[k + 8], lo, hi);
    }
    const int r8 = A::r12(q[8], 4017, q[9], 799), r9 = A::r12(q[8], 799, q[9], -4017);
    const int r10 = A::r12(q[10], 2276, q[11], 3406), r11 = A::r12(q[10], 3406, q[11], -2276);
    const int r12_ = A::r12(q[13], 4017, q[12], -799), r13 = A::r12(q[13], 799, q[12], 4017);
    const int r14 = A::r12(q[15], 2276, q[14], -3406), r15 = A::r12(q[15], 3406, q[14], 2276);
    const int s0 = clampi(q[0] + q[4], lo, hi), s4 = clampi(q[0] - q[4], lo, hi);
    const int s1 = clampi(q[1] + q[5], lo, hi), s5 = clampi(q[1] - q[5], lo, hi);
    const int s2 = clampi(q[2] + q[6], lo, hi), s6 = clampi(q[2] - q[6], lo, hi);
    const int s3 = clampi(q[3] + q[7], lo, hi), s7 = clampi(q[3] - q[7], lo, hi);
    const int s8 = clampi(r8 + r12_, lo, hi), s12 = clampi(r8 - r12_, lo, hi);
    const int s9 = clampi(r9 + r13, lo, hi), s13 = clampi(r9 - r13, lo, hi);
    const int s10 = clampi(r10 + r14, lo, hi), s14 = clampi(r10 - r14, lo, hi);
    const int s11 = clampi(r11 + r15, lo, hi), s15 = clampi(r11 - r15, lo, hi);
    const int u4 = A::r12(s4, 3784, s5, 1567), u5 = A::r12(s4, 1567, s5, -3784);
    const int u6 = A::r12(s7, 3784, s6, -1567), u7 = A::r12(s7, 1567, s6, 3784);
    const int u12 = A::r12(s12, 3784, s13, 1567), u13 = A::r12(s12, 1567, s13, -3784);
    const int u14 = A::r12(s15, 3784, s14, -1567), u15 = A::r12(s15, 1567, s14, 3784);
    out[0] = clampi(s0 + s2, lo, hi);
    out[15] = -clampi(s1 + s3, lo, hi);
    const int v2 = clampi(s0 - s2, lo, hi), v3 = clampi(s1 - s3, lo, hi);
    out[3] = -clampi(u4 + u6, lo, hi);
    out[12] = clampi(u5 + u7, lo, hi);
    const int v6 = clampi(u4 - u6, lo, hi), v7 = clampi(u5 - u7, lo, hi);
    out[1] = -clampi(s8 + s10, lo, hi);
    out[14] = clampi(s9 + s11, lo, hi);
    const int v10 = clampi(s8 - s10, lo, hi), v11 = clampi(s9 - s11, lo, hi);
    out[2] = clampi(u12 + u14, lo, hi);
    out[13] = -clampi(u13 + u15, lo, hi);
    const int v14 = clampi(u12 - u14, lo, hi), v15 = clampi(u13 - u15, lo, hi);
    out[7] = -A::h181(v2 + v3);
    out[8] = A::h181(v2 - v3);
    out[4] = A::h181(v6 + v7);
    out[11] = -A::h181(v6 - v7);
    out[6] = A::h181(v10 + v11);
    out[9] = -A::h181(v10 - v11);
    out[5] = -A::h181(v14 + v15);
    out[10] = A::h181(v14 - v15);
}

#undef E

enum Kind1d { KD = 0, KA = 1, KF = 2, KI = 3 };

// Apply a 1-D transform of kind `k` and length N to the contiguous register array c[N].
// `k` is uniform for the lanes of one transform block, not necessarily for the wave.
template <bool W, int N>
__device__ __forceinline__ void itx1d(int k, int *c, int lo, int hi) {
    if (k == KD) {
        if constexpr (N == 4) idct4<W, 1>(c, lo, hi, false);
        else if constexpr (N == 8) idct8<W, 1>(c, lo, hi, false);
        else if constexpr (N == 16) idct16<W, 1>(c, lo, hi, false);
        else if constexpr (N == 32) idct32<W, 1>(c, lo, hi, false);
        else idct64<W, 1>(c, lo, hi);
    } else if (k == KI) {
#pragma unroll
        for (int i = 0; i < N; i++) {
            const int v = c[i];
            if constexpr (N == 4) c[i] = v + Ar<W>::s12(v, 1697);
            else if constexpr (N == 8) c[i] = v * 2;
            else if constexpr (N == 16) {
                if constexpr (W) c[i] = 2 * v + (int)(((int64_t)v * 1697 + 1024) >> 11);
                else c[i] = 2 * v + ((v * 1697 + 1024) >> 11);
            } else c[i] = v * 4;
        }
    } else {
        if constexpr (N <= 16) {
            int o[N];
            if constexpr (N == 4) iadst4<W>(c, o);
            else if constexpr (N == 8) iadst8<W>(c, o, lo, hi);
            else iadst16<W>(c, o, lo, hi);
            if (k == KF) {
#pragma unroll
                for (int i = 0; i < N; i++) c[i] = o[N - 1 - i];
            } else {
#pragma unroll
                for (int i = 0; i < N; i++) c[i] = o[i];
            }
        }
    }
}

__device__ __forceinline__ void iwht4(int *c) {
    const int a = c[0] + c[1], b = c[2] - c[3];
    const int m = (a - b) >> 1;
    const int d = m - c[3], e = m - c[1];
    c[0] = a - d;
    c[1] = d;
    c[2] = e;
    c[3] = b + e;
}

} // namespace mi
