/*
 * oracle/itx.c — CPU restatement of the inverse-transform DSP (TEST INFRASTRUCTURE ONLY).
 *
 * Follows FreezyLemon/rav1d:
 *   src/itx.rs:64-188     inv_txfm_add_rust (2-D driver; C twin src/itx_tmpl.c:40-100)
 *   src/itx.rs:475-526    inv_txfm_add_wht_wht_4x4_rust (C src/itx_tmpl.c:162-181)
 *   src/itx.rs:400-457    table fill / per-size shift (C src/itx_tmpl.c:142-160, 191-254)
 *   src/itx_1d.rs:5-1140  1-D kernels (C src/itx_1d.c:66-1034)
 *
 * Arithmetic note. The reference writes each rotation as e.g.
 *   ((a*1567 - b*(3784-4096) + 2048) >> 12) - b
 * which is, for every input, exactly floor((a*1567 - b*3784 + 2048) / 4096) (the 4096*b
 * term is a multiple of 4096) — the form only exists to keep 12-bit streams inside 32 bits
 * (comment at src/itx_1d.c:38-64). Likewise (x*1703 + y*1138 + 1024) >> 11 equals
 * (x*3406 + y*2276 + 2048) >> 12 and ((x)*181 + 128) >> 8 equals (x*2896 + 2048) >> 12.
 * This restatement evaluates every rotation in 64-bit, so it computes the same exact
 * values for any input without the rewrite. CLIP points, rounding points and output
 * negations are kept exactly where the reference has them.
 */
#include <stdint.h>
#include <string.h>
#include "oracle.h"

typedef int64_t i64;

/* rounded rotation term: (a*ca + b*cb + 2048) >> 12, exact in 64-bit */
#define R12(a, ca, b, cb) ((int)(((i64)(a) * (ca) + (i64)(b) * (cb) + 2048) >> 12))
/* single-input scale by c/4096 with rounding */
#define S12(a, ca) ((int)(((i64)(a) * (ca) + 2048) >> 12))
/* (x * 181 + 128) >> 8 : multiply by 1/sqrt(2) */
#define H181(x) ((int)(((i64)(x) * 181 + 128) >> 8))

static inline int clipi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
#define CL(x) clipi((x), lo, hi)

/* ---------------- DCT (itx_1d.rs dct4..dct64; itx_1d.c:66-781) ---------------- */
/* `half` mirrors the reference's tx64 flag: only the first half of the inputs is nonzero. */

static void dct4(int32_t *c, ptrdiff_t s, int lo, int hi, int half)
{
    int a0, a1, a2, a3;
    if (half) {
        a0 = a1 = H181(c[0]);
        a2 = S12(c[s], 1567);
        a3 = S12(c[s], 3784);
    } else {
        const int x0 = c[0], x1 = c[s], x2 = c[2 * s], x3 = c[3 * s];
        a0 = H181(x0 + x2);
        a1 = H181(x0 - x2);
        a2 = R12(x1, 1567, x3, -3784);
        a3 = R12(x1, 3784, x3, 1567);
    }
    c[0] = CL(a0 + a3);
    c[s] = CL(a1 + a2);
    c[2 * s] = CL(a1 - a2);
    c[3 * s] = CL(a0 - a3);
}

static void dct8(int32_t *c, ptrdiff_t s, int lo, int hi, int half)
{
    dct4(c, 2 * s, lo, hi, half);
    int p4, p5, p6, p7;
    const int x1 = c[s], x3 = c[3 * s];
    if (half) {
        p4 = S12(x1, 799);
        p5 = S12(x3, -2276);
        p6 = S12(x3, 3406);
        p7 = S12(x1, 4017);
    } else {
        const int x5 = c[5 * s], x7 = c[7 * s];
        p4 = R12(x1, 799, x7, -4017);
        p5 = R12(x5, 3406, x3, -2276);
        p6 = R12(x5, 2276, x3, 3406);
        p7 = R12(x1, 4017, x7, 799);
    }
    const int q4 = CL(p4 + p5), q5 = CL(p4 - p5);
    const int q7 = CL(p7 + p6), q6 = CL(p7 - p6);
    const int r5 = H181(q6 - q5), r6 = H181(q6 + q5);
    const int e0 = c[0], e1 = c[2 * s], e2 = c[4 * s], e3 = c[6 * s];
    c[0] = CL(e0 + q7);
    c[s] = CL(e1 + r6);
    c[2 * s] = CL(e2 + r5);
    c[3 * s] = CL(e3 + q4);
    c[4 * s] = CL(e3 - q4);
    c[5 * s] = CL(e2 - r5);
    c[6 * s] = CL(e1 - r6);
    c[7 * s] = CL(e0 - q7);
}

static void dct16(int32_t *c, ptrdiff_t s, int lo, int hi, int half)
{
    dct8(c, 2 * s, lo, hi, half);
    const int x1 = c[s], x3 = c[3 * s], x5 = c[5 * s], x7 = c[7 * s];
    int a8, a9, a10, a11, a12, a13, a14, a15;
    if (half) {
        a8 = S12(x1, 401);   a9 = S12(x7, -2598);
        a10 = S12(x5, 1931); a11 = S12(x3, -1189);
        a12 = S12(x3, 3920); a13 = S12(x5, 3612);
        a14 = S12(x7, 3166); a15 = S12(x1, 4076);
    } else {
        const int x9 = c[9 * s], x11 = c[11 * s], x13 = c[13 * s], x15 = c[15 * s];
        a8 = R12(x1, 401, x15, -4076);
        a9 = R12(x9, 3166, x7, -2598);
        a10 = R12(x5, 1931, x11, -3612);
        a11 = R12(x13, 3920, x3, -1189);
        a12 = R12(x13, 1189, x3, 3920);
        a13 = R12(x5, 3612, x11, 1931);
        a14 = R12(x9, 2598, x7, 3166);
        a15 = R12(x1, 4076, x15, 401);
    }
    int b8 = CL(a8 + a9), b9 = CL(a8 - a9), b10 = CL(a11 - a10), b11 = CL(a11 + a10);
    int b12 = CL(a12 + a13), b13 = CL(a12 - a13), b14 = CL(a15 - a14), b15 = CL(a15 + a14);

    const int c9 = R12(b14, 1567, b9, -3784);
    const int c14 = R12(b14, 3784, b9, 1567);
    const int c10 = R12(b13, -3784, b10, -1567);
    const int c13 = R12(b13, 1567, b10, -3784);

    const int d8 = CL(b8 + b11), d9 = CL(c9 + c10), d10 = CL(c9 - c10), d11 = CL(b8 - b11);
    const int d12 = CL(b15 - b12), d13 = CL(c14 - c13), d14 = CL(c14 + c13), d15 = CL(b15 + b12);

    const int f10 = H181(d13 - d10), f13 = H181(d13 + d10);
    const int f11 = H181(d12 - d11), f12 = H181(d12 + d11);

    const int o[8] = { d8, d9, f10, f11, f12, f13, d14, d15 };
    int e[8];
    for (int i = 0; i < 8; i++) e[i] = c[2 * i * s];
    for (int i = 0; i < 8; i++) {
        c[i * s] = CL(e[i] + o[7 - i]);
        c[(15 - i) * s] = CL(e[i] - o[7 - i]);
    }
}

static void dct32(int32_t *c, ptrdiff_t s, int lo, int hi, int half)
{
    dct16(c, 2 * s, lo, hi, half);
    int x[32];
    for (int i = 1; i < 32; i += 2) x[i] = (half && i > 15) ? 0 : c[i * s];
    int a[32]; /* a[16..31] = t16a..t31a */
    if (half) {
        a[16] = S12(x[1], 201);   a[17] = S12(x[15], -2751);
        a[18] = S12(x[9], 1751);  a[19] = S12(x[7], -1380);
        a[20] = S12(x[5], 995);   a[21] = S12(x[11], -2106);
        a[22] = S12(x[13], 2440); a[23] = S12(x[3], -601);
        a[24] = S12(x[3], 4052);  a[25] = S12(x[13], 3290);
        a[26] = S12(x[11], 3513); a[27] = S12(x[5], 3973);
        a[28] = S12(x[7], 3857);  a[29] = S12(x[9], 3703);
        a[30] = S12(x[15], 3035); a[31] = S12(x[1], 4091);
    } else {
        a[16] = R12(x[1], 201, x[31], -4091);
        a[17] = R12(x[17], 3035, x[15], -2751);
        a[18] = R12(x[9], 1751, x[23], -3703);
        a[19] = R12(x[25], 3857, x[7], -1380);
        a[20] = R12(x[5], 995, x[27], -3973);
        a[21] = R12(x[21], 3513, x[11], -2106);
        a[22] = R12(x[13], 2440, x[19], -3290);
        a[23] = R12(x[29], 4052, x[3], -601);
        a[24] = R12(x[29], 601, x[3], 4052);
        a[25] = R12(x[13], 3290, x[19], 2440);
        a[26] = R12(x[21], 2106, x[11], 3513);
        a[27] = R12(x[5], 3973, x[27], 995);
        a[28] = R12(x[25], 1380, x[7], 3857);
        a[29] = R12(x[9], 3703, x[23], 1751);
        a[30] = R12(x[17], 2751, x[15], 3035);
        a[31] = R12(x[1], 4091, x[31], 201);
    }
    /* stage 1 butterflies */
    int b16 = CL(a[16] + a[17]), b17 = CL(a[16] - a[17]);
    int b18 = CL(a[19] - a[18]), b19 = CL(a[19] + a[18]);
    int b20 = CL(a[20] + a[21]), b21 = CL(a[20] - a[21]);
    int b22 = CL(a[23] - a[22]), b23 = CL(a[23] + a[22]);
    int b24 = CL(a[24] + a[25]), b25 = CL(a[24] - a[25]);
    int b26 = CL(a[27] - a[26]), b27 = CL(a[27] + a[26]);
    int b28 = CL(a[28] + a[29]), b29 = CL(a[28] - a[29]);
    int b30 = CL(a[31] - a[30]), b31 = CL(a[31] + a[30]);
    /* rotations */
    int r17 = R12(b30, 799, b17, -4017);
    int r30 = R12(b30, 4017, b17, 799);
    int r18 = R12(b29, -4017, b18, -799);
    int r29 = R12(b29, 799, b18, -4017);
    int r21 = R12(b26, 3406, b21, -2276);
    int r26 = R12(b26, 2276, b21, 3406);
    int r22 = R12(b25, -2276, b22, -3406);
    int r25 = R12(b25, 3406, b22, -2276);
    /* stage 2 butterflies */
    int c16 = CL(b16 + b19), c17 = CL(r17 + r18), c18 = CL(r17 - r18), c19 = CL(b16 - b19);
    int c20 = CL(b23 - b20), c21 = CL(r22 - r21), c22 = CL(r22 + r21), c23 = CL(b23 + b20);
    int c24 = CL(b24 + b27), c25 = CL(r25 + r26), c26 = CL(r25 - r26), c27 = CL(b24 - b27);
    int c28 = CL(b31 - b28), c29 = CL(r30 - r29), c30 = CL(r30 + r29), c31 = CL(b31 + b28);
    /* rotations */
    int s18 = R12(c29, 1567, c18, -3784);
    int s29 = R12(c29, 3784, c18, 1567);
    int s19 = R12(c28, 1567, c19, -3784);
    int s28 = R12(c28, 3784, c19, 1567);
    int s20 = R12(c27, -3784, c20, -1567);
    int s27 = R12(c27, 1567, c20, -3784);
    int s21 = R12(c26, -3784, c21, -1567);
    int s26 = R12(c26, 1567, c21, -3784);
    /* stage 3 butterflies */
    int d16 = CL(c16 + c23), d17 = CL(c17 + c22), d18 = CL(s18 + s21), d19 = CL(s19 + s20);
    int d20 = CL(s19 - s20), d21 = CL(s18 - s21), d22 = CL(c17 - c22), d23 = CL(c16 - c23);
    int d24 = CL(c31 - c24), d25 = CL(c30 - c25), d26 = CL(s29 - s26), d27 = CL(s28 - s27);
    int d28 = CL(s28 + s27), d29 = CL(s29 + s26), d30 = CL(c30 + c25), d31 = CL(c31 + c24);
    /* 1/sqrt2 */
    int f20 = H181(d27 - d20), f27 = H181(d27 + d20);
    int f21 = H181(d26 - d21), f26 = H181(d26 + d21);
    int f22 = H181(d25 - d22), f25 = H181(d25 + d22);
    int f23 = H181(d24 - d23), f24 = H181(d24 + d23);

    const int o[16] = { d16, d17, d18, d19, f20, f21, f22, f23,
                        f24, f25, f26, f27, d28, d29, d30, d31 };
    int e[16];
    for (int i = 0; i < 16; i++) e[i] = c[2 * i * s];
    for (int i = 0; i < 16; i++) {
        c[i * s] = CL(e[i] + o[15 - i]);
        c[(31 - i) * s] = CL(e[i] - o[15 - i]);
    }
}

/* dct64: only the first 32 inputs are read (itx_1d.c:436-781, itx_1d.rs:426-773). */
static void dct64(int32_t *c, ptrdiff_t s, int lo, int hi)
{
    dct32(c, 2 * s, lo, hi, 1);
    int x[32];
    for (int i = 1; i < 32; i += 2) x[i] = c[i * s];
    int a[64];
    static const struct { int in, k; } init[32] = {
        { 1, 101 },  { 31, -2824 }, { 17, 1660 }, { 15, -1474 },
        { 9, 897 },  { 23, -2191 }, { 25, 2359 }, { 7, -700 },
        { 5, 501 },  { 27, -2520 }, { 21, 2019 }, { 11, -1092 },
        { 13, 1285 }, { 19, -1842 }, { 29, 2675 }, { 3, -301 },
        { 3, 4085 }, { 29, 3102 },  { 19, 3659 }, { 13, 3889 },
        { 11, 3948 }, { 21, 3564 }, { 27, 3229 }, { 5, 4065 },
        { 7, 4036 }, { 25, 3349 },  { 23, 3461 }, { 9, 3996 },
        { 15, 3822 }, { 17, 3745 }, { 31, 2967 }, { 1, 4095 },
    };
    for (int i = 0; i < 32; i++) a[32 + i] = S12(x[init[i].in], init[i].k);

    int t[64];
    /* stage 1: butterflies in groups of 4: (+,-) then (-,+) patterns */
    for (int g = 32; g < 64; g += 4) {
        t[g + 0] = CL(a[g + 0] + a[g + 1]);
        t[g + 1] = CL(a[g + 0] - a[g + 1]);
        t[g + 2] = CL(a[g + 3] - a[g + 2]);
        t[g + 3] = CL(a[g + 3] + a[g + 2]);
    }
    /* stage 1 rotations (itx_1d.c:509-524) */
    int u[64];
    memcpy(u, t, sizeof(u));
    u[33] = R12(t[33], -4076, t[62], 401);
    u[34] = R12(t[34], -401, t[61], -4076);
    u[37] = R12(t[37], -2598, t[58], 3166);
    u[38] = R12(t[38], -3166, t[57], -2598);
    u[41] = R12(t[41], -3612, t[54], 1931);
    u[42] = R12(t[42], -1931, t[53], -3612);
    u[45] = R12(t[45], -1189, t[50], 3920);
    u[46] = R12(t[46], -3920, t[49], -1189);
    u[49] = R12(t[46], -1189, t[49], 3920);
    u[50] = R12(t[45], 3920, t[50], 1189);
    u[53] = R12(t[42], -3612, t[53], 1931);
    u[54] = R12(t[41], 1931, t[54], 3612);
    u[57] = R12(t[38], -2598, t[57], 3166);
    u[58] = R12(t[37], 3166, t[58], 2598);
    u[61] = R12(t[34], -4076, t[61], 401);
    u[62] = R12(t[33], 401, t[62], 4076);
    /* stage 2 butterflies (itx_1d.c:526-557) */
    int v[64];
    for (int g = 32; g < 64; g += 8) {
        v[g + 0] = CL(u[g + 0] + u[g + 3]);
        v[g + 1] = CL(u[g + 1] + u[g + 2]);
        v[g + 2] = CL(u[g + 1] - u[g + 2]);
        v[g + 3] = CL(u[g + 0] - u[g + 3]);
        v[g + 4] = CL(u[g + 7] - u[g + 4]);
        v[g + 5] = CL(u[g + 6] - u[g + 5]);
        v[g + 6] = CL(u[g + 6] + u[g + 5]);
        v[g + 7] = CL(u[g + 7] + u[g + 4]);
    }
    /* stage 2 rotations (itx_1d.c:559-574) */
    int w[64];
    memcpy(w, v, sizeof(w));
    w[34] = R12(v[34], -4017, v[61], 799);
    w[35] = R12(v[35], -4017, v[60], 799);
    w[36] = R12(v[36], -799, v[59], -4017);
    w[37] = R12(v[37], -799, v[58], -4017);
    w[42] = R12(v[42], -2276, v[53], 3406);
    w[43] = R12(v[43], -2276, v[52], 3406);
    w[44] = R12(v[44], -3406, v[51], -2276);
    w[45] = R12(v[45], -3406, v[50], -2276);
    w[50] = R12(v[45], -2276, v[50], 3406);
    w[51] = R12(v[44], -2276, v[51], 3406);
    w[52] = R12(v[43], 3406, v[52], 2276);
    w[53] = R12(v[42], 3406, v[53], 2276);
    w[58] = R12(v[37], -4017, v[58], 799);
    w[59] = R12(v[36], -4017, v[59], 799);
    w[60] = R12(v[35], 799, v[60], 4017);
    w[61] = R12(v[34], 799, v[61], 4017);
    /* stage 3 butterflies (itx_1d.c:576-607) */
    int y[64];
    for (int g = 32; g < 64; g += 16) {
        for (int k = 0; k < 4; k++) {
            y[g + k] = CL(w[g + k] + w[g + 7 - k]);
            y[g + 7 - k] = CL(w[g + k] - w[g + 7 - k]);
            y[g + 8 + k] = CL(w[g + 15 - k] - w[g + 8 + k]);
            y[g + 15 - k] = CL(w[g + 15 - k] + w[g + 8 + k]);
        }
    }
    /* stage 3 rotations (itx_1d.c:609-624) */
    int z[64];
    memcpy(z, y, sizeof(z));
    for (int k = 0; k < 4; k++) {
        const int lo_i = 36 + k, hi_i = 59 - k;   /* (36,59) (37,58) (38,57) (39,56) */
        z[lo_i] = R12(y[lo_i], -3784, y[hi_i], 1567);
        z[hi_i] = R12(y[lo_i], 1567, y[hi_i], 3784);
        const int lo_j = 40 + k, hi_j = 55 - k;   /* (40,55) (41,54) (42,53) (43,52) */
        z[lo_j] = R12(y[lo_j], -1567, y[hi_j], -3784);
        z[hi_j] = R12(y[lo_j], -3784, y[hi_j], 1567);
    }
    /* stage 4 butterflies (itx_1d.c:626-657) */
    int q[64];
    for (int k = 0; k < 8; k++) {
        q[32 + k] = CL(z[32 + k] + z[47 - k]);
        q[47 - k] = CL(z[32 + k] - z[47 - k]);
        q[48 + k] = CL(z[63 - k] - z[48 + k]);
        q[63 - k] = CL(z[63 - k] + z[48 + k]);
    }
    /* 1/sqrt2 stage (itx_1d.c:659-674) */
    for (int k = 0; k < 8; k++) {
        const int l = 40 + k, h = 55 - k;
        const int ql = q[l], qh = q[h];
        q[l] = H181(qh - ql);
        q[h] = H181(qh + ql);
    }
    int e[32];
    for (int i = 0; i < 32; i++) e[i] = c[2 * i * s];
    for (int i = 0; i < 32; i++) {
        c[i * s] = CL(e[i] + q[63 - i]);
        c[(63 - i) * s] = CL(e[i] - q[63 - i]);
    }
}

/* ---------------- ADST (itx_1d.rs:774-1044; itx_1d.c:783-1002) ---------------- */

static void adst4(const int32_t *in, ptrdiff_t is, int32_t *out, ptrdiff_t os)
{
    const i64 x0 = in[0], x1 = in[is], x2 = in[2 * is], x3 = in[3 * is];
    out[0] = (int)((1321 * x0 + 3803 * x2 + 2482 * x3 + 3344 * x1 + 2048) >> 12);
    out[os] = (int)((2482 * x0 - 1321 * x2 - 3803 * x3 + 3344 * x1 + 2048) >> 12);
    out[2 * os] = (int)((209 * (x0 - x2 + x3) + 128) >> 8);
    out[3 * os] = (int)((3803 * x0 + 2482 * x2 - 1321 * x3 - 3344 * x1 + 2048) >> 12);
}

static void adst8(const int32_t *in, ptrdiff_t is, int32_t *out, ptrdiff_t os, int lo, int hi)
{
    int x[8];
    for (int i = 0; i < 8; i++) x[i] = in[i * is];
    const int a0 = R12(x[7], 4076, x[0], 401);
    const int a1 = R12(x[7], 401, x[0], -4076);
    const int a2 = R12(x[5], 3612, x[2], 1931);
    const int a3 = R12(x[5], 1931, x[2], -3612);
    const int a4 = R12(x[3], 2598, x[4], 3166);
    const int a5 = R12(x[3], 3166, x[4], -2598);
    const int a6 = R12(x[1], 1189, x[6], 3920);
    const int a7 = R12(x[1], 3920, x[6], -1189);

    const int b0 = CL(a0 + a4), b1 = CL(a1 + a5), b2 = CL(a2 + a6), b3 = CL(a3 + a7);
    const int b4 = CL(a0 - a4), b5 = CL(a1 - a5), b6 = CL(a2 - a6), b7 = CL(a3 - a7);

    const int r4 = R12(b4, 3784, b5, 1567);
    const int r5 = R12(b4, 1567, b5, -3784);
    const int r6 = R12(b7, 3784, b6, -1567);
    const int r7 = R12(b7, 1567, b6, 3784);

    out[0] = CL(b0 + b2);
    out[7 * os] = -CL(b1 + b3);
    const int d2 = CL(b0 - b2), d3 = CL(b1 - b3);
    out[os] = -CL(r4 + r6);
    out[6 * os] = CL(r5 + r7);
    const int d6 = CL(r4 - r6), d7 = CL(r5 - r7);
    out[3 * os] = -H181(d2 + d3);
    out[4 * os] = H181(d2 - d3);
    out[2 * os] = H181(d6 + d7);
    out[5 * os] = -H181(d6 - d7);
}

static void adst16(const int32_t *in, ptrdiff_t is, int32_t *out, ptrdiff_t os, int lo, int hi)
{
    int x[16];
    for (int i = 0; i < 16; i++) x[i] = in[i * is];
    /* input rotations: pairs (hi input, lo input) with angle constants */
    static const struct { int a, b, c0, c1; } rot[8] = {
        /* t[2k]   = R(x[a]*c0 + x[b]*c1),  t[2k+1] = R(x[a]*c1 - x[b]*c0) */
        { 15, 0, 4091, 201 }, { 13, 2, 3973, 995 }, { 11, 4, 3703, 1751 }, { 9, 6, 3290, 2440 },
        { 7, 8, 2751, 3035 }, { 5, 10, 2106, 3513 }, { 3, 12, 1380, 3857 }, { 1, 14, 601, 4052 },
    };
    int t[16];
    for (int k = 0; k < 8; k++) {
        t[2 * k] = R12(x[rot[k].a], rot[k].c0, x[rot[k].b], rot[k].c1);
        t[2 * k + 1] = R12(x[rot[k].a], rot[k].c1, x[rot[k].b], -rot[k].c0);
    }
    int u[16];
    for (int k = 0; k < 8; k++) {
        u[k] = CL(t[k] + t[k + 8]);
        u[k + 8] = CL(t[k] - t[k + 8]);
    }
    /* rotations of the odd half (itx_1d.c:929-936) */
    const int v8 = R12(u[8], 4017, u[9], 799);
    const int v9 = R12(u[8], 799, u[9], -4017);
    const int v10 = R12(u[10], 2276, u[11], 3406);
    const int v11 = R12(u[10], 3406, u[11], -2276);
    const int v12 = R12(u[13], 4017, u[12], -799);
    const int v13 = R12(u[13], 799, u[12], 4017);
    const int v14 = R12(u[15], 2276, u[14], -3406);
    const int v15 = R12(u[15], 3406, u[14], 2276);

    const int w0 = CL(u[0] + u[4]), w1 = CL(u[1] + u[5]), w2 = CL(u[2] + u[6]), w3 = CL(u[3] + u[7]);
    const int w4 = CL(u[0] - u[4]), w5 = CL(u[1] - u[5]), w6 = CL(u[2] - u[6]), w7 = CL(u[3] - u[7]);
    const int w8 = CL(v8 + v12), w9 = CL(v9 + v13), w10 = CL(v10 + v14), w11 = CL(v11 + v15);
    const int w12 = CL(v8 - v12), w13 = CL(v9 - v13), w14 = CL(v10 - v14), w15 = CL(v11 - v15);

    const int y4 = R12(w4, 3784, w5, 1567);
    const int y5 = R12(w4, 1567, w5, -3784);
    const int y6 = R12(w7, 3784, w6, -1567);
    const int y7 = R12(w7, 1567, w6, 3784);
    const int y12 = R12(w12, 3784, w13, 1567);
    const int y13 = R12(w12, 1567, w13, -3784);
    const int y14 = R12(w15, 3784, w14, -1567);
    const int y15 = R12(w15, 1567, w14, 3784);

    out[0] = CL(w0 + w2);
    out[15 * os] = -CL(w1 + w3);
    const int z2 = CL(w0 - w2), z3 = CL(w1 - w3);
    out[3 * os] = -CL(y4 + y6);
    out[12 * os] = CL(y5 + y7);
    const int z6 = CL(y4 - y6), z7 = CL(y5 - y7);
    out[os] = -CL(w8 + w10);
    out[14 * os] = CL(w9 + w11);
    const int z10 = CL(w8 - w10), z11 = CL(w9 - w11);
    out[2 * os] = CL(y12 + y14);
    out[13 * os] = -CL(y13 + y15);
    const int z14 = CL(y12 - y14), z15 = CL(y13 - y15);

    out[7 * os] = -H181(z2 + z3);
    out[8 * os] = H181(z2 - z3);
    out[4 * os] = H181(z6 + z7);
    out[11 * os] = -H181(z6 - z7);
    out[6 * os] = H181(z10 + z11);
    out[9 * os] = -H181(z10 - z11);
    out[5 * os] = -H181(z14 + z15);
    out[10 * os] = H181(z14 - z15);
}

/* ---------------- identity / WHT (itx_1d.rs:1055-1140; itx_1d.c:1004-1034) ---------------- */

static void identity(int32_t *c, ptrdiff_t s, int n)
{
    for (int i = 0; i < n; i++) {
        const i64 v = c[i * s];
        switch (n) {
        case 4:  c[i * s] = (int)(v + ((v * 1697 + 2048) >> 12)); break;
        case 8:  c[i * s] = (int)(v * 2); break;
        case 16: c[i * s] = (int)(2 * v + ((v * 1697 + 1024) >> 11)); break;
        default: c[i * s] = (int)(v * 4); break;
        }
    }
}

static void wht4(int32_t *c, ptrdiff_t s)
{
    const int x0 = c[0], x1 = c[s], x2 = c[2 * s], x3 = c[3 * s];
    const int a = x0 + x1, b = x2 - x3;
    const int m = (a - b) >> 1;
    const int d = m - x3, e = m - x1;
    c[0] = a - d;
    c[s] = d;
    c[2 * s] = e;
    c[3 * s] = b + e;
}

enum { K_DCT, K_ADST, K_FLIPADST, K_IDENTITY, K_WHT };

void oracle_itx_1d(int kind, int n, int32_t *c, ptrdiff_t s, int lo, int hi)
{
    int32_t tmp[16];
    switch (kind) {
    case K_DCT:
        if (n == 4) dct4(c, s, lo, hi, 0);
        else if (n == 8) dct8(c, s, lo, hi, 0);
        else if (n == 16) dct16(c, s, lo, hi, 0);
        else if (n == 32) dct32(c, s, lo, hi, 0);
        else dct64(c, s, lo, hi);
        break;
    case K_ADST:
    case K_FLIPADST: {
        /* flipadst = adst writing its outputs in reverse order (itx_1d.c:985-1000) */
        int32_t *out = kind == K_ADST ? c : c + (n - 1) * s;
        const ptrdiff_t os = kind == K_ADST ? s : -s;
        if (n == 4) adst4(c, s, out, os);
        else if (n == 8) adst8(c, s, out, os, lo, hi);
        else adst16(c, s, out, os, lo, hi);
        (void)tmp;
        break;
    }
    case K_IDENTITY: identity(c, s, n); break;
    default: wht4(c, s); break;
    }
}

/* ---------------- 2-D driver ---------------- */

/* RectTxfmSize -> (w, h) in pixels, src/levels.rs:46-82; per-size shift, itx.rs:439-457 */
static const uint8_t tx_w[19] = { 4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64 };
static const uint8_t tx_h[19] = { 4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16 };
static const uint8_t tx_shift[19] = { 0, 1, 2, 2, 2, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2 };

/* TxfmType -> (vertical kind, horizontal kind); naming is VERT_HORZ (levels.rs TxfmType,
 * mapping to row/column functions at itx_tmpl.c:196-233 / itx.rs:1012-1031). */
static const uint8_t ty_col[16] = { K_DCT, K_ADST, K_DCT, K_ADST, K_FLIPADST, K_DCT, K_FLIPADST,
                                    K_ADST, K_FLIPADST, K_IDENTITY, K_DCT, K_IDENTITY, K_ADST,
                                    K_IDENTITY, K_FLIPADST, K_IDENTITY };
static const uint8_t ty_row[16] = { K_DCT, K_DCT, K_ADST, K_ADST, K_DCT, K_FLIPADST, K_FLIPADST,
                                    K_FLIPADST, K_ADST, K_IDENTITY, K_IDENTITY, K_DCT, K_IDENTITY,
                                    K_ADST, K_IDENTITY, K_FLIPADST };

static inline int clip_px(int v, int bdmax) { return v < 0 ? 0 : v > bdmax ? bdmax : v; }

void oracle_itxfm_add(int tx, int txtp, void *dst_, ptrdiff_t stride, void *coeff_,
                      int eob, int bdmax)
{
    const int hbd = bdmax > 255;
    uint8_t *dst8 = dst_;
    uint16_t *dst16 = dst_;
    int16_t *cf16 = coeff_;
    int32_t *cf32 = coeff_;
    const ptrdiff_t ps = hbd ? stride / 2 : stride;
#define PX(x, y) (hbd ? dst16[(y) * ps + (x)] : dst8[(y) * ps + (x)])
#define SETPX(x, y, v) do { if (hbd) dst16[(y) * ps + (x)] = (uint16_t)(v); \
                            else dst8[(y) * ps + (x)] = (uint8_t)(v); } while (0)
#define CF(i) (hbd ? cf32[i] : (int)cf16[i])

    if (txtp == 16) {
        /* lossless WHT, itx_tmpl.c:162-181 / itx.rs:475-526 */
        int32_t t[16];
        for (int y = 0; y < 4; y++) {
            for (int x = 0; x < 4; x++) t[y * 4 + x] = CF(y + x * 4) >> 2;
            wht4(&t[y * 4], 1);
        }
        if (hbd) memset(cf32, 0, 16 * 4); else memset(cf16, 0, 16 * 2);
        for (int x = 0; x < 4; x++) wht4(&t[x], 4);
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) SETPX(x, y, clip_px(PX(x, y) + t[y * 4 + x], bdmax));
        return;
    }

    const int w = tx_w[tx], h = tx_h[tx], shift = tx_shift[tx];
    const int rect2 = (w == 2 * h) || (h == 2 * w);
    const int rnd = (1 << shift) >> 1;
    const int dconly = txtp == 0; /* has_dconly: DCT_DCT only */

    if (eob < dconly) {
        int dc = CF(0);
        if (hbd) cf32[0] = 0; else cf16[0] = 0;
        if (rect2) dc = (dc * 181 + 128) >> 8;
        dc = (dc * 181 + 128) >> 8;
        dc = (dc + rnd) >> shift;
        dc = (dc * 181 + 128 + 2048) >> 12;
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) SETPX(x, y, clip_px(PX(x, y) + dc, bdmax));
        return;
    }

    const int sh = h < 32 ? h : 32, sw = w < 32 ? w : 32;
    int row_lo, col_lo;
    if (!hbd) { row_lo = INT16_MIN; col_lo = INT16_MIN; }
    else { row_lo = (int)((unsigned)~bdmax << 7); col_lo = (int)((unsigned)~bdmax << 5); }
    const int row_hi = ~row_lo, col_hi = ~col_lo;

    static _Thread_local int32_t tmp[64 * 64];
    memset(tmp, 0, sizeof(tmp));
    const int rk = ty_row[txtp], ck = ty_col[txtp];
    for (int y = 0; y < sh; y++) {
        int32_t *r = &tmp[y * w];
        for (int x = 0; x < sw; x++) {
            const int v = CF(y + x * sh);
            r[x] = rect2 ? (v * 181 + 128) >> 8 : v;
        }
        oracle_itx_1d(rk, w, r, 1, row_lo, row_hi);
    }
    if (hbd) memset(cf32, 0, sizeof(int32_t) * sw * sh);
    else memset(cf16, 0, sizeof(int16_t) * sw * sh);
    for (int i = 0; i < w * sh; i++)
        tmp[i] = clipi((tmp[i] + rnd) >> shift, col_lo, col_hi);
    for (int x = 0; x < w; x++) oracle_itx_1d(ck, h, &tmp[x], w, col_lo, col_hi);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++)
            SETPX(x, y, clip_px(PX(x, y) + ((tmp[y * w + x] + 8) >> 4), bdmax));
#undef PX
#undef SETPX
#undef CF
}

/* Frame-batched driver: identical block semantics, processed in list order. */
typedef struct {
    uint32_t coef_off;
    uint16_t x, y;
    uint8_t plane, tx, txtp, flags;
    int32_t eob;
} OracleTxBlock; /* == MiTxBlock (include/mi_av1dsp.h) */

void oracle_itx_frame(void *const planes[3], const ptrdiff_t strides[3], const void *blocks_,
                      int n_blocks, void *arena, int bdmax)
{
    const OracleTxBlock *b = blocks_;
    const int hbd = bdmax > 255;
    for (int i = 0; i < n_blocks; i++) {
        const int pl = b[i].plane;
        uint8_t *dst = (uint8_t *)planes[pl] + (ptrdiff_t)b[i].y * strides[pl] +
                       (ptrdiff_t)b[i].x * (hbd ? 2 : 1);
        void *cf = (uint8_t *)arena + (size_t)b[i].coef_off * (hbd ? 4 : 2);
        if (b[i].flags & 0x80) {
            /* packed (MI_TX_PACKED, include/mi_av1dsp.h): the arena holds the CW x CH corner,
             * row-major; expand it to itxfm_add's dense layout (column-major, column height
             * min(h,32)), transform, and consume the corner as itxfm_add consumes the dense
             * block (its entries zeroed) */
            const int cw = ((b[i].flags >> 3) & 7) * 4 + 4, ch = (b[i].flags & 7) * 4 + 4;
            const int sh = tx_h[b[i].tx] < 32 ? tx_h[b[i].tx] : 32;
            int32_t dense32[32 * 32];
            int16_t *dense16 = (int16_t *)dense32;
            memset(dense32, 0, sizeof(dense32));
            for (int x = 0; x < cw; x++)
                for (int y = 0; y < ch; y++) {
                    if (hbd && (b[i].flags & 0x40)) {   /* MI_TX_I16: int16 corner in the int32 arena */
                        dense32[y + x * sh] = ((int16_t *)cf)[y * cw + x]; ((int16_t *)cf)[y * cw + x] = 0;
                    } else if (hbd) { dense32[y + x * sh] = ((int32_t *)cf)[y * cw + x]; ((int32_t *)cf)[y * cw + x] = 0; }
                    else { dense16[y + x * sh] = ((int16_t *)cf)[y * cw + x]; ((int16_t *)cf)[y * cw + x] = 0; }
                }
            oracle_itxfm_add(b[i].tx, b[i].txtp, dst, strides[pl], dense32, b[i].eob, bdmax);
            continue;
        }
        oracle_itxfm_add(b[i].tx, b[i].txtp, dst, strides[pl], cf, b[i].eob, bdmax);
    }
}
