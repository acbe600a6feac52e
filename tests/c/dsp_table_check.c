/*
 * dsp_table_check.c — a rav1d-style caller of the slot-exact surface (TEST ONLY): fills a
 * Rav1dDSPContext-layout table with mi_fill_dsp_tables and calls slots through the function
 * pointers, as rav1d's apply modules call f.dsp (itx: recon.rs:1781-1788; loop filter:
 * lf_apply.rs:470-531; CDEF: cdef_apply.rs:390-440), checking every result against the
 * oracle's per-call restatement (oracle/). Host buffers, positive and negative strides.
 * Exit status 0 = every slot matched. Needs a GPU (the slots launch on device 0).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mi_dsp_table.h"

void oracle_itxfm_add(int tx, int txtp, void *dst, ptrdiff_t stride, void *coeff, int eob, int bitdepth_max);
void oracle_lf_sb(int cls, int dir, void *dst, ptrdiff_t stride, const uint32_t *vmask, const uint8_t *lvl,
                  ptrdiff_t b4_stride, const uint8_t *lut_e, const uint8_t *lut_i, int wh, int bdmax);
int oracle_cdef_find_dir(const void *img, ptrdiff_t stride, unsigned *var, int bdmax);
void oracle_cdef_filter_block(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                              const void *left, const void *top, const void *bottom, int pri, int sec, int dir,
                              int damping, int w, int h, int edges, int bdmax);
void oracle_calc_eih(uint8_t *lut_e, uint8_t *lut_i, int sharp);

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)(rng_state >> 16);
}

static const int TXW[19] = { 4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64 };
static const int TXH[19] = { 4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16 };

static int fails = 0, calls = 0;

/* every filled itxfm_add slot, random coefficients, eob regimes DC-only / partial / full */
static void check_itx(const MiDSPContext *c, int bpc, int neg) {
    const int bdmax = (1 << bpc) - 1, pxb = bpc == 8 ? 1 : 2, cb = bpc == 8 ? 2 : 4;
    for (int tx = 0; tx < 19; tx++)
        for (int t = 0; t < 17; t++) {
            if (!c->itx.itxfm_add[tx][t]) continue;
            const int w = TXW[tx], h = TXH[tx], sw = w < 32 ? w : 32, sh = h < 32 ? h : 32, n = sw * sh;
            for (int reg = 0; reg < 3; reg++) {
                const int eob = reg == 0 ? 0 : reg == 1 ? (int)(rnd() % (unsigned)(n / 4 + 1)) : n - 1;
                const ptrdiff_t st = (ptrdiff_t)w * pxb + 64;
                uint8_t *a = malloc(st * h), *b = malloc(st * h);
                for (ptrdiff_t i = 0; i < st * h; i++) a[i] = (uint8_t)rnd();
                if (pxb == 2)
                    for (ptrdiff_t i = 0; i < st * h / 2; i++) ((uint16_t *)a)[i] &= bdmax;
                memcpy(b, a, st * h);
                void *ca = calloc(n, cb), *cc = calloc(n, cb);
                const int lim = t == 16 ? 64 : 1 << (bpc + 1);
                for (int i = 0; i <= eob && i < n; i++) {
                    const int v = (int)(rnd() % (2 * lim + 1)) - lim;
                    if (cb == 2) ((int16_t *)ca)[i] = (int16_t)v; else ((int32_t *)ca)[i] = v;
                }
                memcpy(cc, ca, (size_t)n * cb);
                /* rav1d passes the top-left pixel and the byte stride; with --negstride the
                 * picture is walked bottom-up: the last row's address and a negative stride */
                uint8_t *da = neg ? a + st * (h - 1) : a, *db = neg ? b + st * (h - 1) : b;
                const ptrdiff_t s = neg ? -st : st;
                c->itx.itxfm_add[tx][t](da, s, ca, eob, bdmax);
                oracle_itxfm_add(tx, t, db, s, cc, eob, bdmax);
                calls++;
                int zero = 1;
                for (int i = 0; i < n * cb; i++) zero &= ((uint8_t *)ca)[i] == 0;
                if (memcmp(a, b, st * h) || !zero) {
                    if (fails++ < 10)
                        fprintf(stderr, "itxfm_add[%d][%d] bpc %d eob %d neg %d: %s\n", tx, t, bpc, eob, neg,
                                zero ? "pixels differ" : "coefficients not zeroed");
                }
                free(a); free(b); free(ca); free(cc);
            }
        }
}

static void check_lf(const MiDSPContext *c, int bpc) {
    const int bdmax = (1 << bpc) - 1, pxb = bpc == 8 ? 1 : 2;
    const int W = 160, H = 160;
    const ptrdiff_t st = W * pxb;
    uint8_t lut[144];
    for (int cls = 0; cls < 2; cls++)
        for (int dir = 0; dir < 2; dir++)
            for (int it = 0; it < 6; it++) {
                uint8_t *a = malloc(st * H), *b = malloc(st * H);
                const int base = (int)(rnd() % (unsigned)(bdmax + 1));
                for (int i = 0; i < W * H; i++) {
                    const int v = (rnd() % 10 < 3) ? base : (int)(base + (int)(rnd() % 41) - 20);
                    const int px = v < 0 ? 0 : v > bdmax ? bdmax : v;
                    if (pxb == 1) a[i] = (uint8_t)px; else ((uint16_t *)a)[i] = (uint16_t)px;
                }
                memcpy(b, a, st * H);
                const int b4_stride = 48;
                uint8_t *lvl = malloc(40 * b4_stride * 4);
                for (int i = 0; i < 40 * b4_stride * 4; i++) lvl[i] = rnd() % 100 < 15 ? 0 : rnd() % 64;
                uint32_t vm[3] = { rnd() | rnd() << 16, rnd() | rnd() << 16, cls ? 0 : rnd() | rnd() << 16 };
                vm[1] &= ~vm[2];
                vm[0] = (vm[0] | rnd()) & ~(vm[1] | vm[2]);
                oracle_calc_eih(lut, lut + 64, rnd() % 8);
                memset(lut + 128, 0, 16);
                const int slot = cls ? 2 : 0;
                const uint8_t *l = lvl + (2 * b4_stride + 3) * 4 + slot;
                const ptrdiff_t o = 16 * st + 16 * pxb;
                c->lf.loop_filter_sb[cls][dir](a + o, st, vm, (const uint8_t (*)[4])l, b4_stride, lut, 32, bdmax);
                oracle_lf_sb(cls, dir, b + o, st, vm, l, b4_stride, lut, lut + 64, 32, bdmax);
                calls++;
                if (memcmp(a, b, st * H) && fails++ < 10)
                    fprintf(stderr, "loop_filter_sb[%d][%d] bpc %d iteration %d differs\n", cls, dir, bpc, it);
                free(a); free(b); free(lvl);
            }
}

static void check_cdef(const MiDSPContext *c, int bpc) {
    const int bdmax = (1 << bpc) - 1, pxb = bpc == 8 ? 1 : 2, bdm8 = bpc - 8;
    const int W = 32;
    const ptrdiff_t st = W * pxb;
    for (int it = 0; it < 60; it++) {
        const int fb = rnd() % 3, w = fb == 0 ? 8 : 4, h = fb == 2 ? 4 : 8;
        uint8_t *pic = malloc(st * W), *a = malloc(st * W), *b = malloc(st * W);
        for (int i = 0; i < W * W; i++) {
            const int v = (int)((i % W) * 4 + (i / W) * 3 + rnd() % 24) & bdmax;
            if (pxb == 1) pic[i] = (uint8_t)v; else ((uint16_t *)pic)[i] = (uint16_t)v;
        }
        memcpy(a, pic, st * W);
        memcpy(b, pic, st * W);
        const ptrdiff_t o = 8 * st + 8 * pxb;
        uint8_t left[8 * 2 * 2];
        for (int r = 0; r < h; r++) memcpy(left + r * 2 * pxb, pic + o + r * st - 2 * pxb, 2 * pxb);
        const int edges = rnd() % 16, pri = (rnd() % 16) << bdm8;
        const int secs[4] = { 0, 1, 2, 4 };
        const int sec = secs[rnd() % 4] << bdm8, d = rnd() % 8, damp = 3 + rnd() % 4 + bdm8;
        c->cdef.fb[fb](a + o, st, left, pic + o - 2 * st, pic + o + h * st, pri, sec, d, damp, (unsigned)edges,
                       bdmax);
        oracle_cdef_filter_block(b + o, st, pic + o, st, left, pic + o - 2 * st, pic + o + h * st, pri, sec, d, damp,
                                 w, h, edges, bdmax);
        unsigned va = 0, vb = 0;
        const int da = c->cdef.dir(pic + o, st, &va, bdmax), db = oracle_cdef_find_dir(pic + o, st, &vb, bdmax);
        calls += 2;
        if ((memcmp(a, b, st * W) || da != db || va != vb) && fails++ < 10)
            fprintf(stderr, "cdef fb[%d] / dir bpc %d iteration %d differs\n", fb, bpc, it);
        free(pic); free(a); free(b);
    }
}

int main(void) {
    if (mi_dsp_context_size() != sizeof(MiDSPContext)) {
        fprintf(stderr, "context size mismatch\n");
        return 2;
    }
    for (int bpc = 8; bpc <= 12; bpc += 2) {
        MiDSPContext c;
        if (mi_fill_dsp_tables(&c, bpc) || !c.initialized) {
            fprintf(stderr, "mi_fill_dsp_tables(%d) failed\n", bpc);
            return 2;
        }
        check_itx(&c, bpc, 0);
        check_itx(&c, bpc, 1);
        check_lf(&c, bpc);
        check_cdef(&c, bpc);
    }
    printf("dsp table: %d slot calls, %d mismatches\n", calls, fails);
    return fails ? 1 : 0;
}
