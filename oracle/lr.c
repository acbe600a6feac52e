/*
 * oracle/lr.c — CPU restatement of loop restoration (TEST INFRASTRUCTURE ONLY).
 *
 * Follows FreezyLemon/rav1d:
 *   src/looprestoration.rs:139-268  padding          (C src/looprestoration_tmpl.c:42-137)
 *   src/looprestoration.rs:299-370  wiener           (C looprestoration_tmpl.c:142-200)
 *   src/looprestoration.rs:398-565  boxsum3/boxsum5  (C looprestoration_tmpl.c:222-347)
 *   src/looprestoration.rs:566-684  selfguided_filter(C looprestoration_tmpl.c:349-445)
 *   src/looprestoration.rs:710-912  sgr_5x5/3x3/mix  (C looprestoration_tmpl.c:447-530)
 *   src/lr_apply.rs:28-329          lr_stripe / lr_sbrow / rav1d_lr_sbrow (C src/lr_apply_tmpl.c)
 *   src/lf_apply.rs:24-141          backup_lpf (the deblocked line buffer LR reads across stripes)
 *
 * The frame driver runs the reference's in-place algorithm on a copy of the CDEF output,
 * with the same 4-rows-per-stripe-boundary line buffer (frame-threaded layout,
 * lf_apply.rs:143-260) built from the deblocked picture, and the same left-column backups.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define RUS 390 /* REST_UNIT_STRIDE */

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int iclip(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

enum { LR_HAVE_LEFT = 1, LR_HAVE_RIGHT = 2, LR_HAVE_TOP = 4, LR_HAVE_BOTTOM = 8 };

/* sgr tables (dav1d_sgr_params / dav1d_sgr_x_by_x, src/tables.rs) */
static const uint16_t sgr_params[16][2] = {
    { 140, 3236 }, { 112, 2158 }, { 93, 1618 }, { 80, 1438 }, { 70, 1295 }, { 58, 1177 },
    { 47, 1079 },  { 37, 996 },   { 30, 925 },  { 25, 863 },  { 0, 2589 },  { 0, 1618 },
    { 0, 1177 },   { 0, 925 },    { 56, 0 },    { 22, 0 },
};
/* x_by_x[z] = round(256 / (z + 1)) with the ends pinned to 255 and 0; checked against the
 * reference table by tests/test_oracle_lr.py when the reference is mounted. */
static _Thread_local uint8_t sgr_x_by_x[256];
static void init_tables(void)
{
    static _Thread_local int done;
    if (done) return;
    for (int z = 0; z < 256; z++) sgr_x_by_x[z] = (uint8_t)((256 + (z + 1) / 2) / (z + 1));
    sgr_x_by_x[0] = 255;
    sgr_x_by_x[255] = 0;
    done = 1;
}
const uint8_t *oracle_sgr_x_by_x(void) { init_tables(); return sgr_x_by_x; }

typedef struct { int hbd, bdmax, bd; } PX;
static inline int RD(const PX *px, const void *b, ptrdiff_t i)
{ return px->hbd ? ((const uint16_t *)b)[i] : ((const uint8_t *)b)[i]; }
static inline void WR(const PX *px, void *b, ptrdiff_t i, int v)
{ if (px->hbd) ((uint16_t *)b)[i] = (uint16_t)v; else ((uint8_t *)b)[i] = (uint8_t)v; }

/* padding (looprestoration.rs:139-268). p/lpf in pixels with stride ps; left[h][4]. out: int tmp */
static void padding(const PX *px, int *dst, const void *p, ptrdiff_t ps, const int (*left)[4],
                    const void *lpf, int unit_w, int stripe_h, int edges)
{
    const int have_left = !!(edges & LR_HAVE_LEFT), have_right = !!(edges & LR_HAVE_RIGHT);
    unit_w += 3 * have_left + 3 * have_right;
    int *dst_l = dst + 3 * !have_left;
    const ptrdiff_t poff = -3 * have_left;     /* p -= 3*have_left; lpf -= 3*have_left */
#define PIX(base, i) RD(px, base, (i))
    if (edges & LR_HAVE_TOP) {
        for (int x = 0; x < unit_w; x++) {
            const int a1 = PIX(lpf, poff + x), a2 = PIX(lpf, ps + poff + x);
            dst_l[x] = a1;
            dst_l[RUS + x] = a1;
            dst_l[2 * RUS + x] = a2;
        }
    } else {
        for (int x = 0; x < unit_w; x++) {
            const int v = PIX(p, poff + x);
            dst_l[x] = dst_l[RUS + x] = dst_l[2 * RUS + x] = v;
        }
        if (have_left)
            for (int r = 0; r < 3; r++)
                for (int x = 0; x < 3; x++) dst_l[r * RUS + x] = left[0][1 + x];
    }
    int *dst_tl = dst_l + 3 * RUS;
    if (edges & LR_HAVE_BOTTOM) {
        for (int x = 0; x < unit_w; x++) {
            const int b1 = PIX(lpf, 6 * ps + poff + x), b2 = PIX(lpf, 7 * ps + poff + x);
            dst_tl[stripe_h * RUS + x] = b1;
            dst_tl[(stripe_h + 1) * RUS + x] = b2;
            dst_tl[(stripe_h + 2) * RUS + x] = b2;
        }
    } else {
        for (int x = 0; x < unit_w; x++) {
            const int v = PIX(p, (stripe_h - 1) * ps + poff + x);
            for (int r = 0; r < 3; r++) dst_tl[(stripe_h + r) * RUS + x] = v;
        }
        if (have_left)
            for (int r = 0; r < 3; r++)
                for (int x = 0; x < 3; x++) dst_tl[(stripe_h + r) * RUS + x] = left[stripe_h - 1][1 + x];
    }
    for (int j = 0; j < stripe_h; j++)
        for (int x = 3 * have_left; x < unit_w; x++)
            dst_tl[j * RUS + x] = PIX(p, j * ps + poff + x);
    if (!have_right) {
        for (int j = 0; j < stripe_h + 6; j++) {
            const int last = dst_l[j * RUS + unit_w - 1];
            for (int x = 0; x < 3; x++) dst_l[j * RUS + unit_w + x] = last;
        }
    }
    if (!have_left) {
        for (int j = 0; j < stripe_h + 6; j++)
            for (int x = 0; x < 3; x++) dst[j * RUS + x] = dst_l[j * RUS];
    } else {
        for (int j = 0; j < stripe_h; j++)
            for (int x = 0; x < 3; x++) dst[(j + 3) * RUS + x] = left[j][1 + x];
    }
#undef PIX
}

typedef struct {
    int16_t filter[2][8];
    int s0, s1, w0, w1;
} LrParams;

/* wiener (looprestoration.rs:299-370). The 8-bit centre +128 is folded into filter[0][3]
 * for every bit depth (value-identical to the reference's separate 8-bit term). */
static void wiener(const PX *px, void *p, ptrdiff_t ps, const int (*left)[4], const void *lpf,
                   int w, int h, const LrParams *prm, int edges)
{
    static _Thread_local int tmp[70 * RUS], hor[70 * RUS];
    padding(px, tmp, p, ps, left, lpf, w, h, edges);
    const int bd = px->bd;
    const int rbh = 3 + (bd == 12) * 2;
    const int clip_limit = 1 << (bd + 1 + 7 - rbh);
    for (int j = 0; j < h + 6; j++)
        for (int i = 0; i < w; i++) {
            int sum = 1 << (bd + 6);
            for (int k = 0; k < 7; k++) sum += tmp[j * RUS + i + k] * prm->filter[0][k];
            hor[j * RUS + i] = iclip((sum + (1 << (rbh - 1))) >> rbh, 0, clip_limit - 1);
        }
    const int rbv = 11 - (bd == 12) * 2;
    const int round_offset = 1 << (bd + (rbv - 1));
    for (int j = 0; j < h; j++)
        for (int i = 0; i < w; i++) {
            int sum = -round_offset;
            for (int k = 0; k < 7; k++) sum += hor[(j + k) * RUS + i] * prm->filter[1][k];
            WR(px, p, j * ps + i, iclip((sum + (1 << (rbv - 1))) >> rbv, 0, px->bdmax));
        }
}

/* box sums over 3x3 / 5x5 (looprestoration.rs:398-565), written as the direct windowed sums
 * at the positions the filter reads: rows/cols -1..h/w of the unit for 3x3; for 5x5 rows
 * -1, 1, 3, ... only. sum/sumsq indexed [(y + 3) * RUS + x + 3]. */
static void boxsum(int *sumsq, int *sum, const int *src, int w, int h, int r, int step)
{
    for (int y = -1; y < h + 1; y += step)
        for (int x = -1; x < w + 1; x++) {
            int s = 0, q = 0;
            for (int dy = -r; dy <= r; dy++)
                for (int dx = -r; dx <= r; dx++) {
                    const int v = src[(y + 3 + dy) * RUS + x + 3 + dx];
                    s += v;
                    q += v * v;
                }
            sum[(y + 3) * RUS + x + 3] = s;
            sumsq[(y + 3) * RUS + x + 3] = q;
        }
}

/* selfguided_filter (looprestoration.rs:566-684). dst: [h][384] */
static void selfguided(const PX *px, int *dst, const int *src, int w, int h, int n, unsigned s)
{
    init_tables();
    static _Thread_local int sumsq[70 * RUS], sum[70 * RUS];
    const unsigned one_by_x = n == 25 ? 164 : 455;
    const int step = (n == 25) + 1;
    boxsum(sumsq, sum, src, w, h, n == 25 ? 2 : 1, step);
    const int bdm8 = px->bd - 8;
    for (int j = -1; j < h + 1; j += step)
        for (int i = -1; i < w + 1; i++) {
            int *AA = &sumsq[(j + 3) * RUS + i + 3];
            int *BB = &sum[(j + 3) * RUS + i + 3];
            const int a = (*AA + ((1 << (2 * bdm8)) >> 1)) >> (2 * bdm8);
            const int b = (*BB + ((1 << bdm8) >> 1)) >> bdm8;
            const unsigned p = (unsigned)imax(a * n - b * b, 0);
            const unsigned z = (p * s + (1u << 19)) >> 20;
            const unsigned x = sgr_x_by_x[z < 255 ? z : 255];
            *AA = (int)((x * (unsigned)*BB * one_by_x + (1u << 11)) >> 12);
            *BB = (int)x;
        }
    /* A = sumsq (now the scaled b term), B = sum (now x) */
#define A_(y, x) sumsq[((y) + 3) * RUS + (x) + 3]
#define B_(y, x) sum[((y) + 3) * RUS + (x) + 3]
#define S_(y, x) src[((y) + 3) * RUS + (x) + 3]
    if (n == 25) {
        for (int j = 0; j < h; j++) {
            for (int i = 0; i < w; i++) {
                int a, b;
                if (!(j & 1)) {
                    a = (B_(j - 1, i) + B_(j + 1, i)) * 6 +
                        (B_(j - 1, i - 1) + B_(j + 1, i - 1) + B_(j - 1, i + 1) + B_(j + 1, i + 1)) * 5;
                    b = (A_(j - 1, i) + A_(j + 1, i)) * 6 +
                        (A_(j - 1, i - 1) + A_(j + 1, i - 1) + A_(j - 1, i + 1) + A_(j + 1, i + 1)) * 5;
                    dst[j * 384 + i] = (b - a * S_(j, i) + (1 << 8)) >> 9;
                } else {
                    a = B_(j, i) * 6 + (B_(j, i - 1) + B_(j, i + 1)) * 5;
                    b = A_(j, i) * 6 + (A_(j, i - 1) + A_(j, i + 1)) * 5;
                    dst[j * 384 + i] = (b - a * S_(j, i) + (1 << 7)) >> 8;
                }
            }
        }
    } else {
        for (int j = 0; j < h; j++)
            for (int i = 0; i < w; i++) {
                const int a = (B_(j, i) + B_(j, i - 1) + B_(j, i + 1) + B_(j - 1, i) + B_(j + 1, i)) * 4 +
                              (B_(j - 1, i - 1) + B_(j + 1, i - 1) + B_(j - 1, i + 1) + B_(j + 1, i + 1)) * 3;
                const int b = (A_(j, i) + A_(j, i - 1) + A_(j, i + 1) + A_(j - 1, i) + A_(j + 1, i)) * 4 +
                              (A_(j - 1, i - 1) + A_(j + 1, i - 1) + A_(j - 1, i + 1) + A_(j + 1, i + 1)) * 3;
                dst[j * 384 + i] = (b - a * S_(j, i) + (1 << 8)) >> 9;
            }
    }
#undef A_
#undef B_
#undef S_
}

/* sgr_5x5 / sgr_3x3 / sgr_mix (looprestoration.rs:710-912); kind 0, 1, 2 */
static void sgr(const PX *px, int kind, void *p, ptrdiff_t ps, const int (*left)[4], const void *lpf,
                int w, int h, const LrParams *prm, int edges)
{
    static _Thread_local int tmp[70 * RUS], d0[64 * 384], d1[64 * 384];
    padding(px, tmp, p, ps, left, lpf, w, h, edges);
    if (kind != 1) selfguided(px, d0, tmp, w, h, 25, (unsigned)prm->s0);
    if (kind != 0) selfguided(px, d1, tmp, w, h, 9, (unsigned)prm->s1);
    for (int j = 0; j < h; j++)
        for (int i = 0; i < w; i++) {
            int v;
            if (kind == 0) v = prm->w0 * d0[j * 384 + i];
            else if (kind == 1) v = prm->w1 * d1[j * 384 + i];
            else v = prm->w0 * d0[j * 384 + i] + prm->w1 * d1[j * 384 + i];
            const int o = RD(px, p, j * ps + i);
            WR(px, p, j * ps + i, iclip(o + ((v + (1 << 10)) >> 11), 0, px->bdmax));
        }
}

/* Av1RestorationUnit (src/lf_mask.rs:31-38) and Av1Restoration (one per 128x128) */
typedef struct {
    uint8_t type;
    int8_t filter_h[3], filter_v[3], sgr_weights[2];
} ORestUnit;
typedef struct { ORestUnit lr[3][4]; } ORestoration;

enum { RT_NONE = 0, RT_SWITCHABLE = 1, RT_WIENER = 2, RT_SGRPROJ = 3 };

typedef struct {
    PX px;
    int ss_hor, ss_ver, sb128, sbh, sb128w, w, h;
    const ORestoration *lr_mask;
    int unit_size_log2[2];
    /* line buffer (frame-threaded layout): per plane, 4 rows per stripe boundary */
    uint8_t *lpf[3];
    ptrdiff_t lpf_stride[3];
} LrFrame;

/* lr_stripe (lr_apply.rs:28-123) */
static void lr_stripe(const LrFrame *f, uint8_t *p, ptrdiff_t stride, const int (*left)[4], int x, int y,
                      int plane, int unit_w, int row_h, const ORestUnit *lr, int edges)
{
    const PX *px = &f->px;
    const int pxb = px->hbd ? 2 : 1;
    const int chroma = !!plane;
    const int ss_ver = chroma & f->ss_ver;
    const int sby = (y + (y ? 8 << ss_ver : 0)) >> (6 - ss_ver + f->sb128);
    const ptrdiff_t ps = stride / pxb;
    const uint8_t *lpf = f->lpf[plane] + ((ptrdiff_t)(sby * (4 << f->sb128) - 4) * f->lpf_stride[plane]) + (ptrdiff_t)x * pxb;
    int stripe_h = imin((64 - 8 * !y) >> ss_ver, row_h - y);

    LrParams prm;
    memset(&prm, 0, sizeof(prm));
    int kind;
    if (lr->type == RT_WIENER) {
        prm.filter[0][0] = prm.filter[0][6] = lr->filter_h[0];
        prm.filter[0][1] = prm.filter[0][5] = lr->filter_h[1];
        prm.filter[0][2] = prm.filter[0][4] = lr->filter_h[2];
        prm.filter[0][3] = (int16_t)(-(prm.filter[0][0] + prm.filter[0][1] + prm.filter[0][2]) * 2 + 128);
        prm.filter[1][0] = prm.filter[1][6] = lr->filter_v[0];
        prm.filter[1][1] = prm.filter[1][5] = lr->filter_v[1];
        prm.filter[1][2] = prm.filter[1][4] = lr->filter_v[2];
        prm.filter[1][3] = (int16_t)(128 - (prm.filter[1][0] + prm.filter[1][1] + prm.filter[1][2]) * 2);
        kind = -1;
    } else {
        const int idx = lr->type - RT_SGRPROJ;
        prm.s0 = sgr_params[idx][0];
        prm.s1 = sgr_params[idx][1];
        prm.w0 = lr->sgr_weights[0];
        prm.w1 = 128 - (lr->sgr_weights[0] + lr->sgr_weights[1]);
        kind = !!prm.s0 + !!prm.s1 * 2 - 1;
    }
    while (y + stripe_h <= row_h) {
        const int bottom = (sby + 1 != f->sbh || y + stripe_h != row_h);
        edges = bottom ? (edges | LR_HAVE_BOTTOM) : (edges & ~LR_HAVE_BOTTOM);
        const void *lp = lpf;   /* line buffer shares the picture stride */
        if (kind < 0) wiener(px, p, ps, left, lp, unit_w, stripe_h, &prm, edges);
        else sgr(px, kind, p, ps, left, lp, unit_w, stripe_h, &prm, edges);
        left += stripe_h;
        y += stripe_h;
        p += stripe_h * stride;
        edges |= LR_HAVE_TOP;
        stripe_h = imin(64 >> ss_ver, row_h - y);
        if (stripe_h == 0) break;
        lpf += 4 * f->lpf_stride[plane];
    }
}

/* lr_sbrow (lr_apply.rs:151-259) */
static void lr_sbrow(const LrFrame *f, uint8_t *p, ptrdiff_t stride, int y, int w, int h, int row_h,
                     int plane)
{
    const PX *px = &f->px;
    const int pxb = px->hbd ? 2 : 1;
    const int chroma = !!plane;
    const int ss_ver = chroma & f->ss_ver, ss_hor = chroma & f->ss_hor;
    const int unit_size_log2 = f->unit_size_log2[chroma];
    const int unit_size = 1 << unit_size_log2;
    const int half_unit_size = unit_size >> 1;
    const int max_unit_size = unit_size + half_unit_size;
    const int row_y = y + ((8 >> ss_ver) * !!y);
    const int shift_hor = 7 - ss_hor;
    static _Thread_local int pre_lr_border[2][128 + 8][4];
    const ORestUnit *lr[2];
    int edges = (y > 0 ? LR_HAVE_TOP : 0) | LR_HAVE_RIGHT;
    int aligned_unit_pos = row_y & ~(unit_size - 1);
    if (aligned_unit_pos && aligned_unit_pos + half_unit_size > h) aligned_unit_pos -= unit_size;
    aligned_unit_pos <<= ss_ver;
    const int sb_idx = (aligned_unit_pos >> 7) * f->sb128w;
    const int unit_idx = ((aligned_unit_pos >> 6) & 1) << 1;
    lr[0] = &f->lr_mask[sb_idx].lr[plane][unit_idx];
    int restore = lr[0]->type != RT_NONE;
    int x = 0, bit = 0;
    for (; x + max_unit_size <= w; p += (ptrdiff_t)unit_size * pxb, edges |= LR_HAVE_LEFT, bit ^= 1) {
        const int next_x = x + unit_size;
        const int next_u_idx = unit_idx + ((next_x >> (shift_hor - 1)) & 1);
        lr[!bit] = &f->lr_mask[sb_idx + (next_x >> shift_hor)].lr[plane][next_u_idx];
        const int restore_next = lr[!bit]->type != RT_NONE;
        if (restore_next)   /* backup4xU: pre-LR last 4 columns of this unit */
            for (int r = 0; r < row_h - y; r++)
                for (int c = 0; c < 4; c++)
                    pre_lr_border[bit][r][c] = RD(px, p + r * stride, unit_size - 4 + c);
        if (restore)
            lr_stripe(f, p, stride, (const int (*)[4])pre_lr_border[!bit], x, y, plane, unit_size, row_h,
                      lr[bit], edges);
        x = next_x;
        restore = restore_next;
    }
    if (restore) {
        edges &= ~LR_HAVE_RIGHT;
        lr_stripe(f, p, stride, (const int (*)[4])pre_lr_border[!bit], x, y, plane, w - x, row_h,
                  lr[bit], edges);
    }
}

/* backup_lpf (lf_apply.rs:24-141) for every sbrow, frame-threaded layout: the block for the
 * boundary after stripe k holds rows B-2, B-1, B, B+1 (B+1 clamped to the last row). */
static void build_lpf(LrFrame *f, int plane, const uint8_t *d, ptrdiff_t stride, int w, int h)
{
    const int ss_ver = plane ? f->ss_ver : 0;
    const int pxb = f->px.hbd ? 2 : 1;
    const int n_blocks = f->sbh * (1 << f->sb128) + 2;
    f->lpf_stride[plane] = stride;
    /* one extra block in front so that "sby * (4 << sb128) - 4" is valid for sby = 0 */
    uint8_t *buf = calloc((size_t)(n_blocks + 1) * 4, (size_t)stride);
    f->lpf[plane] = buf + 4 * stride;
    for (int sby = 0; sby < f->sbh; sby++) {
        const int sbsz = (64 << f->sb128) >> ss_ver;
        int row = sby ? sby * sbsz - (8 >> ss_ver) : 0;
        const int row_h = imin((sby + 1) * sbsz, h - 1);
        uint8_t *dst = f->lpf[plane] + (ptrdiff_t)sby * (4 << f->sb128) * stride;
        int stripe_h = (64 - 8 * !row) >> ss_ver;
        while (row + stripe_h <= row_h) {
            const int B = row + stripe_h;
            const int n_lines = 4 - (B + 1 == h);
            for (int i = 0; i < 4; i++) {
                const uint8_t *src = i == n_lines ? dst - stride : d + (ptrdiff_t)(B - 2 + i) * stride;
                memcpy(dst, src, (size_t)w * pxb);
                dst += stride;
            }
            row += stripe_h;
            stripe_h = 64 >> ss_ver;
        }
    }
}

/* Whole-frame loop restoration.
 * cdef: the CDEF output (LR input, read only); deblocked: the pre-CDEF picture (line buffer
 * source); dst: output (may alias nothing). restore_planes: bit0 Y, bit1 U, bit2 V.
 * lr_mask: Av1Restoration [sb128h][sb128w]. All planes 128-row aligned with `strides`. */
void oracle_lr_frame(void *const dst[3], void *const cdef[3], void *const deblocked[3],
                     const ptrdiff_t strides[3], int w, int h, int layout, int bpc, int sb128,
                     int restore_planes, const int unit_size_log2[2], const void *lr_mask,
                     int sb128w)
{
    LrFrame f;
    memset(&f, 0, sizeof(f));
    f.px.hbd = bpc > 8;
    f.px.bdmax = (1 << bpc) - 1;
    f.px.bd = bpc;
    f.ss_ver = layout == 1;
    f.ss_hor = layout == 1 || layout == 2;
    f.sb128 = sb128;
    f.sbh = (h + (64 << sb128) - 1) >> (6 + sb128);
    f.sb128w = sb128w;
    f.w = w;
    f.h = h;
    f.lr_mask = lr_mask;
    f.unit_size_log2[0] = unit_size_log2[0];
    f.unit_size_log2[1] = unit_size_log2[1];
    const int rows_y = (h + 127) & ~127;
    const int nplanes = layout ? 3 : 1;
    for (int p = 0; p < nplanes; p++) {
        const int rows = p ? rows_y >> f.ss_ver : rows_y;
        memcpy(dst[p], cdef[p], (size_t)rows * strides[p]);
    }
    for (int p = 0; p < nplanes; p++) {
        if (!(restore_planes & (1 << p))) continue;
        const int ph = p ? (h + f.ss_ver) >> f.ss_ver : h;
        const int bw8 = p ? ((((w + 7) >> 3) << 3) >> f.ss_hor) : (((w + 7) >> 3) << 3);
        build_lpf(&f, p, deblocked[p], strides[p], bw8, ph);
    }
    const int pxb = f.px.hbd ? 2 : 1;
    for (int sby = 0; sby < f.sbh; sby++) {
        const int not_last = sby + 1 < f.sbh;
        const int offset_y = 8 * !!sby;
        if (restore_planes & 1) {
            const int next_row_y = (sby + 1) << (6 + sb128);
            const int row_h = imin(next_row_y - 8 * not_last, h);
            const int y_stripe = (sby << (6 + sb128)) - offset_y;
            lr_sbrow(&f, (uint8_t *)dst[0] + (ptrdiff_t)y_stripe * strides[0], strides[0], y_stripe, w, h,
                     row_h, 0);
        }
        if (layout && (restore_planes & 6)) {
            const int ss_ver = f.ss_ver, ss_hor = f.ss_hor;
            const int ph = (h + ss_ver) >> ss_ver, pw = (w + ss_hor) >> ss_hor;
            const int next_row_y = (sby + 1) << ((6 - ss_ver) + sb128);
            const int row_h = imin(next_row_y - (8 >> ss_ver) * not_last, ph);
            const int offset_uv = offset_y >> ss_ver;
            const int y_stripe = (sby << ((6 - ss_ver) + sb128)) - offset_uv;
            for (int p = 1; p <= 2; p++)
                if (restore_planes & (1 << p))
                    lr_sbrow(&f, (uint8_t *)dst[p] + (ptrdiff_t)y_stripe * strides[p], strides[p], y_stripe,
                             pw, ph, row_h, p);
        }
    }
    (void)pxb;
    for (int p = 0; p < 3; p++)
        if (f.lpf[p]) free(f.lpf[p] - 4 * f.lpf_stride[p]);
}

/* Per-call lr.wiener / lr.sgr[kind] (looprestoration.rs:91-107): the table slots' semantics on
 * one unit. left: [h][4] pixels; lpf: rows 0, 1 (above) and 6, 7 (below) at stride `stride`;
 * filter: LooprestorationParams.filter as the reference builds it (lr_apply.rs:59-82: the
 * 8-bit centre without its +128, folded here as the restatement expects). */
void oracle_lr_wiener(void *p, ptrdiff_t stride, const void *left_px, const void *lpf, int w, int h,
                      const int16_t filter[2][8], int edges, int bdmax)
{
    PX px = { bdmax > 255, bdmax, bdmax == 255 ? 8 : bdmax == 1023 ? 10 : 12 };
    const ptrdiff_t ps = stride / (px.hbd ? 2 : 1);
    int left[64][4];
    for (int j = 0; j < h; j++)
        for (int k = 0; k < 4; k++) left[j][k] = RD(&px, left_px, j * 4 + k);
    LrParams prm;
    memset(&prm, 0, sizeof(prm));
    memcpy(prm.filter, filter, sizeof(prm.filter));
    if (px.bd == 8) prm.filter[0][3] += 128;
    wiener(&px, p, ps, (const int (*)[4])left, lpf, w, h, &prm, edges);
}

void oracle_lr_sgr(int kind, void *p, ptrdiff_t stride, const void *left_px, const void *lpf, int w, int h,
                   unsigned s0, unsigned s1, int w0, int w1, int edges, int bdmax)
{
    PX px = { bdmax > 255, bdmax, bdmax == 255 ? 8 : bdmax == 1023 ? 10 : 12 };
    const ptrdiff_t ps = stride / (px.hbd ? 2 : 1);
    int left[64][4];
    for (int j = 0; j < h; j++)
        for (int k = 0; k < 4; k++) left[j][k] = RD(&px, left_px, j * 4 + k);
    LrParams prm;
    memset(&prm, 0, sizeof(prm));
    prm.s0 = (int)s0; prm.s1 = (int)s1; prm.w0 = w0; prm.w1 = w1;
    sgr(&px, kind, p, ps, (const int (*)[4])left, lpf, w, h, &prm, edges);
}
