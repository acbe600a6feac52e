/*
 * ipred.c — CPU restatement of the intra-prediction DSP family. TEST INFRASTRUCTURE ONLY.
 *
 * Follows rav1d src/ipred.rs (`*_rust` fallbacks) == dav1d C src/ipred_tmpl.c:
 *   splat_dc / cfl_pred            ipred_tmpl.c:39-84     (ipred.rs :172, :236)
 *   dc / dc_top / dc_left / dc_128 ipred_tmpl.c:86-218    (ipred.rs dc_gen :260-400)
 *   v / h / paeth                  ipred_tmpl.c:220-265   (ipred.rs :409, :458, :507)
 *   smooth / _v / _h               ipred_tmpl.c:267-325   (ipred.rs :568, :625, :677)
 *   edge filter / upsample         ipred_tmpl.c:327-406   (ipred.rs :730-854)
 *   z1 / z2 / z3                   ipred_tmpl.c:408-616   (ipred.rs :855, :948, :1085)
 *   filter (recursive 4x2)         ipred_tmpl.c:618-655   (ipred.rs :1206-1325)
 *   cfl_ac                         ipred_tmpl.c:657-715   (ipred.rs :1326)
 *   pal_pred                       ipred_tmpl.c:717-727   (ipred.rs :1433)
 * Table index = the reference's intra_pred[] slot (levels.h IntraPredMode, implementation
 * modes): 0 DC, 1 V, 2 H, 3 LEFT_DC, 4 TOP_DC, 5 DC_128, 6 Z1, 7 Z2, 8 Z3, 9 SMOOTH,
 * 10 SMOOTH_V, 11 SMOOTH_H, 12 PAETH, 13 FILTER.
 *
 * `topleft` points at the corner sample of an edge buffer laid out as the reference's:
 * topleft[1 + i] = top row, topleft[-(1 + i)] = left column. Pixels are uint8_t (bpc 8) or
 * uint16_t (bpc 10/12); strides in bytes.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static const uint8_t sm_weights[128] = {
#include "../rav1d_amd/csrc/tables/sm_weights.inc"
};
static const uint16_t dr_intra_derivative[44] = {
#include "../rav1d_amd/csrc/tables/dr_intra_derivative.inc"
};
static const int8_t filter_intra_taps[5][64] = {
#include "../rav1d_amd/csrc/tables/filter_intra_taps.inc"
};

static inline int clip(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
static inline int ctz(unsigned v) { return __builtin_ctz(v); }

/* Edge and destination access: indices relative to the topleft pointer / dst origin. */
typedef struct {
    const void *tl;
    int bpc;
} Edge;
static inline int E(Edge e, int i) {
    return e.bpc == 8 ? ((const uint8_t *)e.tl)[i] : ((const uint16_t *)e.tl)[i];
}
static inline void D(void *dst, ptrdiff_t stride, int y, int x, int v, int bpc) {
    uint8_t *r = (uint8_t *)dst + y * stride;
    if (bpc == 8) r[x] = (uint8_t)v;
    else ((uint16_t *)r)[x] = (uint16_t)v;
}
static inline int Dget(const void *dst, ptrdiff_t stride, int y, int x, int bpc) {
    const uint8_t *r = (const uint8_t *)dst + y * stride;
    return bpc == 8 ? r[x] : ((const uint16_t *)r)[x];
}

static void splat(void *dst, ptrdiff_t stride, int w, int h, int v, int bpc) {
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) D(dst, stride, y, x, v, bpc);
}

static unsigned dc_top(Edge e, int w) {
    unsigned dc = w >> 1;
    for (int i = 0; i < w; i++) dc += E(e, 1 + i);
    return dc >> ctz(w);
}
static unsigned dc_left(Edge e, int h) {
    unsigned dc = h >> 1;
    for (int i = 0; i < h; i++) dc += E(e, -(1 + i));
    return dc >> ctz(h);
}
/* dc_gen (ipred_tmpl.c:150-166): 8-bit multipliers 0x5556/0x3334 >> 16, hbd 0xAAAB/0x6667 >> 17 */
static unsigned dc_both(Edge e, int w, int h, int bpc) {
    unsigned dc = (w + h) >> 1;
    for (int i = 0; i < w; i++) dc += E(e, i + 1);
    for (int i = 0; i < h; i++) dc += E(e, -(i + 1));
    dc >>= ctz(w + h);
    if (w != h) {
        const int q = w > h * 2 || h > w * 2;
        if (bpc == 8) dc = (dc * (q ? 0x3334u : 0x5556u)) >> 16;
        else dc = (dc * (q ? 0x6667u : 0xAAABu)) >> 17;
    }
    return dc;
}

/* get_filter_strength (ipred_tmpl.c:327-360) */
static int filter_strength(int wh, int angle, int is_sm) {
    if (is_sm) {
        if (wh <= 8) { if (angle >= 64) return 2; if (angle >= 40) return 1; }
        else if (wh <= 16) { if (angle >= 48) return 2; if (angle >= 20) return 1; }
        else if (wh <= 24) { if (angle >= 4) return 3; }
        else return 3;
    } else {
        if (wh <= 8) { if (angle >= 56) return 1; }
        else if (wh <= 16) { if (angle >= 40) return 1; }
        else if (wh <= 24) { if (angle >= 32) return 3; if (angle >= 16) return 2; if (angle >= 8) return 1; }
        else if (wh <= 32) { if (angle >= 32) return 3; if (angle >= 4) return 2; return 1; }
        else return 3;
    }
    return 0;
}

/* filter_edge (ipred_tmpl.c:362-385): in[] indices are relative to `in` */
static void filter_edge(int *out, int sz, int lim_from, int lim_to, Edge e, int in0, int from, int to, int strength) {
    static const uint8_t kernel[3][5] = { { 0, 4, 8, 4, 0 }, { 0, 5, 6, 5, 0 }, { 2, 4, 4, 4, 2 } };
    int i = 0;
    for (; i < (sz < lim_from ? sz : lim_from); i++) out[i] = E(e, in0 + clip(i, from, to - 1));
    for (; i < (lim_to < sz ? lim_to : sz); i++) {
        int s = 0;
        for (int j = 0; j < 5; j++) s += E(e, in0 + clip(i - 2 + j, from, to - 1)) * kernel[strength - 1][j];
        out[i] = (s + 8) >> 4;
    }
    for (; i < sz; i++) out[i] = E(e, in0 + clip(i, from, to - 1));
}

static int get_upsample(int wh, int angle, int is_sm) { return angle < 40 && wh <= 16 >> is_sm; }

/* upsample_edge (ipred_tmpl.c:391-406) */
static void upsample_edge(int *out, int hsz, Edge e, int in0, int from, int to, int bdmax) {
    static const int8_t kernel[4] = { -1, 9, 9, -1 };
    int i;
    for (i = 0; i < hsz - 1; i++) {
        out[i * 2] = E(e, in0 + clip(i, from, to - 1));
        int s = 0;
        for (int j = 0; j < 4; j++) s += E(e, in0 + clip(i + j - 1, from, to - 1)) * kernel[j];
        out[i * 2 + 1] = clip((s + 8) >> 4, 0, bdmax);
    }
    out[i * 2] = E(e, in0 + clip(i, from, to - 1));
}

static void z1(void *dst, ptrdiff_t stride, Edge e, int w, int h, int angle, int bpc) {
    const int bdmax = (1 << bpc) - 1;
    const int is_sm = (angle >> 9) & 1, eef = angle >> 10;
    angle &= 511;
    int dx = dr_intra_derivative[angle >> 1];
    int top[128 + 64];
    int max_base_x;
    const int up = eef ? get_upsample(w + h, 90 - angle, is_sm) : 0;
    if (up) {
        upsample_edge(top, w + h, e, 1, -1, w + (w < h ? w : h), bdmax);
        max_base_x = 2 * (w + h) - 2;
        dx <<= 1;
    } else {
        const int fs = eef ? filter_strength(w + h, 90 - angle, is_sm) : 0;
        if (fs) {
            filter_edge(top, w + h, 0, w + h, e, 1, -1, w + (w < h ? w : h), fs);
            max_base_x = w + h - 1;
        } else {
            for (int i = 0; i < w + h; i++) top[i] = E(e, 1 + i);
            max_base_x = w + (w < h ? w : h) - 1;
        }
    }
    const int base_inc = 1 + up;
    for (int y = 0, xpos = dx; y < h; y++, xpos += dx) {
        const int frac = xpos & 0x3E;
        for (int x = 0, base = xpos >> 6; x < w; x++, base += base_inc) {
            if (base < max_base_x) {
                D(dst, stride, y, x, (top[base] * (64 - frac) + top[base + 1] * frac + 32) >> 6, bpc);
            } else {
                for (; x < w; x++) D(dst, stride, y, x, top[max_base_x], bpc);
                break;
            }
        }
    }
}

static void z2(void *dst, ptrdiff_t stride, Edge e, int w, int h, int angle, int max_w, int max_h, int bpc) {
    const int bdmax = (1 << bpc) - 1;
    const int is_sm = (angle >> 9) & 1, eef = angle >> 10;
    angle &= 511;
    int dy = dr_intra_derivative[(angle - 90) >> 1];
    int dx = dr_intra_derivative[(180 - angle) >> 1];
    const int up_left = eef ? get_upsample(w + h, 180 - angle, is_sm) : 0;
    const int up_above = eef ? get_upsample(w + h, angle - 90, is_sm) : 0;
    int edge[64 + 64 + 1];
    int *const tl = &edge[64];
    if (up_above) {
        upsample_edge(tl, w + 1, e, 0, 0, w + 1, bdmax);
        dx <<= 1;
    } else {
        const int fs = eef ? filter_strength(w + h, angle - 90, is_sm) : 0;
        if (fs) filter_edge(&tl[1], w, 0, max_w, e, 1, -1, w, fs);
        else for (int i = 0; i < w; i++) tl[1 + i] = E(e, 1 + i);
    }
    if (up_left) {
        upsample_edge(&tl[-h * 2], h + 1, e, -h, 0, h + 1, bdmax);
        dy <<= 1;
    } else {
        const int fs = eef ? filter_strength(w + h, 180 - angle, is_sm) : 0;
        if (fs) filter_edge(&tl[-h], h, h - max_h, h, e, -h, 0, h + 1, fs);
        else for (int i = 0; i < h; i++) tl[-h + i] = E(e, -h + i);
    }
    *tl = E(e, 0);
    const int base_inc_x = 1 + up_above;
    const int *const left = &tl[-(1 + up_left)];
    for (int y = 0, xpos = ((1 + up_above) << 6) - dx; y < h; y++, xpos -= dx) {
        int base_x = xpos >> 6;
        const int frac_x = xpos & 0x3E;
        for (int x = 0, ypos = (y << (6 + up_left)) - dy; x < w; x++, base_x += base_inc_x, ypos -= dy) {
            int v;
            if (base_x >= 0) {
                v = tl[base_x] * (64 - frac_x) + tl[base_x + 1] * frac_x;
            } else {
                const int base_y = ypos >> 6;
                const int frac_y = ypos & 0x3E;
                v = left[-base_y] * (64 - frac_y) + left[-(base_y + 1)] * frac_y;
            }
            D(dst, stride, y, x, (v + 32) >> 6, bpc);
        }
    }
}

static void z3(void *dst, ptrdiff_t stride, Edge e, int w, int h, int angle, int bpc) {
    const int bdmax = (1 << bpc) - 1;
    const int is_sm = (angle >> 9) & 1, eef = angle >> 10;
    angle &= 511;
    int dy = dr_intra_derivative[(270 - angle) >> 1];
    int left_out[128 + 64];
    const int *left;
    int max_base_y;
    const int up = eef ? get_upsample(w + h, angle - 180, is_sm) : 0;
    int copied[128 + 1];
    if (up) {
        upsample_edge(left_out, w + h, e, -(w + h), w - h > 0 ? w - h : 0, w + h + 1, bdmax);
        left = &left_out[2 * (w + h) - 2];
        max_base_y = 2 * (w + h) - 2;
        dy <<= 1;
    } else {
        const int fs = eef ? filter_strength(w + h, angle - 180, is_sm) : 0;
        if (fs) {
            filter_edge(left_out, w + h, 0, w + h, e, -(w + h), w - h > 0 ? w - h : 0, w + h + 1, fs);
            left = &left_out[w + h - 1];
            max_base_y = w + h - 1;
        } else {
            /* left = &topleft_in[-1]: left[-k] = topleft[-1 - k] */
            for (int k = 0; k <= w + h; k++) copied[k] = E(e, -1 - k);
            left = NULL;
            max_base_y = h + (w < h ? w : h) - 1;
        }
    }
    const int base_inc = 1 + up;
#define LEFT(k) (left ? left[-(k)] : copied[(k)])
    for (int x = 0, ypos = dy; x < w; x++, ypos += dy) {
        const int frac = ypos & 0x3E;
        for (int y = 0, base = ypos >> 6; y < h; y++, base += base_inc) {
            if (base < max_base_y) {
                D(dst, stride, y, x, (LEFT(base) * (64 - frac) + LEFT(base + 1) * frac + 32) >> 6, bpc);
            } else {
                for (; y < h; y++) D(dst, stride, y, x, LEFT(max_base_y), bpc);
                break;
            }
        }
    }
#undef LEFT
}

/* ipred_filter_c (ipred_tmpl.c:618-655), generic tap layout taps[idx + 8 k] */
static void filter_pred(void *dst, ptrdiff_t stride, Edge e, int w, int h, int filt_idx, int bpc) {
    const int bdmax = (1 << bpc) - 1;
    filt_idx &= 511;
    const int8_t *flt = filter_intra_taps[filt_idx];
    for (int y = 0; y < h; y += 2) {
        for (int x = 0; x < w; x += 4) {
            /* p0 topleft, p1..p4 top, p5..p6 left (edge or previously predicted samples) */
            int p[7];
            p[0] = y ? (x ? Dget(dst, stride, y - 1, x - 1, bpc) : E(e, -y)) : E(e, x);
            for (int k = 0; k < 4; k++) p[1 + k] = y ? Dget(dst, stride, y - 1, x + k, bpc) : E(e, 1 + x + k);
            for (int k = 0; k < 2; k++) p[5 + k] = x ? Dget(dst, stride, y + k, x - 1, bpc) : E(e, -(1 + y + k));
            for (int yy = 0; yy < 2; yy++)
                for (int xx = 0; xx < 4; xx++) {
                    const int8_t *f = flt + yy * 4 + xx;
                    int acc = 0;
                    for (int k = 0; k < 7; k++) acc += f[8 * k] * p[k];
                    D(dst, stride, y + yy, x + xx, clip((acc + 8) >> 4, 0, bdmax), bpc);
                }
        }
    }
}

void oracle_intra_pred(int mode, void *dst, ptrdiff_t stride, const void *topleft, int w, int h,
                       int angle, int max_w, int max_h, int bpc) {
    const Edge e = { topleft, bpc };
    const int bdmax = (1 << bpc) - 1;
    switch (mode) {
    case 0: splat(dst, stride, w, h, (int)dc_both(e, w, h, bpc), bpc); break;
    case 1:
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) D(dst, stride, y, x, E(e, 1 + x), bpc);
        break;
    case 2:
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) D(dst, stride, y, x, E(e, -(1 + y)), bpc);
        break;
    case 3: splat(dst, stride, w, h, (int)dc_left(e, h), bpc); break;
    case 4: splat(dst, stride, w, h, (int)dc_top(e, w), bpc); break;
    case 5: splat(dst, stride, w, h, bpc == 8 ? 128 : (bdmax + 1) >> 1, bpc); break;
    case 6: z1(dst, stride, e, w, h, angle, bpc); break;
    case 7: z2(dst, stride, e, w, h, angle, max_w, max_h, bpc); break;
    case 8: z3(dst, stride, e, w, h, angle, bpc); break;
    case 9: {
        const uint8_t *wh = &sm_weights[w], *wv = &sm_weights[h];
        const int right = E(e, w), bottom = E(e, -h);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                const int pred = wv[y] * E(e, 1 + x) + (256 - wv[y]) * bottom + wh[x] * E(e, -(1 + y)) + (256 - wh[x]) * right;
                D(dst, stride, y, x, (pred + 256) >> 9, bpc);
            }
        break;
    }
    case 10: {
        const uint8_t *wv = &sm_weights[h];
        const int bottom = E(e, -h);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++)
                D(dst, stride, y, x, (wv[y] * E(e, 1 + x) + (256 - wv[y]) * bottom + 128) >> 8, bpc);
        break;
    }
    case 11: {
        const uint8_t *wh = &sm_weights[w];
        const int right = E(e, w);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++)
                D(dst, stride, y, x, (wh[x] * E(e, -(y + 1)) + (256 - wh[x]) * right + 128) >> 8, bpc);
        break;
    }
    case 12: {
        const int tl = E(e, 0);
        for (int y = 0; y < h; y++) {
            const int left = E(e, -(y + 1));
            for (int x = 0; x < w; x++) {
                const int top = E(e, 1 + x);
                const int base = left + top - tl;
                const int ld = abs(left - base), td = abs(top - base), tld = abs(tl - base);
                D(dst, stride, y, x, ld <= td && ld <= tld ? left : td <= tld ? top : tl, bpc);
            }
        }
        break;
    }
    case 13: filter_pred(dst, stride, e, w, h, angle, bpc); break;
    }
}

/* cfl_ac_c (ipred_tmpl.c:657-705) */
void oracle_cfl_ac(int16_t *ac, const void *ypx, ptrdiff_t stride, int w_pad, int h_pad, int cw, int ch,
                   int ss_hor, int ss_ver, int bpc) {
    int16_t *a = ac;
    int y, x;
    for (y = 0; y < ch - 4 * h_pad; y++) {
        for (x = 0; x < cw - 4 * w_pad; x++) {
            const int yy = y << ss_ver, xx = x << ss_hor;
            int s = Dget(ypx, stride, yy, xx, bpc);
            if (ss_hor) s += Dget(ypx, stride, yy, xx + 1, bpc);
            if (ss_ver) {
                s += Dget(ypx, stride, yy + 1, xx, bpc);
                if (ss_hor) s += Dget(ypx, stride, yy + 1, xx + 1, bpc);
            }
            a[x] = (int16_t)(s << (1 + !ss_ver + !ss_hor));
        }
        for (; x < cw; x++) a[x] = a[x - 1];
        a += cw;
    }
    for (; y < ch; y++) {
        memcpy(a, a - cw, (size_t)cw * sizeof(*a));
        a += cw;
    }
    const int log2sz = ctz(cw) + ctz(ch);
    int sum = (1 << log2sz) >> 1;
    for (int i = 0; i < cw * ch; i++) sum += ac[i];
    sum >>= log2sz;
    for (int i = 0; i < cw * ch; i++) ac[i] = (int16_t)(ac[i] - sum);
}

/* cfl_pred[mode] (mode 0 DC, 3 LEFT_DC, 4 TOP_DC, 5 DC_128; ipred_tmpl.c:71-84, 103-216) */
void oracle_cfl_pred(int mode, void *dst, ptrdiff_t stride, const void *topleft, int w, int h,
                     const int16_t *ac, int alpha, int bpc) {
    const Edge e = { topleft, bpc };
    const int bdmax = (1 << bpc) - 1;
    int dc;
    switch (mode) {
    case 0: dc = (int)dc_both(e, w, h, bpc); break;
    case 3: dc = (int)dc_left(e, h); break;
    case 4: dc = (int)dc_top(e, w); break;
    default: dc = bpc == 8 ? 128 : (bdmax + 1) >> 1; break;
    }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const int diff = alpha * ac[y * w + x];
            const int m = (abs(diff) + 32) >> 6;
            D(dst, stride, y, x, clip(dc + (diff < 0 ? -m : m), 0, bdmax), bpc);
        }
}

/* pal_pred_c (ipred_tmpl.c:717-727) */
void oracle_pal_pred(void *dst, ptrdiff_t stride, const void *pal, const uint8_t *idx, int w, int h, int bpc) {
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const int i = idx[y * w + x];
            D(dst, stride, y, x, bpc == 8 ? ((const uint8_t *)pal)[i] : ((const uint16_t *)pal)[i], bpc);
        }
}

/* ---- rav1d_prepare_intra_edges (src/ipred_prepare.rs:118-204; C ipred_prepare_tmpl.c) ----
 * In pixel units: x, y, the block's top-left; tile_w / tile_h the tile's column / row end
 * (the reference's w, h in 4-px units times 4); w, h the transform size. Fills topleft[-2h ..
 * 2w] and returns the implementation mode; *angle in: delta, out: the final angle. */
static const uint8_t needs_tab[14] = { 3, 2, 1, 1, 2, 0, 14, 7, 21, 3, 3, 3, 7, 7 };  /* :76-115 */
static const uint8_t mode_angle[8] = { 90, 180, 45, 135, 113, 157, 203, 67 };
enum { N_LEFT = 1, N_TOP = 2, N_TOP_LEFT = 4, N_TOP_RIGHT = 8, N_BOTTOM_LEFT = 16 };

int oracle_prepare_intra_edges(int x, int have_left, int y, int have_top, int tile_w, int tile_h,
                               int top_has_right, int left_has_bottom, const void *pic, ptrdiff_t stride,
                               int mode, int *angle, int w, int h, int filter_edge, void *topleft_, int bpc) {
    const int pb = bpc == 8 ? 1 : 2;
#define PIC(yy, xx) Dget((const uint8_t *)pic + (ptrdiff_t)(yy) * stride, 0, 0, (xx), bpc)
#define TL(i) Dget((const uint8_t *)topleft_ + (ptrdiff_t)(i) * pb, 0, 0, 0, bpc)
#define SET(i, v) D((uint8_t *)topleft_ + (ptrdiff_t)(i) * pb, 0, 0, 0, (v), bpc)
    if (mode >= 1 && mode <= 8) {                         /* VERT_PRED ..= VERT_LEFT_PRED */
        *angle = mode_angle[mode - 1] + 3 * *angle;
        if (*angle <= 90) mode = *angle < 90 && have_top ? 6 : 1;
        else if (*angle < 180) mode = 7;
        else mode = *angle > 180 && have_left ? 8 : 2;
    } else if (mode == 0) {                               /* av1_mode_conv */
        mode = have_left ? (have_top ? 0 : 3) : (have_top ? 4 : 5);
    } else if (mode == 12) {
        mode = have_left ? (have_top ? 12 : 2) : (have_top ? 1 : 5);
    }
    const int needs = needs_tab[mode];
    /* dst_top: row y - 1 starting at x - have_left */
    if (needs & N_LEFT) {
        const int sz = h;
        if (have_left) {
            const int px_have = sz < tile_h - y ? sz : tile_h - y;
            for (int i = 0; i < px_have; i++) SET(-1 - i, PIC(y + i, x - 1));
            for (int i = px_have; i < sz; i++) SET(-1 - i, TL(-px_have));
        } else {
            const int v = have_top ? PIC(y - 1, x) : (1 << bpc >> 1) + 1;
            for (int i = 0; i < sz; i++) SET(-1 - i, v);
        }
        if (needs & N_BOTTOM_LEFT) {
            const int hbl = !have_left || y + h >= tile_h ? 0 : left_has_bottom;
            if (hbl) {
                const int px_have = sz < tile_h - y - h ? sz : tile_h - y - h;
                for (int i = 0; i < px_have; i++) SET(-1 - sz - i, PIC(y + sz + i, x - 1));
                for (int i = px_have; i < sz; i++) SET(-1 - sz - i, TL(-sz - px_have));
            } else {
                const int v = TL(-sz);
                for (int i = 0; i < sz; i++) SET(-1 - sz - i, v);
            }
        }
    }
    if (needs & N_TOP) {
        const int sz = w;
        if (have_top) {
            const int px_have = sz < tile_w - x ? sz : tile_w - x;
            for (int i = 0; i < px_have; i++) SET(1 + i, PIC(y - 1, x + i));
            for (int i = px_have; i < sz; i++) SET(1 + i, TL(px_have));
        } else {
            const int v = have_left ? PIC(y, x - 1) : (1 << bpc >> 1) - 1;
            for (int i = 0; i < sz; i++) SET(1 + i, v);
        }
        if (needs & N_TOP_RIGHT) {
            const int htr = !have_top || x + w >= tile_w ? 0 : top_has_right;
            if (htr) {
                const int px_have = sz < tile_w - x - w ? sz : tile_w - x - w;
                for (int i = 0; i < px_have; i++) SET(1 + sz + i, PIC(y - 1, x + sz + i));
                for (int i = px_have; i < sz; i++) SET(1 + sz + i, TL(sz + px_have));
            } else {
                const int v = TL(sz);
                for (int i = 0; i < sz; i++) SET(1 + sz + i, v);
            }
        }
    }
    if (needs & N_TOP_LEFT) {
        int c = have_top ? PIC(y - 1, x - have_left) : have_left ? PIC(y, x - 1) : 1 << bpc >> 1;
        if (mode == 7 && (w >> 2) + (h >> 2) >= 6 && filter_edge) c = ((TL(-1) + TL(1)) * 5 + c * 6 + 8) >> 4;
        SET(0, c);
    }
#undef PIC
#undef TL
#undef SET
    return mode;
}

/* recon_b_intra's per-transform-block step (recon.rs:2470-2600, 2735-2859) over MiIntraBlock
 * records in order: palette, or prepare edges + intra_pred / cfl_pred, optionally blended
 * (inter-intra, mc.blend). Sequential, so each block sees its predecessors' pixels. */
typedef struct {
    uint16_t x, y;
    uint8_t w, h, plane, mode;
    int8_t angle;
    uint8_t flags, filt_idx;
    int8_t alpha;
    uint16_t tile_w, tile_h, max_w, max_h;
    uint32_t aux_off, pal_off, reserved;
} IntraBlock;   /* == MiIntraBlock, 32 bytes */

void oracle_intra_blocks(void *const planes[3], const ptrdiff_t strides[2], int bpc, const void *blocks, int n,
                         const int16_t *ac, const uint8_t *idx, const void *pal) {
    const IntraBlock *bl = blocks;
    const int pb = bpc == 8 ? 1 : 2;
    uint8_t edge[(2 * 128 + 1) * 2], tmp[64 * 64 * 2];
    for (int k = 0; k < n; k++) {
        const IntraBlock *b = &bl[k];
        if (b->mode == 97) continue;   /* MI_INTRA_RESID: the residual only (no prediction) */
        const ptrdiff_t st = strides[b->plane ? 1 : 0];
        uint8_t *dst = (uint8_t *)planes[b->plane] + b->y * st + b->x * pb;
        const int ii = b->flags & 64;
        uint8_t *out = ii ? tmp : dst;
        const ptrdiff_t ost = ii ? b->w * pb : st;
        if (b->mode == 96) {
            /* intra block copy: mc() with the current picture as reference, bilinear (recon.rs) */
            const int mvx = (int16_t)(b->reserved & 0xffff), mvy = (int16_t)(b->reserved >> 16);
            const int ssh = b->filt_idx & 1, ssv = (b->filt_idx >> 1) & 1;
            const int dx = b->x + (mvx >> (3 + ssh)), dy = b->y + (mvy >> (3 + ssv));
            const int mx = (mvx & (15 >> !ssh)) << !ssh, my = (mvy & (15 >> !ssv)) << !ssv;
            const uint8_t *src = (const uint8_t *)planes[b->plane] + (ptrdiff_t)dy * st + (ptrdiff_t)dx * pb;
            ptrdiff_t sst = st;
            /* recon.rs:2052-2083 (C recon_tmpl.c mc()): the intrabc reference area is
             * f.bw*4 >> ss_hor by f.bh*4 >> ss_ver (max_w x max_h here); a footprint leaving it
             * goes through emu_edge into a (bw+7) x (bh+7) scratch with the block at (3, 3) */
            static uint8_t emu[(128 + 7) * (128 + 7) * 2];
            if (dx < !!mx * 3 || dy < !!my * 3 || dx + b->w + !!mx * 4 > b->max_w || dy + b->h + !!my * 4 > b->max_h) {
                const ptrdiff_t es = (ptrdiff_t)(b->w + 7) * pb;
                oracle_mc_emu_edge(b->w + 7, b->h + 7, b->max_w, b->max_h, dx - 3, dy - 3, emu, es, planes[b->plane], st,
                                   bpc);
                src = emu + 3 * es + 3 * pb;
                sst = es;
            }
            oracle_mc_put(9, out, ost, src, sst, b->w, b->h, mx, my, bpc);
        } else if (b->mode == 64) {
            oracle_pal_pred(out, ost, (const uint8_t *)pal + (size_t)b->pal_off * pb, idx + b->aux_off, b->w, b->h, bpc);
        } else {
            const int cfl = b->mode == 32;
            int angle = b->angle;
            void *tl = edge + 128 * pb;
            const int m = oracle_prepare_intra_edges(b->x, b->flags & 1, b->y, (b->flags >> 1) & 1, b->tile_w, b->tile_h,
                                                     (b->flags >> 2) & 1, (b->flags >> 3) & 1, planes[b->plane], st,
                                                     cfl ? 0 : b->mode, &angle, b->w, b->h, (b->flags >> 5) & 1, tl, bpc);
            if (cfl && (b->flags & 128)) {
                /* MI_INTRA_CFL_AC: cfl_ac over the reconstructed luma under the block
                 * (recon.rs:2735-2800: the AC is taken from the luma just reconstructed) */
                int16_t acd[32 * 32];
                const int ssh = (b->reserved >> 16) & 1, ssv = (b->reserved >> 17) & 1;
                const uint8_t *yp = (const uint8_t *)planes[0] + (ptrdiff_t)(b->y << ssv) * strides[0] +
                                    (ptrdiff_t)(b->x << ssh) * pb;
                oracle_cfl_ac(acd, yp, strides[0], b->reserved & 0xff, (b->reserved >> 8) & 0xff, b->w, b->h, ssh, ssv,
                              bpc);
                oracle_cfl_pred(m, out, ost, tl, b->w, b->h, acd, b->alpha, bpc);
            } else if (cfl) {
                oracle_cfl_pred(m, out, ost, tl, b->w, b->h, ac + b->aux_off, b->alpha, bpc);
            } else {
                const int aw = m == 13 ? b->filt_idx : angle | ((b->flags & 16) ? 512 : 0) | ((b->flags & 32) ? 1024 : 0);
                oracle_intra_pred(m, out, ost, tl, b->w, b->h, aw, b->max_w, b->max_h, bpc);
            }
        }
        if (ii) {
            const uint8_t *mk = idx + b->aux_off;
            for (int y = 0; y < b->h; y++)
                for (int x = 0; x < b->w; x++) {
                    const int a = Dget(dst, st, y, x, bpc), t = Dget(tmp, ost, y, x, bpc), mm = mk[y * b->w + x];
                    D(dst, st, y, x, (a * (64 - mm) + t * mm + 32) >> 6, bpc);
                }
        }
    }
}

/* Interleaved intra reconstruction in decode order (recon.rs:2402-3160: for every transform
 * block, prepare_intra_edges + intra_pred / cfl_pred / pal_pred, then itxfm_add before the next
 * block reads its edges). tx_blocks[k] is the residual (MiTxBlock) of blocks[k]; the arena is
 * zeroed as the blocks consume it (itx.rs:152-158). */
void oracle_intra_recon(void *const planes[3], const ptrdiff_t strides[2], int bpc, const void *blocks,
                        const void *tx_blocks, int n, const int16_t *ac, const uint8_t *idx, const void *pal,
                        void *coef) {
    const ptrdiff_t st3[3] = {strides[0], strides[1], strides[1]};
    for (int k = 0; k < n; k++) {
        oracle_intra_blocks(planes, strides, bpc, (const IntraBlock *)blocks + k, 1, ac, idx, pal);
        oracle_itx_frame(planes, st3, (const uint8_t *)tx_blocks + 16 * k, 1, coef, (1 << bpc) - 1);
    }
}
