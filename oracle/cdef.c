/*
 * oracle/cdef.c — CPU restatement of CDEF (TEST INFRASTRUCTURE ONLY).
 *
 * Follows FreezyLemon/rav1d:
 *   src/cdef.rs:545-565    constrain (C src/cdef_tmpl.c:37-42)
 *   src/cdef.rs:567-665    padding   (C cdef_tmpl.c:55-117): unavailable samples = i16::MIN
 *   src/cdef.rs:668-820    cdef_filter_block (C cdef_tmpl.c:119-240)
 *   src/cdef.rs:921-1031   cdef_find_dir (C cdef_tmpl.c:261-331)
 *   src/cdef_apply.rs:145-507  adjust_strength + rav1d_cdef_brow (C src/cdef_apply_tmpl.c:95-309)
 *
 * Frame driver. rav1d_cdef_brow filters in place and keeps line/column backups
 * (cdef_apply.rs:36-143, 202-303) so that every 8x8 block reads only pre-CDEF (deblocked)
 * samples. The driver here states that contract directly: it reads an immutable deblocked
 * picture `src` and writes `dst`; blocks the reference skips are copied.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline unsigned umin(unsigned a, unsigned b) { return a < b ? a : b; }
static inline int iclip(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
static inline int ulog2(unsigned v) { return 31 - __builtin_clz(v); }

enum { HAVE_LEFT = 1, HAVE_RIGHT = 2, HAVE_TOP = 4, HAVE_BOTTOM = 8 };

/* (dy, dx) per direction and tap distance (dav1d_cdef_directions, src/tables.rs:698) */
static const int8_t cdef_dir_dydx[8][2][2] = {
    { { -1, 1 }, { -2, 2 } }, { { 0, 1 }, { -1, 2 } }, { { 0, 1 }, { 0, 2 } }, { { 0, 1 }, { 1, 2 } },
    { { 1, 1 }, { 2, 2 } },   { { 1, 0 }, { 2, 1 } },  { { 1, 0 }, { 2, 0 } }, { { 1, 0 }, { 2, -1 } },
};
#define TS 12
static inline int doff(int dir, int k) { return cdef_dir_dydx[dir & 7][k][0] * TS + cdef_dir_dydx[dir & 7][k][1]; }

static inline int constrain(int diff, int threshold, int shift)
{
    const int adiff = abs(diff);
    const int v = imin(adiff, imax(0, threshold - (adiff >> shift)));
    return diff < 0 ? -v : v;
}

static inline int px_at(const uint8_t *p, ptrdiff_t i, int hbd)
{
    return hbd ? ((const uint16_t *)p)[i] : p[i];
}

/* padding (cdef.rs:567-665): builds the (h+4) x (w+4) int16 window, stride 12. */
static void padding(int16_t *tmp, const uint8_t *src, ptrdiff_t ps, const uint8_t *left /* [h][2] px */,
                    const uint8_t *top, const uint8_t *bottom, int w, int h, int edges, int hbd)
{
    int x0 = -2, x1 = w + 2, y0 = -2, y1 = h + 2;
    for (int y = -2; y < h + 2; y++)
        for (int x = -2; x < w + 2; x++) tmp[y * TS + x] = INT16_MIN;
    if (!(edges & HAVE_TOP)) y0 = 0;
    if (!(edges & HAVE_BOTTOM)) y1 -= 2;
    if (!(edges & HAVE_LEFT)) x0 = 0;
    if (!(edges & HAVE_RIGHT)) x1 -= 2;
    for (int y = y0; y < 0; y++)
        for (int x = x0; x < x1; x++) tmp[y * TS + x] = (int16_t)px_at(top, (y + 2) * ps + x, hbd);
    for (int y = 0; y < h; y++)
        for (int x = x0; x < 0; x++) tmp[y * TS + x] = (int16_t)px_at(left, y * 2 + 2 + x, hbd);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < x1; x++) tmp[y * TS + x] = (int16_t)px_at(src, y * ps + x, hbd);
    for (int y = h; y < y1; y++)
        for (int x = x0; x < x1; x++) tmp[y * TS + x] = (int16_t)px_at(bottom, (y - h) * ps + x, hbd);
}

/* cdef_filter_block (cdef.rs:668-820). `src` is the block's input; output written to `dst`
 * (the reference filters in place: dst == src). */
void oracle_cdef_filter_block(void *dst_, ptrdiff_t dst_stride, const void *src_, ptrdiff_t src_stride,
                              const void *left, const void *top, const void *bottom, int pri, int sec,
                              int dir, int damping, int w, int h, int edges, int bdmax)
{
    const int hbd = bdmax > 255;
    const int pxb = hbd ? 2 : 1;
    const ptrdiff_t ps = src_stride / pxb, pd = dst_stride / pxb;
    int16_t buf[TS * TS];
    int16_t *tmp = buf + 2 * TS + 2;
    padding(tmp, src_, ps, left, top, bottom, w, h, edges, hbd);
    const int bdm8 = bdmax == 255 ? 0 : bdmax == 1023 ? 2 : 4;
    uint8_t *d8 = dst_;
    uint16_t *d16 = dst_;

    const int pri_tap = 4 - ((pri >> bdm8) & 1);
    const int pri_shift = pri ? imax(0, damping - ulog2(pri)) : 0;
    const int sec_shift = sec ? damping - ulog2(sec) : 0;
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++) {
            const int c = tmp[y * TS + x];
            int sum = 0, mx = c;
            unsigned mn = (unsigned)c;
            if (pri) {
                int tap = pri_tap;
                for (int k = 0; k < 2; k++) {
                    const int o = doff(dir, k);
                    const int a = tmp[y * TS + x + o], b = tmp[y * TS + x - o];
                    sum += tap * constrain(a - c, pri, pri_shift);
                    sum += tap * constrain(b - c, pri, pri_shift);
                    tap = (tap & 3) | 2;
                    mn = umin((unsigned)a, mn); mx = imax(a, mx);
                    mn = umin((unsigned)b, mn); mx = imax(b, mx);
                }
            }
            if (sec) {
                for (int k = 0; k < 2; k++) {
                    const int o2 = doff(dir + 2, k), o3 = doff(dir + 6, k);
                    const int s0 = tmp[y * TS + x + o2], s1 = tmp[y * TS + x - o2];
                    const int s2 = tmp[y * TS + x + o3], s3 = tmp[y * TS + x - o3];
                    const int tap = 2 - k;
                    sum += tap * constrain(s0 - c, sec, sec_shift);
                    sum += tap * constrain(s1 - c, sec, sec_shift);
                    sum += tap * constrain(s2 - c, sec, sec_shift);
                    sum += tap * constrain(s3 - c, sec, sec_shift);
                    mn = umin((unsigned)s0, mn); mx = imax(s0, mx);
                    mn = umin((unsigned)s1, mn); mx = imax(s1, mx);
                    mn = umin((unsigned)s2, mn); mx = imax(s2, mx);
                    mn = umin((unsigned)s3, mn); mx = imax(s3, mx);
                }
            }
            int v = c + ((sum - (sum < 0) + 8) >> 4);
            /* min/max clamping only when both strengths are active (cdef.rs:700-760) */
            if (pri && sec) v = iclip(v, (int)mn, mx);
            if (hbd) d16[y * pd + x] = (uint16_t)v;
            else d8[y * pd + x] = (uint8_t)v;
        }
    }
}

/* cdef_find_dir (cdef.rs:921-1031) */
int oracle_cdef_find_dir(const void *img_, ptrdiff_t stride, unsigned *var, int bdmax)
{
    const int hbd = bdmax > 255;
    const ptrdiff_t ps = stride / (hbd ? 2 : 1);
    const int bdm8 = bdmax == 255 ? 0 : bdmax == 1023 ? 2 : 4;
    int hv[2][8] = { { 0 } }, dg[2][15] = { { 0 } }, alt[4][11] = { { 0 } };
    for (int y = 0; y < 8; y++) {
        for (int x = 0; x < 8; x++) {
            const int p = (px_at(img_, y * ps + x, hbd) >> bdm8) - 128;
            dg[0][y + x] += p;
            alt[0][y + (x >> 1)] += p;
            hv[0][y] += p;
            alt[1][3 + y - (x >> 1)] += p;
            dg[1][7 + y - x] += p;
            alt[2][3 - (y >> 1) + x] += p;
            hv[1][x] += p;
            alt[3][(y >> 1) + x] += p;
        }
    }
    static const unsigned div_table[7] = { 840, 420, 280, 210, 168, 140, 120 };
    unsigned cost[8] = { 0 };
    for (int n = 0; n < 8; n++) {
        cost[2] += (unsigned)(hv[0][n] * hv[0][n]);
        cost[6] += (unsigned)(hv[1][n] * hv[1][n]);
    }
    cost[2] *= 105;
    cost[6] *= 105;
    for (int n = 0; n < 7; n++) {
        cost[0] += (unsigned)(dg[0][n] * dg[0][n] + dg[0][14 - n] * dg[0][14 - n]) * div_table[n];
        cost[4] += (unsigned)(dg[1][n] * dg[1][n] + dg[1][14 - n] * dg[1][14 - n]) * div_table[n];
    }
    cost[0] += (unsigned)(dg[0][7] * dg[0][7]) * 105;
    cost[4] += (unsigned)(dg[1][7] * dg[1][7]) * 105;
    for (int n = 0; n < 4; n++) {
        unsigned c = 0;
        for (int m = 0; m < 5; m++) c += (unsigned)(alt[n][3 + m] * alt[n][3 + m]);
        c *= 105;
        for (int m = 0; m < 3; m++)
            c += (unsigned)(alt[n][m] * alt[n][m] + alt[n][10 - m] * alt[n][10 - m]) * div_table[2 * m + 1];
        cost[2 * n + 1] += c;
    }
    int best = 0;
    unsigned best_cost = cost[0];
    for (int n = 1; n < 8; n++)
        if (cost[n] > best_cost) { best_cost = cost[n]; best = n; }
    *var = (best_cost - cost[best ^ 4]) >> 10;
    return best;
}

/* adjust_strength (cdef_apply.rs:145-157) */
static int adjust_strength(int strength, unsigned var)
{
    if (!var) return 0;
    const int i = var >> 6 ? imin(ulog2(var >> 6), 12) : 0;
    return (strength * (4 + i) + 8) >> 4;
}

typedef struct {
    uint16_t filter_y[2][32][3][2];
    uint16_t filter_uv[2][32][2][2];
    int8_t cdef_idx[4];
    uint16_t noskip_mask[16][2];
} OAv1Filter;

/* Whole-frame CDEF: src = deblocked picture (read only), dst = output picture.
 * y_strength/uv_strength: frame_hdr.cdef.{y,uv}_strength[8]; damping: frame_hdr.cdef.damping. */
void oracle_cdef_frame(void *const dst[3], void *const src[3], const ptrdiff_t strides[3], int w,
                       int h, int layout, int bpc, const void *masks_, int sb128w, int damping_hdr,
                       const uint8_t *y_strength, const uint8_t *uv_strength)
{
    const OAv1Filter *masks = masks_;
    const int bdmax = (1 << bpc) - 1, hbd = bpc > 8, pxb = hbd ? 2 : 1;
    const int bdm8 = bpc - 8;
    const int bw = ((w + 7) >> 3) << 1, bh = ((h + 7) >> 3) << 1;
    const int ss_ver = layout == 1, ss_hor = layout == 1 || layout == 2;
    const int uv_w = 8 >> ss_hor, uv_h = 8 >> ss_ver;
    static const uint8_t uv_dirs[2][8] = { { 0, 1, 2, 3, 4, 5, 6, 7 }, { 7, 0, 2, 4, 5, 6, 6, 6 } };
    const uint8_t *uv_dir = uv_dirs[layout == 2];
    const int damping = damping_hdr + bdm8;
    const int nplanes = layout ? 3 : 1;

    /* start from a copy of the deblocked picture (skipped blocks stay deblocked) */
    const int rows_y = (h + 127) & ~127;
    for (int p = 0; p < nplanes; p++) {
        const int rows = p ? rows_y >> ss_ver : rows_y;
        memcpy(dst[p], src[p], (size_t)rows * strides[p]);
    }

    for (int by = 0; by < bh; by += 2) {
        for (int bx = 0; bx < bw; bx += 2) {
            const OAv1Filter *lf = &masks[(by >> 5) * sb128w + (bx >> 5)];
            const int sb64_idx = ((by & 16) >> 3) + ((bx >> 4) & 1);
            const int cdef_idx = lf->cdef_idx[sb64_idx];
            if (cdef_idx == -1 || (!y_strength[cdef_idx] && !uv_strength[cdef_idx])) continue;
            const int by_idx = (by & 30) >> 1;
            const unsigned noskip = (unsigned)lf->noskip_mask[by_idx][1] << 16 | lf->noskip_mask[by_idx][0];
            if (!(noskip & (3u << (bx & 30)))) continue;

            const int y_lvl = y_strength[cdef_idx], uv_lvl = uv_strength[cdef_idx];
            const int y_pri = (y_lvl >> 2) << bdm8;
            int y_sec = y_lvl & 3;
            y_sec += y_sec == 3;
            y_sec <<= bdm8;
            const int uv_pri = (uv_lvl >> 2) << bdm8;
            int uv_sec = uv_lvl & 3;
            uv_sec += uv_sec == 3;
            uv_sec <<= bdm8;

            const int edges = (bx > 0 ? HAVE_LEFT : 0) | (bx + 2 < bw ? HAVE_RIGHT : 0) |
                              (by > 0 ? HAVE_TOP : 0) | (by + 2 < bh ? HAVE_BOTTOM : 0);
            int dir = 0;
            unsigned var = 0;
            const uint8_t *sy = (const uint8_t *)src[0] + (ptrdiff_t)by * 4 * strides[0] + (ptrdiff_t)bx * 4 * pxb;
            if (y_pri || uv_pri) dir = oracle_cdef_find_dir(sy, strides[0], &var, bdmax);

            for (int p = 0; p < nplanes; p++) {
                if (p && !uv_lvl) break;
                const int bw_ = p ? uv_w : 8, bh_ = p ? uv_h : 8;
                const int x = p ? (bx * 4) >> ss_hor : bx * 4, y = p ? (by * 4) >> ss_ver : by * 4;
                int pri, sec, d, damp;
                if (!p) {
                    if (y_pri) {
                        pri = adjust_strength(y_pri, var);
                        sec = y_sec;
                        d = dir;
                        if (!pri && !sec) continue;
                    } else if (y_sec) {
                        pri = 0; sec = y_sec; d = 0;
                    } else continue;
                    damp = damping;
                } else {
                    pri = uv_pri; sec = uv_sec;
                    d = uv_pri ? uv_dir[dir] : 0;
                    damp = damping - 1;
                }
                const ptrdiff_t st = strides[p];
                const uint8_t *s = (const uint8_t *)src[p] + (ptrdiff_t)y * st + (ptrdiff_t)x * pxb;
                uint8_t left[8 * 2 * 2];
                for (int r = 0; r < bh_; r++)
                    memcpy(left + r * 2 * pxb, s + r * st - 2 * pxb, 2 * pxb);
                uint8_t *dd = (uint8_t *)dst[p] + (ptrdiff_t)y * st + (ptrdiff_t)x * pxb;
                oracle_cdef_filter_block(dd, st, s, st, left, s - 2 * st, s + bh_ * st, pri, sec, d,
                                         damp, bw_, bh_, edges, bdmax);
            }
        }
    }
}
