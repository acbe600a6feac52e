/*
 * oracle/filmgrain.c — CPU restatement of film-grain synthesis (TEST INFRASTRUCTURE ONLY).
 *
 * Follows FreezyLemon/rav1d:
 *   src/filmgrain.rs:255-282   get_random_number / row seeds (C src/filmgrain_tmpl.c:38-49)
 *   src/filmgrain.rs:298-474   generate_grain_y / generate_grain_uv (C filmgrain_tmpl.c:51-153)
 *   src/filmgrain.rs:503-830   sample_lut, fgy_32x32xn, fguv_32x32xn (C filmgrain_tmpl.c:165-413)
 *   src/fg_apply.rs:14-284     generate_scaling, prep_grain, apply_grain_row, apply_grain
 *                              (C src/fg_apply_tmpl.c:40-242)
 * The odd-width luma padding write into the *input* (fg_apply.rs:219-226) is performed on a
 * private copy of the input luma here, so the caller's input stays untouched.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define GW 82
#define GH 73
#define BS 32

static const int16_t gaussian_sequence[2048] = {
#include "../rav1d_amd/csrc/tables/gaussian_sequence.inc"
};

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int iclip(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* Dav1dFilmGrainData (include/dav1d/headers.h:315-333) */
typedef struct {
    unsigned seed;
    int num_y_points;
    uint8_t y_points[14][2];
    int chroma_scaling_from_luma;
    int num_uv_points[2];
    uint8_t uv_points[2][10][2];
    int scaling_shift;
    int ar_coeff_lag;
    int8_t ar_coeffs_y[24];
    int8_t ar_coeffs_uv[2][25 + 3];
    uint64_t ar_coeff_shift;
    int grain_scale_shift;
    int uv_mult[2];
    int uv_luma_mult[2];
    int uv_offset[2];
    int overlap_flag;
    int clip_to_restricted_range;
} FGData;

static inline int get_random_number(int bits, unsigned *state)
{
    const int r = (int)*state;
    const unsigned bit = ((r >> 0) ^ (r >> 1) ^ (r >> 3) ^ (r >> 12)) & 1;
    *state = ((unsigned)r >> 1) | (bit << 15);
    return (int)((*state >> (16 - bits)) & ((1u << bits) - 1));
}

static inline int round2(int x, int shift) { return (x + ((1 << shift) >> 1)) >> shift; }

/* generate_grain_y (filmgrain.rs:298-343). buf: [GH][GW] int16 */
void oracle_fg_generate_grain_y(int16_t *buf, const void *data_, int bdmax)
{
    const FGData *data = data_;
    const int bdm8 = bdmax == 255 ? 0 : bdmax == 1023 ? 2 : 4;
    unsigned seed = data->seed;
    const int shift = 4 - bdm8 + data->grain_scale_shift;
    const int gctr = 128 << bdm8, gmin = -gctr, gmax = gctr - 1;
    for (int y = 0; y < GH; y++)
        for (int x = 0; x < GW; x++)
            buf[y * GW + x] = (int16_t)round2(gaussian_sequence[get_random_number(11, &seed)], shift);
    const int lag = data->ar_coeff_lag;
    for (int y = 3; y < GH; y++)
        for (int x = 3; x < GW - 3; x++) {
            const int8_t *c = data->ar_coeffs_y;
            int sum = 0;
            for (int dy = -lag; dy <= 0; dy++)
                for (int dx = -lag; dx <= lag; dx++) {
                    if (!dx && !dy) break;
                    sum += *c++ * buf[(y + dy) * GW + x + dx];
                }
            buf[y * GW + x] = (int16_t)iclip(buf[y * GW + x] + round2(sum, (int)data->ar_coeff_shift), gmin, gmax);
        }
}

/* generate_grain_uv (filmgrain.rs:345-474) */
void oracle_fg_generate_grain_uv(int16_t *buf, const int16_t *buf_y, const void *data_, int uv,
                                 int subx, int suby, int bdmax)
{
    const FGData *data = data_;
    const int bdm8 = bdmax == 255 ? 0 : bdmax == 1023 ? 2 : 4;
    unsigned seed = data->seed ^ (uv ? 0x49d8 : 0xb524);
    const int shift = 4 - bdm8 + data->grain_scale_shift;
    const int gctr = 128 << bdm8, gmin = -gctr, gmax = gctr - 1;
    const int cw = subx ? 44 : GW, chh = suby ? 38 : GH;
    for (int y = 0; y < chh; y++)
        for (int x = 0; x < cw; x++)
            buf[y * GW + x] = (int16_t)round2(gaussian_sequence[get_random_number(11, &seed)], shift);
    const int lag = data->ar_coeff_lag;
    for (int y = 3; y < chh; y++)
        for (int x = 3; x < cw - 3; x++) {
            const int8_t *c = data->ar_coeffs_uv[uv];
            int sum = 0;
            for (int dy = -lag; dy <= 0; dy++)
                for (int dx = -lag; dx <= lag; dx++) {
                    if (!dx && !dy) {
                        if (!data->num_y_points) break;
                        int luma = 0;
                        const int lx = ((x - 3) << subx) + 3, ly = ((y - 3) << suby) + 3;
                        for (int i = 0; i <= suby; i++)
                            for (int j = 0; j <= subx; j++) luma += buf_y[(ly + i) * GW + lx + j];
                        luma = round2(luma, subx + suby);
                        sum += luma * *c;
                        break;
                    }
                    sum += *c++ * buf[(y + dy) * GW + x + dx];
                }
            buf[y * GW + x] = (int16_t)iclip(buf[y * GW + x] + round2(sum, (int)data->ar_coeff_shift), gmin, gmax);
        }
}

/* generate_scaling (fg_apply.rs:14-72) */
void oracle_fg_generate_scaling(int bitdepth, const uint8_t (*points)[2], int num, uint8_t *scaling)
{
    const int shift_x = bitdepth - 8;
    const int size = 1 << bitdepth;
    if (num == 0) { memset(scaling, 0, size); return; }
    memset(scaling, points[0][1], (size_t)points[0][0] << shift_x);
    for (int i = 0; i < num - 1; i++) {
        const int bx = points[i][0], by = points[i][1], ex = points[i + 1][0], ey = points[i + 1][1];
        const int dx = ex - bx, dy = ey - by;
        const int delta = dy * ((0x10000 + (dx >> 1)) / dx);
        for (int x = 0, d = 0x8000; x < dx; x++) {
            scaling[(bx + x) << shift_x] = (uint8_t)(by + (d >> 16));
            d += delta;
        }
    }
    const int n = points[num - 1][0] << shift_x;
    memset(&scaling[n], points[num - 1][1], size - n);
    if (bitdepth > 8) {
        const int pad = 1 << shift_x, rnd = pad >> 1;
        for (int i = 0; i < num - 1; i++) {
            const int bx = points[i][0] << shift_x, ex = points[i + 1][0] << shift_x;
            const int dx = ex - bx;
            for (int x = 0; x < dx; x += pad) {
                const int range = scaling[bx + x + pad] - scaling[bx + x];
                for (int k = 1, r = rnd; k < pad; k++) {
                    r += range;
                    scaling[bx + x + k] = (uint8_t)(scaling[bx + x] + (r >> shift_x));
                }
            }
        }
    }
}

typedef struct { int hbd, bdmax, bdm8; } FPX;
static inline int RDp(const FPX *p, const uint8_t *b, ptrdiff_t i) { return p->hbd ? ((const uint16_t *)b)[i] : b[i]; }
static inline void WRp(const FPX *p, uint8_t *b, ptrdiff_t i, int v)
{ if (p->hbd) ((uint16_t *)b)[i] = (uint16_t)v; else b[i] = (uint8_t)v; }

static inline int sample_lut(const int16_t *lut, const int off[2][2], int subx, int suby, int bx, int by, int x, int y)
{
    const int rv = off[bx][by];
    const int ox = 3 + (2 >> subx) * (3 + (rv >> 4));
    const int oy = 3 + (2 >> suby) * (3 + (rv & 0xF));
    return lut[(oy + y + (BS >> suby) * by) * GW + ox + x + (BS >> subx) * bx];
}

/* fgy_32x32xn / fguv_32x32xn (filmgrain.rs:549-830), unified: luma when `luma_row` is NULL */
static void fg_row(const FPX *px, uint8_t *dst_row, const uint8_t *src_row, ptrdiff_t ps,
                   const FGData *data, int pw, const uint8_t *scaling, const int16_t *lut, int bh,
                   int row_num, const uint8_t *luma_row, ptrdiff_t lps, int uv, int is_id, int sx, int sy)
{
    const int luma = luma_row == NULL;
    const int rows = 1 + (data->overlap_flag && row_num > 0);
    const int gctr = 128 << px->bdm8, gmin = -gctr, gmax = gctr - 1;
    int minv, maxv;
    if (data->clip_to_restricted_range) {
        minv = 16 << px->bdm8;
        maxv = (luma ? 235 : (is_id ? 235 : 240)) << px->bdm8;
    } else {
        minv = 0;
        maxv = px->bdmax;
    }
    unsigned seed[2];
    for (int i = 0; i < rows; i++) {
        seed[i] = data->seed;
        seed[i] ^= (unsigned)((((row_num - i) * 37 + 178) & 0xFF) << 8);
        seed[i] ^= (unsigned)(((row_num - i) * 173 + 105) & 0xFF);
    }
    int off[2][2] = { { 0, 0 }, { 0, 0 } };
    static const int wl[2][2] = { { 27, 17 }, { 17, 27 } };
    static const int wc[2][2][2] = { { { 27, 17 }, { 17, 27 } }, { { 23, 22 }, { 0, 0 } } };
    const int bsw = BS >> sx;
    for (int bx = 0; bx < pw; bx += bsw) {
        const int bw = imin(bsw, pw - bx);
        if (data->overlap_flag && bx)
            for (int i = 0; i < rows; i++) off[1][i] = off[0][i];
        for (int i = 0; i < rows; i++) off[0][i] = get_random_number(8, &seed[i]);
        const int ystart = data->overlap_flag && row_num ? imin(2 >> sy, bh) : 0;
        const int xstart = data->overlap_flag && bx ? imin(2 >> sx, bw) : 0;
        for (int y = 0; y < bh; y++)
            for (int x = 0; x < bw; x++) {
                int grain;
                const int wx0 = luma ? wl[x & 1][0] : wc[sx][x & 1][0], wx1 = luma ? wl[x & 1][1] : wc[sx][x & 1][1];
                const int wy0 = luma ? wl[y & 1][0] : wc[sy][y & 1][0], wy1 = luma ? wl[y & 1][1] : wc[sy][y & 1][1];
                if (y >= ystart && x >= xstart) {
                    grain = sample_lut(lut, off, sx, sy, 0, 0, x, y);
                } else if (y >= ystart) {
                    grain = sample_lut(lut, off, sx, sy, 0, 0, x, y);
                    const int old = sample_lut(lut, off, sx, sy, 1, 0, x, y);
                    grain = iclip(round2(old * wx0 + grain * wx1, 5), gmin, gmax);
                } else if (x >= xstart) {
                    grain = sample_lut(lut, off, sx, sy, 0, 0, x, y);
                    const int old = sample_lut(lut, off, sx, sy, 0, 1, x, y);
                    grain = iclip(round2(old * wy0 + grain * wy1, 5), gmin, gmax);
                } else {
                    int top = sample_lut(lut, off, sx, sy, 0, 1, x, y);
                    int old = sample_lut(lut, off, sx, sy, 1, 1, x, y);
                    top = iclip(round2(old * wx0 + top * wx1, 5), gmin, gmax);
                    grain = sample_lut(lut, off, sx, sy, 0, 0, x, y);
                    old = sample_lut(lut, off, sx, sy, 1, 0, x, y);
                    grain = iclip(round2(old * wx0 + grain * wx1, 5), gmin, gmax);
                    grain = iclip(round2(top * wy0 + grain * wy1, 5), gmin, gmax);
                }
                const int s = RDp(px, src_row, y * ps + bx + x);
                int val = s;
                if (!luma) {
                    const int lx = (bx + x) << sx, ly = y << sy;
                    int avg = RDp(px, luma_row, ly * lps + lx);
                    if (sx) avg = (avg + RDp(px, luma_row, ly * lps + lx + 1) + 1) >> 1;
                    val = avg;
                    if (!data->chroma_scaling_from_luma) {
                        const int combined = avg * data->uv_luma_mult[uv] + s * data->uv_mult[uv];
                        val = iclip((combined >> 6) + data->uv_offset[uv] * (1 << px->bdm8), 0, px->bdmax);
                    }
                }
                const int noise = round2(scaling[val] * grain, data->scaling_shift);
                WRp(px, dst_row, y * ps + bx + x, iclip(s + noise, minv, maxv));
            }
    }
}

/* rav1d_apply_grain (fg_apply.rs:272-284): out = in + grain. Planes are (rows, stride) with
 * 128-aligned rows; `in` is not modified (the odd-width luma padding goes to a copy). */
void oracle_fg_apply(void *const out[3], void *const in[3], const ptrdiff_t strides[3], int w, int h,
                     int layout, int bpc, const void *data_, int is_id)
{
    const FGData *data = data_;
    FPX px = { bpc > 8, (1 << bpc) - 1, bpc - 8 };
    const int bdmax = px.bdmax;
    static _Thread_local int16_t lut[3][GH + 1][GW];
    static _Thread_local uint8_t scaling[3][4096];
    const int ss_y = layout == 1, ss_x = layout == 1 || layout == 2;

    oracle_fg_generate_grain_y(&lut[0][0][0], data, bdmax);
    if (layout && (data->num_uv_points[0] || data->chroma_scaling_from_luma))
        oracle_fg_generate_grain_uv(&lut[1][0][0], &lut[0][0][0], data, 0, ss_x, ss_y, bdmax);
    if (layout && (data->num_uv_points[1] || data->chroma_scaling_from_luma))
        oracle_fg_generate_grain_uv(&lut[2][0][0], &lut[0][0][0], data, 1, ss_x, ss_y, bdmax);
    if (data->num_y_points || data->chroma_scaling_from_luma)
        oracle_fg_generate_scaling(bpc, data->y_points, data->num_y_points, scaling[0]);
    if (data->num_uv_points[0])
        oracle_fg_generate_scaling(bpc, data->uv_points[0], data->num_uv_points[0], scaling[1]);
    if (data->num_uv_points[1])
        oracle_fg_generate_scaling(bpc, data->uv_points[1], data->num_uv_points[1], scaling[2]);

    /* planes that get no grain are copied (prep_grain, fg_apply.rs:130-170) */
    const int rows_y = (h + 127) & ~127;
    const int nplanes = layout ? 3 : 1;
    for (int p = 0; p < nplanes; p++)
        memcpy(out[p], in[p], (size_t)(p ? rows_y >> ss_y : rows_y) * strides[p]);
    /* private luma copy for the odd-width padding write */
    uint8_t *luma_in = malloc((size_t)rows_y * strides[0]);
    memcpy(luma_in, in[0], (size_t)rows_y * strides[0]);

    const int pxb = px.hbd ? 2 : 1;
    const int cpw = (w + ss_x) >> ss_x;
    const int nrows = (h + 31) >> 5;
    for (int row = 0; row < nrows; row++) {
        uint8_t *lsrc = luma_in + (ptrdiff_t)row * BS * strides[0];
        if (data->num_y_points) {
            const int bh = imin(h - row * BS, BS);
            fg_row(&px, (uint8_t *)out[0] + (ptrdiff_t)row * BS * strides[0], lsrc, strides[0] / pxb,
                   data, w, scaling[0], &lut[0][0][0], bh, row, NULL, 0, 0, 0, 0, 0);
        }
        if (!layout || (!data->num_uv_points[0] && !data->num_uv_points[1] && !data->chroma_scaling_from_luma))
            continue;
        const int bh = (imin(h - row * BS, BS) + ss_y) >> ss_y;
        if (w & ss_x) {
            for (int y = 0; y < bh; y++) {
                uint8_t *r = lsrc + (ptrdiff_t)(y << ss_y) * strides[0];
                WRp(&px, r, w, RDp(&px, r, w - 1));
            }
        }
        const ptrdiff_t uv_off = ((ptrdiff_t)row * BS >> ss_y) * strides[1];
        for (int pl = 0; pl < 2; pl++) {
            if (!data->chroma_scaling_from_luma && !data->num_uv_points[pl]) continue;
            const uint8_t *scl = data->chroma_scaling_from_luma ? scaling[0] : scaling[1 + pl];
            fg_row(&px, (uint8_t *)out[1 + pl] + uv_off, (const uint8_t *)in[1 + pl] + uv_off, strides[1] / pxb,
                   data, cpw, scl, &lut[1 + pl][0][0], bh, row, lsrc, strides[0] / pxb, pl, is_id, ss_x, ss_y);
        }
    }
    free(luma_in);
}

/* Per-call fgy_32x32xn (pl 0) / fguv_32x32xn (pl 1 + uv) (filmgrain.rs:87-191, 549-830): one
 * strip; strides in bytes; lut = the plane's template as int16 [73][82]; layout 1..3. */
void oracle_fg_32x32xn(int pl, int layout, void *dst_row, const void *src_row, ptrdiff_t stride, const void *data,
                       int pw, const uint8_t *scaling, const int16_t *lut, int bh, int row_num,
                       const void *luma_row, ptrdiff_t luma_stride, int is_id, int bdmax)
{
    FPX px = { bdmax > 255, bdmax, bdmax == 255 ? 0 : bdmax == 1023 ? 2 : 4 };
    const int pxb = px.hbd ? 2 : 1;
    const int sx = pl && layout != 3, sy = pl && layout == 1;
    fg_row(&px, dst_row, src_row, stride / pxb, data, pw, scaling, lut, bh, row_num,
           pl ? luma_row : NULL, luma_stride / pxb, pl ? pl - 1 : 0, is_id, sx, sy);
}
