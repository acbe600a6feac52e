/*
 * oracle/loopfilter.c — CPU restatement of the deblocking filter (TEST INFRASTRUCTURE ONLY).
 *
 * Follows FreezyLemon/rav1d:
 *   src/loopfilter.rs:396-721   loop_filter (C src/loopfilter_tmpl.c:37-160)
 *   src/loopfilter.rs:745-985   loop_filter_{h,v}_sb128{y,uv} (C loopfilter_tmpl.c:162-250)
 *   src/lf_apply.rs:388-834     filter_plane_{cols,rows}_{y,uv}, rav1d_loopfilter_sbrow_{cols,rows}
 *                               (C src/lf_apply_tmpl.c:174-466)
 * The frame driver walks superblock rows in the reference's order (columns then rows per
 * sbrow, src/recon.rs:4319-4338). Tile-boundary mask fixups (lf_apply.rs:625-705) are a
 * property of the input masks here: callers pass masks with the fixups already applied.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int iclip(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

typedef struct {
    int hbd, bdmax, bdm8;
} Px;

static inline int rd(const Px *px, const uint8_t *base, ptrdiff_t off)
{
    return px->hbd ? ((const uint16_t *)base)[off] : base[off];
}
static inline void wr(const Px *px, uint8_t *base, ptrdiff_t off, int v)
{
    if (px->hbd) ((uint16_t *)base)[off] = (uint16_t)v;
    else base[off] = (uint8_t)v;
}

/* One 4-line edge segment. `dst` points at q0 of line 0; sa steps between lines, sb across
 * the edge (both in pixels). wd in {4, 6, 8, 16}. loopfilter.rs:396-721. */
static void filter4lines(const Px *px, uint8_t *dst, int E, int I, int H, ptrdiff_t sa,
                         ptrdiff_t sb, int wd)
{
    const int F = 1 << px->bdm8;
    E <<= px->bdm8;
    I <<= px->bdm8;
    H <<= px->bdm8;
    const int dlo = -128 * (1 << px->bdm8), dhi = 128 * (1 << px->bdm8) - 1;
    const int fmax = (128 << px->bdm8) - 1;

    for (int i = 0; i < 4; i++) {
        const ptrdiff_t o = i * sa;
#define P(k) rd(px, dst, o - (k + 1) * sb)
#define Q(k) rd(px, dst, o + (k) * sb)
#define SP(k, v) wr(px, dst, o - (k + 1) * sb, v)
#define SQ(k, v) wr(px, dst, o + (k) * sb, v)
        const int p1 = P(1), p0 = P(0), q0 = Q(0), q1 = Q(1);
        int p2 = 0, p3 = 0, q2 = 0, q3 = 0, p4 = 0, p5 = 0, p6 = 0, q4 = 0, q5 = 0, q6 = 0;
        int fm = abs(p1 - p0) <= I && abs(q1 - q0) <= I &&
                 abs(p0 - q0) * 2 + (abs(p1 - q1) >> 1) <= E;
        if (wd > 4) {
            p2 = P(2); q2 = Q(2);
            fm &= abs(p2 - p1) <= I && abs(q2 - q1) <= I;
            if (wd > 6) {
                p3 = P(3); q3 = Q(3);
                fm &= abs(p3 - p2) <= I && abs(q3 - q2) <= I;
            }
        }
        if (!fm) continue;

        int flat8out = 0, flat8in = 0;
        if (wd >= 16) {
            p6 = P(6); p5 = P(5); p4 = P(4);
            q4 = Q(4); q5 = Q(5); q6 = Q(6);
            flat8out = abs(p6 - p0) <= F && abs(p5 - p0) <= F && abs(p4 - p0) <= F &&
                       abs(q4 - q0) <= F && abs(q5 - q0) <= F && abs(q6 - q0) <= F;
        }
        if (wd >= 6)
            flat8in = abs(p2 - p0) <= F && abs(p1 - p0) <= F &&
                      abs(q1 - q0) <= F && abs(q2 - q0) <= F;
        if (wd >= 8)
            flat8in &= abs(p3 - p0) <= F && abs(q3 - q0) <= F;

        if (wd >= 16 && flat8out && flat8in) {
            SP(5, (p6 * 7 + p5 * 2 + p4 * 2 + p3 + p2 + p1 + p0 + q0 + 8) >> 4);
            SP(4, (p6 * 5 + p5 * 2 + p4 * 2 + p3 * 2 + p2 + p1 + p0 + q0 + q1 + 8) >> 4);
            SP(3, (p6 * 4 + p5 + p4 * 2 + p3 * 2 + p2 * 2 + p1 + p0 + q0 + q1 + q2 + 8) >> 4);
            SP(2, (p6 * 3 + p5 + p4 + p3 * 2 + p2 * 2 + p1 * 2 + p0 + q0 + q1 + q2 + q3 + 8) >> 4);
            SP(1, (p6 * 2 + p5 + p4 + p3 + p2 * 2 + p1 * 2 + p0 * 2 + q0 + q1 + q2 + q3 + q4 + 8) >> 4);
            SP(0, (p6 + p5 + p4 + p3 + p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1 + q2 + q3 + q4 + q5 + 8) >> 4);
            SQ(0, (p5 + p4 + p3 + p2 + p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2 + q3 + q4 + q5 + q6 + 8) >> 4);
            SQ(1, (p4 + p3 + p2 + p1 + p0 + q0 * 2 + q1 * 2 + q2 * 2 + q3 + q4 + q5 + q6 * 2 + 8) >> 4);
            SQ(2, (p3 + p2 + p1 + p0 + q0 + q1 * 2 + q2 * 2 + q3 * 2 + q4 + q5 + q6 * 3 + 8) >> 4);
            SQ(3, (p2 + p1 + p0 + q0 + q1 + q2 * 2 + q3 * 2 + q4 * 2 + q5 + q6 * 4 + 8) >> 4);
            SQ(4, (p1 + p0 + q0 + q1 + q2 + q3 * 2 + q4 * 2 + q5 * 2 + q6 * 5 + 8) >> 4);
            SQ(5, (p0 + q0 + q1 + q2 + q3 + q4 * 2 + q5 * 2 + q6 * 7 + 8) >> 4);
        } else if (wd >= 8 && flat8in) {
            SP(2, (p3 * 3 + p2 * 2 + p1 + p0 + q0 + 4) >> 3);
            SP(1, (p3 * 2 + p2 + p1 * 2 + p0 + q0 + q1 + 4) >> 3);
            SP(0, (p3 + p2 + p1 + p0 * 2 + q0 + q1 + q2 + 4) >> 3);
            SQ(0, (p2 + p1 + p0 + q0 * 2 + q1 + q2 + q3 + 4) >> 3);
            SQ(1, (p1 + p0 + q0 + q1 * 2 + q2 + q3 * 2 + 4) >> 3);
            SQ(2, (p0 + q0 + q1 + q2 * 2 + q3 * 3 + 4) >> 3);
        } else if (wd == 6 && flat8in) {
            SP(1, (p2 * 3 + p1 * 2 + p0 * 2 + q0 + 4) >> 3);
            SP(0, (p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1 + 4) >> 3);
            SQ(0, (p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2 + 4) >> 3);
            SQ(1, (p0 + q0 * 2 + q1 * 2 + q2 * 3 + 4) >> 3);
        } else {
            const int hev = abs(p1 - p0) > H || abs(q1 - q0) > H;
            int f, f1, f2;
            if (hev) {
                f = iclip(p1 - q1, dlo, dhi);
                f = iclip(3 * (q0 - p0) + f, dlo, dhi);
                f1 = imin(f + 4, fmax) >> 3;
                f2 = imin(f + 3, fmax) >> 3;
                SP(0, iclip(p0 + f2, 0, px->bdmax));
                SQ(0, iclip(q0 - f1, 0, px->bdmax));
            } else {
                f = iclip(3 * (q0 - p0), dlo, dhi);
                f1 = imin(f + 4, fmax) >> 3;
                f2 = imin(f + 3, fmax) >> 3;
                SP(0, iclip(p0 + f2, 0, px->bdmax));
                SQ(0, iclip(q0 - f1, 0, px->bdmax));
                f = (f1 + 1) >> 1;
                SP(1, iclip(p1 + f, 0, px->bdmax));
                SQ(1, iclip(q1 - f, 0, px->bdmax));
            }
        }
#undef P
#undef Q
#undef SP
#undef SQ
    }
}

/* loop_filter_sb[plane class][dir] (loopfilter.rs:745-985).
 * cls 0 luma, 1 chroma; dir 0 = column edges (filtering along rows, "h"), 1 = row edges.
 * `lvl` points at the level slot to use; level entries are 4 bytes. */
void oracle_lf_sb(int cls, int dir, void *dst_, ptrdiff_t stride, const uint32_t *vmask,
                  const uint8_t *lvl, ptrdiff_t b4_stride, const uint8_t *lut_e,
                  const uint8_t *lut_i, int wh, int bdmax)
{
    (void)wh;
    Px px = { bdmax > 255, bdmax, 0 };
    px.bdm8 = bdmax == 255 ? 0 : bdmax == 1023 ? 2 : 4;
    const int pxb = px.hbd ? 2 : 1;
    const ptrdiff_t ps = stride / pxb;
    uint8_t *dst = dst_;
    const unsigned vm = cls == 0 ? (vmask[0] | vmask[1] | vmask[2]) : (vmask[0] | vmask[1]);
    /* step to the next 4-px unit along the edge run, and to the neighbour for the fallback */
    const ptrdiff_t unit_px = dir == 0 ? 4 * ps : 4;
    const ptrdiff_t unit_lv = dir == 0 ? b4_stride * 4 : 4;
    const ptrdiff_t prev_lv = dir == 0 ? -4 : -b4_stride * 4;
    for (unsigned bit = 1, k = 0; vm & ~(bit - 1); bit <<= 1, k++) {
        if (!(vm & bit)) continue;
        const uint8_t *l = lvl + k * unit_lv;
        int L = l[0] ? l[0] : l[prev_lv];
        if (!L) continue;
        const int H = L >> 4, E = lut_e[L], I = lut_i[L];
        int wd;
        if (cls == 0) {
            const int idx = (vmask[2] & bit) ? 2 : !!(vmask[1] & bit);
            wd = 4 << idx;
        } else {
            wd = 4 + 2 * !!(vmask[1] & bit);
        }
        uint8_t *d = dst + (ptrdiff_t)k * unit_px * pxb;
        if (dir == 0) filter4lines(&px, d, E, I, H, ps, 1, wd);
        else filter4lines(&px, d, E, I, H, 1, ps, wd);
    }
}

/* Av1Filter (src/lf_mask.rs:40-51): only the deblock part is read here. */
typedef struct {
    uint16_t filter_y[2][32][3][2];
    uint16_t filter_uv[2][32][2][2];
    int8_t cdef_idx[4];
    uint16_t noskip_mask[16][2];
} OAv1Filter;

/* Whole-frame deblocking in the reference's sbrow order.
 * planes/strides: picture (bytes). level: [u8;4] per 4x4 unit, b4_stride units per row.
 * masks: Av1Filter per 128x128 ([sb128h][sb128w]). sb128: superblock size flag (affects only
 * the traversal order). filter_uv: frame_hdr.loopfilter.level_u || level_v. */
void oracle_deblock_frame(void *const planes[3], const ptrdiff_t strides[3], int w, int h,
                          int layout, int bpc, const uint8_t *level, ptrdiff_t b4_stride,
                          const void *masks_, int sb128w, int sb128, const uint8_t *lut_e,
                          const uint8_t *lut_i, int filter_y, int filter_uv)
{
    const OAv1Filter *masks = masks_;
    const int bdmax = (1 << bpc) - 1, pxb = bpc > 8 ? 2 : 1;
    const int w4 = (w + 3) >> 2, h4 = (h + 3) >> 2;
    const int is_sb64 = !sb128;
    const int sbsz = 32 >> is_sb64;
    const int sbh = (h4 + sbsz - 1) / sbsz;
    const int ss_ver = layout == 1, ss_hor = layout == 1 || layout == 2;
    const int has_uv = layout != 0 && filter_uv;
    /* deblocking is skipped as a whole when both luma levels are 0 (recon.rs:4047-4060) */
    if (!filter_y) return;

    for (int sby = 0; sby < sbh; sby++) {
        const int starty4 = (sby & is_sb64) << 4;
        const int endy4 = starty4 + imin(h4 - sby * sbsz, sbsz);
        const int uv_endy4 = (endy4 + ss_ver) >> ss_ver;
        const OAv1Filter *lflvl = masks + (sby >> is_sb64) * sb128w;
        const int row0 = sby * sbsz * 4; /* first luma pixel row of this sbrow */

        {
            /* ---- luma column edges (filter_plane_cols_y) ---- */
            for (int X = 0; X < sb128w; X++) {
                const int wx = imin(32, w4 - X * 32);
                const uint8_t *lv = level + ((ptrdiff_t)sby * sbsz * b4_stride + X * 32) * 4;
                uint8_t *p = (uint8_t *)planes[0] + (ptrdiff_t)row0 * strides[0] + (ptrdiff_t)X * 128 * pxb;
                for (int x = 0; x < wx; x++) {
                    if (X == 0 && x == 0) continue;
                    uint32_t hm[4];
                    const uint16_t (*m)[2] = lflvl[X].filter_y[0][x];
                    if (!starty4) {
                        for (int k = 0; k < 3; k++) {
                            hm[k] = m[k][0];
                            if (endy4 > 16) hm[k] |= (uint32_t)m[k][1] << 16;
                        }
                    } else {
                        for (int k = 0; k < 3; k++) hm[k] = m[k][1];
                    }
                    hm[3] = 0;
                    oracle_lf_sb(0, 0, p + x * 4 * pxb, strides[0], hm, lv + x * 4 + 0, b4_stride,
                                 lut_e, lut_i, endy4 - starty4, bdmax);
                }
            }
        }
        if (has_uv) {
            const int cw_sb = 32 >> ss_hor;
            const int crow0 = (sby * sbsz >> ss_ver) * 4;
            for (int X = 0; X < sb128w; X++) {
                const int wx = (imin(32, w4 - X * 32) + ss_hor) >> ss_hor;
                const uint8_t *lv = level + ((ptrdiff_t)(sby * sbsz >> ss_ver) * b4_stride + X * cw_sb) * 4;
                for (int x = 0; x < wx; x++) {
                    if (X == 0 && x == 0) continue;
                    uint32_t hm[3];
                    const uint16_t (*m)[2] = lflvl[X].filter_uv[0][x];
                    const int sty = starty4 >> ss_ver;
                    if (!sty) {
                        for (int k = 0; k < 2; k++) {
                            hm[k] = m[k][0];
                            if (uv_endy4 > (16 >> ss_ver)) hm[k] |= (uint32_t)m[k][1] << (16 >> ss_ver);
                        }
                    } else {
                        for (int k = 0; k < 2; k++) hm[k] = m[k][1];
                    }
                    hm[2] = 0;
                    for (int pl = 1; pl <= 2; pl++) {
                        uint8_t *p = (uint8_t *)planes[pl] + (ptrdiff_t)crow0 * strides[pl] +
                                     ((ptrdiff_t)X * cw_sb * 4 + x * 4) * pxb;
                        oracle_lf_sb(1, 0, p, strides[pl], hm, lv + x * 4 + 1 + pl, b4_stride,
                                     lut_e, lut_i, uv_endy4 - sty, bdmax);
                    }
                }
            }
        }
        {
            /* ---- luma row edges (filter_plane_rows_y) ---- */
            for (int X = 0; X < sb128w; X++) {
                for (int y = starty4; y < endy4; y++) {
                    if (sby == 0 && y == 0) continue;
                    const int ry = sby * sbsz + (y - starty4);  /* absolute 4x4 row */
                    const uint16_t (*m)[2] = lflvl[X].filter_y[1][y];
                    uint32_t vm[4] = { m[0][0] | ((uint32_t)m[0][1] << 16),
                                       m[1][0] | ((uint32_t)m[1][1] << 16),
                                       m[2][0] | ((uint32_t)m[2][1] << 16), 0 };
                    uint8_t *p = (uint8_t *)planes[0] + (ptrdiff_t)ry * 4 * strides[0] + (ptrdiff_t)X * 128 * pxb;
                    const uint8_t *lv = level + ((ptrdiff_t)ry * b4_stride + X * 32) * 4;
                    oracle_lf_sb(0, 1, p, strides[0], vm, lv + 1, b4_stride, lut_e, lut_i,
                                 imin(32, w4 - X * 32), bdmax);
                }
            }
        }
        if (has_uv) {
            const int cw_sb = 32 >> ss_hor;
            const int sty = starty4 >> ss_ver;
            for (int X = 0; X < sb128w; X++) {
                for (int y = sty; y < uv_endy4; y++) {
                    if (sby == 0 && y == 0) continue;
                    const int ry = (sby * sbsz >> ss_ver) + (y - sty);
                    const uint16_t (*m)[2] = lflvl[X].filter_uv[1][y];
                    uint32_t vm[3] = { m[0][0] | ((uint32_t)m[0][1] << (16 >> ss_hor)),
                                       m[1][0] | ((uint32_t)m[1][1] << (16 >> ss_hor)), 0 };
                    const uint8_t *lv = level + ((ptrdiff_t)ry * b4_stride + X * cw_sb) * 4;
                    for (int pl = 1; pl <= 2; pl++) {
                        uint8_t *p = (uint8_t *)planes[pl] + (ptrdiff_t)ry * 4 * strides[pl] +
                                     (ptrdiff_t)X * cw_sb * 4 * pxb;
                        oracle_lf_sb(1, 1, p, strides[pl], vm, lv + 1 + pl, b4_stride, lut_e,
                                     lut_i, (imin(32, w4 - X * 32) + ss_hor) >> ss_hor, bdmax);
                    }
                }
            }
        }
    }
}

/* rav1d_calc_eih (src/lf_mask.rs:608-626; C src/lf_mask.c:408-425) */
void oracle_calc_eih(uint8_t *lut_e, uint8_t *lut_i, int sharp)
{
    for (int level = 0; level < 64; level++) {
        int limit = level;
        if (sharp > 0) {
            limit >>= (sharp + 3) >> 2;
            limit = imin(limit, 9 - sharp);
        }
        limit = imax(limit, 1);
        lut_i[level] = (uint8_t)limit;
        lut_e[level] = (uint8_t)(2 * (level + 2) + limit);
    }
}
