/*
 * oracle.h — CPU restatement of rav1d's DSP hot path. TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker for the HIP path in rav1d_amd/. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * library (rav1d_amd/librav1d_amd.so) never links or calls it.
 *
 * Each function restates the scalar reference implementation (the Rust `*_rust`/`*_c`
 * fallbacks in FreezyLemon/rav1d, identical to the same-commit dav1d C templates) and
 * cites the reference file:line it follows.
 *
 * Parity pinning status: see DESIGN.md §Oracle. The reference's C build needs the
 * meson-generated config.h, so per the project rules it is unbuildable here; the
 * restatement is pinned by the reference's own fixtures only where the repo's
 * front-end can replay them (not yet) — until then it is "parity unpinned".
 *
 * Conventions (as the reference): pixels are uint8_t (bpc 8) or uint16_t (bpc 10/12),
 * strides are in BYTES (BD::pxstride, include/common/bitdepth.rs:113-125), coefficients
 * are int16_t (bpc 8) or int32_t (bpc 10/12) (bitdepth.rs:272-401).
 */
#ifndef MI_ORACLE_H
#define MI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- itx (src/itx.rs, src/itx_1d.rs; C twin src/itx_tmpl.c, src/itx_1d.c) ---- */
/* One table entry: itxfm_add[tx][txtp](dst, stride, coeff, eob, bitdepth_max).  */
void oracle_itxfm_add(int tx, int txtp, void *dst, ptrdiff_t stride, void *coeff,
                      int eob, int bitdepth_max);
/* Frame-batched form used by the parity tests: blocks as in include/mi_av1dsp.h. */
void oracle_itx_frame(void *const planes[3], const ptrdiff_t strides[3],
                      const void *blocks, int n_blocks, void *coef_arena,
                      int bitdepth_max);
/* 1-D transforms exposed for the numeric sanity tests (kind: 0 dct,1 adst,2 flipadst,3 identity,4 wht) */
void oracle_itx_1d(int kind, int n, int32_t *c, ptrdiff_t stride, int min, int max);

/* ---- mc (src/mc.rs; C twin src/mc_tmpl.c), pixels u8/u16 by bpc, strides in bytes ---- */
/* filter2d: levels.rs Filter2d (0..8 8-tap combos, 9 bilinear); mx/my in 1/16 pel */
void oracle_mc_put(int filter2d, void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                   int w, int h, int mx, int my, int bpc);
void oracle_mc_prep(int filter2d, int16_t *tmp, const void *src, ptrdiff_t src_stride,
                    int w, int h, int mx, int my, int bpc);
void oracle_mc_scaled(int filter2d, int prep, void *dst, ptrdiff_t dst_stride, int16_t *tmp,
                      const void *src, ptrdiff_t src_stride, int w, int h, int mx, int my,
                      int dx, int dy, int bpc);
void oracle_mc_avg(void *dst, ptrdiff_t ds, const int16_t *t1, const int16_t *t2, int w, int h, int bpc);
void oracle_mc_w_avg(void *dst, ptrdiff_t ds, const int16_t *t1, const int16_t *t2, int w, int h,
                     int weight, int bpc);
void oracle_mc_mask(void *dst, ptrdiff_t ds, const int16_t *t1, const int16_t *t2, int w, int h,
                    const uint8_t *mask, int bpc);
void oracle_mc_w_mask(void *dst, ptrdiff_t ds, const int16_t *t1, const int16_t *t2, int w, int h,
                      uint8_t *mask, int sign, int ss_hor, int ss_ver, int bpc);
void oracle_mc_blend(void *dst, ptrdiff_t ds, const void *tmp, int w, int h, const uint8_t *mask, int bpc);
void oracle_mc_blend_v(void *dst, ptrdiff_t ds, const void *tmp, int w, int h, int bpc);
void oracle_mc_blend_h(void *dst, ptrdiff_t ds, const void *tmp, int w, int h, int bpc);
void oracle_mc_warp8x8(int prep, void *dst, ptrdiff_t ds, int16_t *tmp, ptrdiff_t tmp_stride,
                       const void *src, ptrdiff_t ss, const int16_t abcd[4], int mx, int my, int bpc);
void oracle_mc_emu_edge(int bw, int bh, int iw, int ih, int x, int y, void *dst, ptrdiff_t ds,
                        const void *ref, ptrdiff_t rs, int bpc);
void oracle_mc_resize(void *dst, ptrdiff_t ds, const void *src, ptrdiff_t ss, int dst_w, int h,
                      int src_w, int dx, int mx0, int bpc);
/* Frame driver: recon mc() + compound dispatch (recon_tmpl.c:962-1011, 1836-1921) over
 * MiMcBlock records; refs[r*3+p] plane pointers, ref_strides[r*2+{0,1}], ref_wh[r*2+{0,1}]. */
void oracle_mc_frame(void *const cur[3], const ptrdiff_t cur_stride[2], int layout, int bpc,
                     void *const *const refs, const ptrdiff_t *ref_strides, const int *ref_wh,
                     const void *blocks, int n, uint8_t *masks, int16_t *tmp_arena);
void oracle_mc_scaled_frame(void *const cur[3], const ptrdiff_t cur_stride[2], int layout, int bpc, int cur_w,
                            int cur_h, void *const *const refs, const ptrdiff_t *ref_strides, const int *ref_wh,
                            const void *blocks, int n, int16_t *tmp_arena);
void oracle_mc_warp_frame(void *const cur[3], const ptrdiff_t cur_stride[2], int layout, int bpc,
                          void *const *const refs, const ptrdiff_t *ref_strides, const int *ref_wh,
                          const void *blocks, int n, int16_t *tmp_arena);
void oracle_mc_combine_frame(void *const cur[3], const ptrdiff_t cur_stride[2], int layout, int bpc,
                             const void *units, int n, const int16_t *tmp_arena, uint8_t *masks);
void oracle_superres_frame(void *const src[3], const ptrdiff_t src_stride[2], void *const dst[3],
                           const ptrdiff_t dst_stride[2], int layout, int bpc, int src_w, int dst_w, int h);

/* ---- frame driver (decode.c) ---- */
/* refs: 7 x 3 plane pointers (LAST .. ALTREF), ref_strides 7 x 2, ref_wh 7 x 2 (luma w, h) */
struct MiDecFrame;
void oracle_decode_frame_refs(const struct MiDecFrame *f, void *const pic[3], void *const scratch1[3],
                              void *const scratch2[3], const ptrdiff_t strides[3], void *const *refs,
                              const ptrdiff_t *ref_strides, const int *ref_wh, void **out);

/* ---- ipred (src/ipred.rs; C twin src/ipred_tmpl.c) ---- */
/* mode = intra_pred[] slot: 0 DC,1 V,2 H,3 LEFT_DC,4 TOP_DC,5 DC_128,6 Z1,7 Z2,8 Z3,9 SMOOTH,
 * 10 SMOOTH_V,11 SMOOTH_H,12 PAETH,13 FILTER; `angle` carries is_sm (bit 9) and the edge-filter
 * enable (bit 10) for Z1-Z3, the filter index for FILTER. */
void oracle_intra_pred(int mode, void *dst, ptrdiff_t stride, const void *topleft, int w, int h,
                       int angle, int max_w, int max_h, int bpc);
void oracle_cfl_ac(int16_t *ac, const void *ypx, ptrdiff_t stride, int w_pad, int h_pad, int cw, int ch,
                   int ss_hor, int ss_ver, int bpc);
void oracle_cfl_pred(int mode, void *dst, ptrdiff_t stride, const void *topleft, int w, int h,
                     const int16_t *ac, int alpha, int bpc);
void oracle_pal_pred(void *dst, ptrdiff_t stride, const void *pal, const uint8_t *idx, int w, int h, int bpc);
int oracle_prepare_intra_edges(int x, int have_left, int y, int have_top, int tile_w, int tile_h,
                               int top_has_right, int left_has_bottom, const void *pic, ptrdiff_t stride,
                               int mode, int *angle, int w, int h, int filter_edge, void *topleft, int bpc);
void oracle_intra_blocks(void *const planes[3], const ptrdiff_t strides[2], int bpc, const void *blocks, int n,
                         const int16_t *ac, const uint8_t *idx, const void *pal);
void oracle_intra_recon(void *const planes[3], const ptrdiff_t strides[2], int bpc, const void *blocks,
                        const void *tx_blocks, int n, const int16_t *ac, const uint8_t *idx, const void *pal,
                        void *coef);

/* lr.c: per-call loop restoration (one unit, in place) */
void oracle_lr_wiener(void *p, ptrdiff_t stride, const void *left_px, const void *lpf, int w, int h,
                      const int16_t filter[2][8], int edges, int bdmax);
void oracle_lr_sgr(int kind, void *p, ptrdiff_t stride, const void *left_px, const void *lpf, int w, int h,
                   unsigned s0, unsigned s1, int w0, int w1, int edges, int bdmax);

/* filmgrain.c: per-call table entries */
void oracle_fg_generate_grain_y(int16_t *buf, const void *data, int bdmax);
void oracle_fg_generate_scaling(int bitdepth, const uint8_t (*points)[2], int num, uint8_t *scaling);
void oracle_fg_generate_grain_uv(int16_t *buf, const int16_t *buf_y, const void *data, int uv,
                                 int subx, int suby, int bdmax);
void oracle_fg_32x32xn(int pl, int layout, void *dst_row, const void *src_row, ptrdiff_t stride, const void *data,
                       int pw, const uint8_t *scaling, const int16_t *lut, int bh, int row_num,
                       const void *luma_row, ptrdiff_t luma_stride, int is_id, int bdmax);

#ifdef __cplusplus
}
#endif
#endif
