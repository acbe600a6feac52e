/*
 * mi_dsp_table.h — the slot-exact drop-in surface: one function per Rav1dDSPContext table slot,
 * with the slot's own signature (void return, trailing bitdepth_max where the reference has one),
 * and mi_fill_dsp_tables() filling a struct laid out exactly like the reference's
 * Rav1dDSPContext (src/internal.rs:111-121; C src/internal.h:61-69), as the reference's
 * *_dsp_init functions do (src/decode.rs:4739-4774; itx.rs:1063-1110, mc.rs:2495-2568, ...).
 *
 * A rav1d host drops these in by filling `c.dsp[bpc]` with mi_fill_dsp_tables instead of the
 * rav1d_*_dsp_init calls. Every slot is a synchronous single-call device
 * launch (librav1d_amd.so's mi_dsp_* entries): it accepts host or device pointers and any
 * stride sign. Slots are parity/fallback entries, not the performance path (that is the
 * batched per-frame API of mi_av1dsp.h).
 *
 * Slots whose reference signature has no bitdepth_max (cfl_ac, pal_pred, blend, blend_v,
 * blend_h, emu_edge) come in _8bpc / _16bpc variants; mi_fill_dsp_tables picks by bpc.
 */
#ifndef MI_DSP_TABLE_H
#define MI_DSP_TABLE_H

#include <stddef.h>
#include <stdint.h>

#include "mi_av1dsp.h"

#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* slot signatures (the src/<table>.rs fn types; pixels are void: u8 at 8 bpc, u16 above) */
typedef void (*mi_itxfm_fn)(void *dst, ptrdiff_t stride, void *coeff, int eob, int bitdepth_max);   /* itx.rs:190 */
typedef void (*mi_angular_ipred_fn)(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, int angle,
                                    int max_width, int max_height, int bitdepth_max);               /* ipred.rs:48 */
typedef void (*mi_cfl_ac_fn)(int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad, int cw,
                             int ch);                                                                  /* ipred.rs:82 */
typedef void (*mi_cfl_pred_fn)(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, const int16_t *ac,
                               int alpha, int bitdepth_max);                                         /* ipred.rs:108 */
typedef void (*mi_pal_pred_fn)(void *dst, ptrdiff_t stride, const void *pal, const uint8_t *idx, int w,
                               int h);                                                                /* ipred.rs:138 */
typedef void (*mi_mc_fn)(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int w, int h,
                         int mx, int my, int bitdepth_max);                                           /* mc.rs:1174 */
typedef void (*mi_mc_scaled_fn)(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int w,
                                int h, int mx, int my, int dx, int dy, int bitdepth_max);            /* mc.rs:1186 */
typedef void (*mi_mct_fn)(int16_t *tmp, const void *src, ptrdiff_t src_stride, int w, int h, int mx, int my,
                          int bitdepth_max);                                                          /* mc.rs:1211 */
typedef void (*mi_mct_scaled_fn)(int16_t *tmp, const void *src, ptrdiff_t src_stride, int w, int h, int mx, int my,
                                 int dx, int dy, int bitdepth_max);                                  /* mc.rs:1222 */
typedef void (*mi_avg_fn)(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                          int bitdepth_max);                                                          /* mc.rs:1246 */
typedef void (*mi_w_avg_fn)(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w,
                            int h, int weight, int bitdepth_max);                                    /* mc.rs:1256 */
typedef void (*mi_mask_fn)(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                           const uint8_t *mask, int bitdepth_max);                                    /* mc.rs:1267 */
typedef void (*mi_w_mask_fn)(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w,
                             int h, uint8_t *mask, int sign, int bitdepth_max);                       /* mc.rs:1278 */
typedef void (*mi_blend_fn)(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h,
                            const uint8_t *mask);                                                     /* mc.rs:1290 */
typedef void (*mi_blend_dir_fn)(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h);     /* mc.rs:1293 */
typedef void (*mi_warp8x8_fn)(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                              const int16_t *abcd, int mx, int my, int bitdepth_max);                 /* mc.rs:1200 */
typedef void (*mi_warp8x8t_fn)(int16_t *tmp, ptrdiff_t tmp_stride, const void *src, ptrdiff_t src_stride,
                               const int16_t *abcd, int mx, int my, int bitdepth_max);                /* mc.rs:1235 */
typedef void (*mi_emu_edge_fn)(intptr_t bw, intptr_t bh, intptr_t iw, intptr_t ih, intptr_t x, intptr_t y,
                               void *dst, ptrdiff_t dst_stride, const void *ref, ptrdiff_t ref_stride);   /* mc.rs:1296 */
typedef void (*mi_resize_fn)(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int dst_w,
                             int h, int src_w, int dx, int mx0, int bitdepth_max);                   /* mc.rs:1309 */
typedef void (*mi_loopfilter_sb_fn)(void *dst, ptrdiff_t stride, const uint32_t *mask, const uint8_t (*lvl)[4],
                                    ptrdiff_t lvl_stride, const void *lut, int w, int bitdepth_max);  /* loopfilter.rs:20 */
typedef void (*mi_cdef_fn)(void *dst, ptrdiff_t stride, const void *left, const void *top, const void *bottom,
                           int pri_strength, int sec_strength, int dir, int damping, unsigned edges,
                           int bitdepth_max);                                                         /* cdef.rs:35 */
typedef int (*mi_cdef_dir_fn)(const void *dst, ptrdiff_t stride, unsigned *var, int bitdepth_max);   /* cdef.rs:49 */
typedef void (*mi_lr_fn)(void *dst, ptrdiff_t stride, const void *left, const void *lpf, int w, int h,
                         const void *params, unsigned edges, int bitdepth_max);                       /* looprestoration.rs:91 */
typedef void (*mi_generate_grain_y_fn)(void *buf, const MiFilmGrainData *data, int bitdepth_max);   /* filmgrain.rs:41 */
typedef void (*mi_generate_grain_uv_fn)(void *buf, const void *buf_y, const MiFilmGrainData *data, intptr_t uv,
                                        int bitdepth_max);                                            /* filmgrain.rs:61 */
typedef void (*mi_fgy_32x32xn_fn)(void *dst_row, const void *src_row, ptrdiff_t stride, const MiFilmGrainData *data,
                                  size_t pw, const uint8_t *scaling, const void *grain_lut, int bh, int row_num,
                                  int bitdepth_max);                                                  /* filmgrain.rs:87 */
typedef void (*mi_fguv_32x32xn_fn)(void *dst_row, const void *src_row, ptrdiff_t stride,
                                   const MiFilmGrainData *data, size_t pw, const uint8_t *scaling,
                                   const void *grain_lut, int bh, int row_num, const void *luma_row,
                                   ptrdiff_t luma_stride, int uv_pl, int is_id, int bitdepth_max);   /* filmgrain.rs:128 */

/* Rav1dDSPContext, field for field (src/internal.rs:111-121 and the sub-tables:
 * filmgrain.rs:194-199, ipred.rs:164-169, mc.rs:1322-1338, itx.rs:194-196,
 * loopfilter.rs:32-34, cdef.rs:53-56, looprestoration.rs:104-107). enum_map slots are
 * [I420, I422, I444]; w_mask is [444, 422, 420] (mc.rs:2546-2548). */
typedef struct MiDSPContext {
    struct {
        mi_generate_grain_y_fn generate_grain_y;
        mi_generate_grain_uv_fn generate_grain_uv[3];
        mi_fgy_32x32xn_fn fgy_32x32xn;
        mi_fguv_32x32xn_fn fguv_32x32xn[3];
    } fg;
    struct {
        mi_angular_ipred_fn intra_pred[14];
        mi_cfl_ac_fn cfl_ac[3];
        mi_cfl_pred_fn cfl_pred[6];
        mi_pal_pred_fn pal_pred;
    } ipred;
    struct {
        mi_mc_fn mc[10];
        mi_mc_scaled_fn mc_scaled[10];
        mi_mct_fn mct[10];
        mi_mct_scaled_fn mct_scaled[10];
        mi_avg_fn avg;
        mi_w_avg_fn w_avg;
        mi_mask_fn mask;
        mi_w_mask_fn w_mask[3];
        mi_blend_fn blend;
        mi_blend_dir_fn blend_v;
        mi_blend_dir_fn blend_h;
        mi_warp8x8_fn warp8x8;
        mi_warp8x8t_fn warp8x8t;
        mi_emu_edge_fn emu_edge;
        mi_resize_fn resize;
    } mc;
    struct {
        mi_itxfm_fn itxfm_add[MI_N_RECT_TX_SIZES][17];   /* NULL where the reference has None */
    } itx;
    struct {
        mi_loopfilter_sb_fn loop_filter_sb[2][2];
    } lf;
    struct {
        mi_cdef_dir_fn dir;
        mi_cdef_fn fb[3];
    } cdef;
    struct {
        mi_lr_fn wiener[2];
        mi_lr_fn sgr[3];
    } lr;
    bool initialized;
} MiDSPContext;

/* Fill a Rav1dDSPContext-layout struct for bpc 8, 10 or 12 (10 and 12 share the 16 bpc slots,
 * as the reference's BitDepth16): 0, or -EINVAL. Sets `initialized`. */
int mi_fill_dsp_tables(void *dsp_ctx, int bpc);

/* sizeof(MiDSPContext): 421 function pointers + the bool, as the reference's struct. */
size_t mi_dsp_context_size(void);

/* ---- the slot functions (names follow the reference's asm symbols without the
 * _<bpc>bpc_<isa> suffix, e.g. dav1d_inv_txfm_add_dct_dct_16x16_16bpc_avx2, itx.rs:199-222) ---- */

/* itxfm_add[tx][txtp] = mi_inv_txfm_add_<name>: X(tx, txtp, name) for the 156 slots the
 * reference fills (itx.rs:1072-1110; name = <row fn>_<column fn>_<w>x<h>, itx.rs:960-1060) */
#define MI_ITX_SLOTS(X) \
    X(0, 0, dct_dct_4x4) \
    X(0, 1, dct_adst_4x4) \
    X(0, 2, adst_dct_4x4) \
    X(0, 3, adst_adst_4x4) \
    X(0, 4, dct_flipadst_4x4) \
    X(0, 5, flipadst_dct_4x4) \
    X(0, 6, flipadst_flipadst_4x4) \
    X(0, 7, flipadst_adst_4x4) \
    X(0, 8, adst_flipadst_4x4) \
    X(0, 9, identity_identity_4x4) \
    X(0, 10, identity_dct_4x4) \
    X(0, 11, dct_identity_4x4) \
    X(0, 12, identity_adst_4x4) \
    X(0, 13, adst_identity_4x4) \
    X(0, 14, identity_flipadst_4x4) \
    X(0, 15, flipadst_identity_4x4) \
    X(0, 16, wht_wht_4x4) \
    X(1, 0, dct_dct_8x8) \
    X(1, 1, dct_adst_8x8) \
    X(1, 2, adst_dct_8x8) \
    X(1, 3, adst_adst_8x8) \
    X(1, 4, dct_flipadst_8x8) \
    X(1, 5, flipadst_dct_8x8) \
    X(1, 6, flipadst_flipadst_8x8) \
    X(1, 7, flipadst_adst_8x8) \
    X(1, 8, adst_flipadst_8x8) \
    X(1, 9, identity_identity_8x8) \
    X(1, 10, identity_dct_8x8) \
    X(1, 11, dct_identity_8x8) \
    X(1, 12, identity_adst_8x8) \
    X(1, 13, adst_identity_8x8) \
    X(1, 14, identity_flipadst_8x8) \
    X(1, 15, flipadst_identity_8x8) \
    X(2, 0, dct_dct_16x16) \
    X(2, 1, dct_adst_16x16) \
    X(2, 2, adst_dct_16x16) \
    X(2, 3, adst_adst_16x16) \
    X(2, 4, dct_flipadst_16x16) \
    X(2, 5, flipadst_dct_16x16) \
    X(2, 6, flipadst_flipadst_16x16) \
    X(2, 7, flipadst_adst_16x16) \
    X(2, 8, adst_flipadst_16x16) \
    X(2, 9, identity_identity_16x16) \
    X(2, 10, identity_dct_16x16) \
    X(2, 11, dct_identity_16x16) \
    X(3, 0, dct_dct_32x32) \
    X(3, 9, identity_identity_32x32) \
    X(4, 0, dct_dct_64x64) \
    X(5, 0, dct_dct_4x8) \
    X(5, 1, dct_adst_4x8) \
    X(5, 2, adst_dct_4x8) \
    X(5, 3, adst_adst_4x8) \
    X(5, 4, dct_flipadst_4x8) \
    X(5, 5, flipadst_dct_4x8) \
    X(5, 6, flipadst_flipadst_4x8) \
    X(5, 7, flipadst_adst_4x8) \
    X(5, 8, adst_flipadst_4x8) \
    X(5, 9, identity_identity_4x8) \
    X(5, 10, identity_dct_4x8) \
    X(5, 11, dct_identity_4x8) \
    X(5, 12, identity_adst_4x8) \
    X(5, 13, adst_identity_4x8) \
    X(5, 14, identity_flipadst_4x8) \
    X(5, 15, flipadst_identity_4x8) \
    X(6, 0, dct_dct_8x4) \
    X(6, 1, dct_adst_8x4) \
    X(6, 2, adst_dct_8x4) \
    X(6, 3, adst_adst_8x4) \
    X(6, 4, dct_flipadst_8x4) \
    X(6, 5, flipadst_dct_8x4) \
    X(6, 6, flipadst_flipadst_8x4) \
    X(6, 7, flipadst_adst_8x4) \
    X(6, 8, adst_flipadst_8x4) \
    X(6, 9, identity_identity_8x4) \
    X(6, 10, identity_dct_8x4) \
    X(6, 11, dct_identity_8x4) \
    X(6, 12, identity_adst_8x4) \
    X(6, 13, adst_identity_8x4) \
    X(6, 14, identity_flipadst_8x4) \
    X(6, 15, flipadst_identity_8x4) \
    X(7, 0, dct_dct_8x16) \
    X(7, 1, dct_adst_8x16) \
    X(7, 2, adst_dct_8x16) \
    X(7, 3, adst_adst_8x16) \
    X(7, 4, dct_flipadst_8x16) \
    X(7, 5, flipadst_dct_8x16) \
    X(7, 6, flipadst_flipadst_8x16) \
    X(7, 7, flipadst_adst_8x16) \
    X(7, 8, adst_flipadst_8x16) \
    X(7, 9, identity_identity_8x16) \
    X(7, 10, identity_dct_8x16) \
    X(7, 11, dct_identity_8x16) \
    X(7, 12, identity_adst_8x16) \
    X(7, 13, adst_identity_8x16) \
    X(7, 14, identity_flipadst_8x16) \
    X(7, 15, flipadst_identity_8x16) \
    X(8, 0, dct_dct_16x8) \
    X(8, 1, dct_adst_16x8) \
    X(8, 2, adst_dct_16x8) \
    X(8, 3, adst_adst_16x8) \
    X(8, 4, dct_flipadst_16x8) \
    X(8, 5, flipadst_dct_16x8) \
    X(8, 6, flipadst_flipadst_16x8) \
    X(8, 7, flipadst_adst_16x8) \
    X(8, 8, adst_flipadst_16x8) \
    X(8, 9, identity_identity_16x8) \
    X(8, 10, identity_dct_16x8) \
    X(8, 11, dct_identity_16x8) \
    X(8, 12, identity_adst_16x8) \
    X(8, 13, adst_identity_16x8) \
    X(8, 14, identity_flipadst_16x8) \
    X(8, 15, flipadst_identity_16x8) \
    X(9, 0, dct_dct_16x32) \
    X(9, 9, identity_identity_16x32) \
    X(10, 0, dct_dct_32x16) \
    X(10, 9, identity_identity_32x16) \
    X(11, 0, dct_dct_32x64) \
    X(12, 0, dct_dct_64x32) \
    X(13, 0, dct_dct_4x16) \
    X(13, 1, dct_adst_4x16) \
    X(13, 2, adst_dct_4x16) \
    X(13, 3, adst_adst_4x16) \
    X(13, 4, dct_flipadst_4x16) \
    X(13, 5, flipadst_dct_4x16) \
    X(13, 6, flipadst_flipadst_4x16) \
    X(13, 7, flipadst_adst_4x16) \
    X(13, 8, adst_flipadst_4x16) \
    X(13, 9, identity_identity_4x16) \
    X(13, 10, identity_dct_4x16) \
    X(13, 11, dct_identity_4x16) \
    X(13, 12, identity_adst_4x16) \
    X(13, 13, adst_identity_4x16) \
    X(13, 14, identity_flipadst_4x16) \
    X(13, 15, flipadst_identity_4x16) \
    X(14, 0, dct_dct_16x4) \
    X(14, 1, dct_adst_16x4) \
    X(14, 2, adst_dct_16x4) \
    X(14, 3, adst_adst_16x4) \
    X(14, 4, dct_flipadst_16x4) \
    X(14, 5, flipadst_dct_16x4) \
    X(14, 6, flipadst_flipadst_16x4) \
    X(14, 7, flipadst_adst_16x4) \
    X(14, 8, adst_flipadst_16x4) \
    X(14, 9, identity_identity_16x4) \
    X(14, 10, identity_dct_16x4) \
    X(14, 11, dct_identity_16x4) \
    X(14, 12, identity_adst_16x4) \
    X(14, 13, adst_identity_16x4) \
    X(14, 14, identity_flipadst_16x4) \
    X(14, 15, flipadst_identity_16x4) \
    X(15, 0, dct_dct_8x32) \
    X(15, 9, identity_identity_8x32) \
    X(16, 0, dct_dct_32x8) \
    X(16, 9, identity_identity_32x8) \
    X(17, 0, dct_dct_16x64) \
    X(18, 0, dct_dct_64x16)

#define MI_DECL_ITX(tx, txtp, name) \
    void mi_inv_txfm_add_##name(void *dst, ptrdiff_t stride, void *coeff, int eob, int bitdepth_max);
MI_ITX_SLOTS(MI_DECL_ITX)
#undef MI_DECL_ITX

/* intra_pred[mode] = mi_ipred_<name> (ipred.rs:2203-2255) */
#define MI_IPRED_SLOTS(X) \
    X(0, dc) X(1, v) X(2, h) X(3, dc_left) X(4, dc_top) X(5, dc_128) X(6, z1) X(7, z2) X(8, z3) \
    X(9, smooth) X(10, smooth_v) X(11, smooth_h) X(12, paeth) X(13, filter)
#define MI_DECL_IPRED(mode, name) \
    void mi_ipred_##name(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, int angle, \
                         int max_width, int max_height, int bitdepth_max);
MI_IPRED_SLOTS(MI_DECL_IPRED)
#undef MI_DECL_IPRED

/* cfl_pred[mode]: DC_PRED 0, LEFT_DC 3, TOP_DC 4, DC_128 5 (ipred.rs:2075-2078) */
void mi_ipred_cfl(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, const int16_t *ac, int alpha,
                  int bitdepth_max);
void mi_ipred_cfl_left(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, const int16_t *ac,
                       int alpha, int bitdepth_max);
void mi_ipred_cfl_top(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, const int16_t *ac,
                      int alpha, int bitdepth_max);
void mi_ipred_cfl_128(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, const int16_t *ac,
                      int alpha, int bitdepth_max);
/* cfl_pred[1] / [2]: the reference's never-called default (wrap_fn_ptr.rs:71-80); aborts */
void mi_ipred_cfl_unimplemented(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, const int16_t *ac,
                                int alpha, int bitdepth_max);
/* cfl_ac[I420, I422, I444] and pal_pred: no bitdepth argument, one variant per pixel size */
#define MI_BPC_SLOTS(X) X(8bpc) X(16bpc)
#define MI_DECL_BPC(bpc) \
    void mi_ipred_cfl_ac_420_##bpc(int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad, int cw, \
                                   int ch); \
    void mi_ipred_cfl_ac_422_##bpc(int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad, int cw, \
                                   int ch); \
    void mi_ipred_cfl_ac_444_##bpc(int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad, int cw, \
                                   int ch); \
    void mi_pal_pred_##bpc(void *dst, ptrdiff_t stride, const void *pal, const uint8_t *idx, int w, int h); \
    void mi_blend_##bpc(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h, const uint8_t *mask); \
    void mi_blend_v_##bpc(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h); \
    void mi_blend_h_##bpc(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h); \
    void mi_emu_edge_##bpc(intptr_t bw, intptr_t bh, intptr_t iw, intptr_t ih, intptr_t x, intptr_t y, void *dst, \
                           ptrdiff_t dst_stride, const void *ref, ptrdiff_t ref_stride);
MI_BPC_SLOTS(MI_DECL_BPC)
#undef MI_DECL_BPC

/* mc[f] / mc_scaled[f] / mct[f] / mct_scaled[f] = mi_{put,prep}_<name>[_scaled], f = Filter2d
 * (levels.rs:172-183; mc.rs:2495-2540) */
#define MI_FILTER2D_SLOTS(X) \
    X(0, 8tap_regular) X(1, 8tap_regular_smooth) X(2, 8tap_regular_sharp) X(3, 8tap_sharp_regular) \
    X(4, 8tap_sharp_smooth) X(5, 8tap_sharp) X(6, 8tap_smooth_regular) X(7, 8tap_smooth) \
    X(8, 8tap_smooth_sharp) X(9, bilin)
#define MI_DECL_MC(f, name) \
    void mi_put_##name(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int w, int h, \
                       int mx, int my, int bitdepth_max); \
    void mi_put_##name##_scaled(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int w, \
                                int h, int mx, int my, int dx, int dy, int bitdepth_max); \
    void mi_prep_##name(int16_t *tmp, const void *src, ptrdiff_t src_stride, int w, int h, int mx, int my, \
                        int bitdepth_max); \
    void mi_prep_##name##_scaled(int16_t *tmp, const void *src, ptrdiff_t src_stride, int w, int h, int mx, \
                                 int my, int dx, int dy, int bitdepth_max);
MI_FILTER2D_SLOTS(MI_DECL_MC)
#undef MI_DECL_MC

void mi_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
            int bitdepth_max);
void mi_w_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h, int weight,
              int bitdepth_max);
void mi_mask(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
             const uint8_t *mask, int bitdepth_max);
void mi_w_mask_444(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                   uint8_t *mask, int sign, int bitdepth_max);
void mi_w_mask_422(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                   uint8_t *mask, int sign, int bitdepth_max);
void mi_w_mask_420(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                   uint8_t *mask, int sign, int bitdepth_max);
void mi_warp_affine_8x8(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                        const int16_t *abcd, int mx, int my, int bitdepth_max);
void mi_warp_affine_8x8t(int16_t *tmp, ptrdiff_t tmp_stride, const void *src, ptrdiff_t src_stride,
                         const int16_t *abcd, int mx, int my, int bitdepth_max);
void mi_resize(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int dst_w, int h, int src_w,
               int dx, int mx0, int bitdepth_max);

/* loop_filter_sb[luma, chroma][column edges, row edges] (loopfilter.rs:745-985) */
void mi_lpf_h_sb_y(void *dst, ptrdiff_t stride, const uint32_t *mask, const uint8_t (*lvl)[4], ptrdiff_t lvl_stride,
                   const void *lut, int w, int bitdepth_max);
void mi_lpf_v_sb_y(void *dst, ptrdiff_t stride, const uint32_t *mask, const uint8_t (*lvl)[4], ptrdiff_t lvl_stride,
                   const void *lut, int w, int bitdepth_max);
void mi_lpf_h_sb_uv(void *dst, ptrdiff_t stride, const uint32_t *mask, const uint8_t (*lvl)[4], ptrdiff_t lvl_stride,
                    const void *lut, int w, int bitdepth_max);
void mi_lpf_v_sb_uv(void *dst, ptrdiff_t stride, const uint32_t *mask, const uint8_t (*lvl)[4], ptrdiff_t lvl_stride,
                    const void *lut, int w, int bitdepth_max);

/* cdef.dir, cdef.fb[8x8, 4x8, 4x4] (cdef.rs:35-56) */
int mi_cdef_dir(const void *dst, ptrdiff_t stride, unsigned *var, int bitdepth_max);
#define MI_DECL_CDEF(wh) \
    void mi_cdef_filter_##wh(void *dst, ptrdiff_t stride, const void *left, const void *top, const void *bottom, \
                             int pri_strength, int sec_strength, int dir, int damping, unsigned edges, \
                             int bitdepth_max);
MI_DECL_CDEF(8x8) MI_DECL_CDEF(4x8) MI_DECL_CDEF(4x4)
#undef MI_DECL_CDEF

/* lr.wiener[7-tap, 5-tap], lr.sgr[5x5, 3x3, mix] (looprestoration.rs:104-107) */
#define MI_DECL_LR(name) \
    void mi_##name(void *dst, ptrdiff_t stride, const void *left, const void *lpf, int w, int h, const void *params, \
                   unsigned edges, int bitdepth_max);
MI_DECL_LR(wiener_filter7) MI_DECL_LR(wiener_filter5) MI_DECL_LR(sgr_filter_5x5) MI_DECL_LR(sgr_filter_3x3)
MI_DECL_LR(sgr_filter_mix)
#undef MI_DECL_LR

/* film grain (filmgrain.rs:194-199) */
void mi_generate_grain_y(void *buf, const MiFilmGrainData *data, int bitdepth_max);
#define MI_DECL_FG(ss) \
    void mi_generate_grain_uv_##ss(void *buf, const void *buf_y, const MiFilmGrainData *data, intptr_t uv, \
                                   int bitdepth_max); \
    void mi_fguv_32x32xn_##ss(void *dst_row, const void *src_row, ptrdiff_t stride, const MiFilmGrainData *data, \
                              size_t pw, const uint8_t *scaling, const void *grain_lut, int bh, int row_num, \
                              const void *luma_row, ptrdiff_t luma_stride, int uv_pl, int is_id, int bitdepth_max);
MI_DECL_FG(420) MI_DECL_FG(422) MI_DECL_FG(444)
#undef MI_DECL_FG
void mi_fgy_32x32xn(void *dst_row, const void *src_row, ptrdiff_t stride, const MiFilmGrainData *data, size_t pw,
                    const uint8_t *scaling, const void *grain_lut, int bh, int row_num, int bitdepth_max);

#ifdef __cplusplus
}
#endif
#endif /* MI_DSP_TABLE_H */
