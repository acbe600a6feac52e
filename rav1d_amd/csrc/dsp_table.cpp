// dsp_table.cpp — the slot-exact drop-in surface (include/mi_dsp_table.h): one void function
// per Rav1dDSPContext slot with the slot's own signature, each a thunk over the per-call
// entries (capi.cpp mi_dsp_*), and mi_fill_dsp_tables filling the reference's table layout as
// its *_dsp_init functions do (src/decode.rs:4739-4774).
//
// The reference's slots return void and leave preconditions to the caller (assert /
// unreachable!); a slot here drops the per-call entry's -errno the same way: invalid arguments
// write nothing.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mi_dsp_table.h"

static_assert(sizeof(MiDSPContext) == 421 * sizeof(void *) + sizeof(void *), "Rav1dDSPContext layout");
static_assert(offsetof(MiDSPContext, ipred) == 8 * sizeof(void *), "fg table: 8 slots");
static_assert(offsetof(MiDSPContext, mc) == 32 * sizeof(void *), "ipred table: 24 slots");
static_assert(offsetof(MiDSPContext, itx) == 85 * sizeof(void *), "mc table: 53 slots");
static_assert(offsetof(MiDSPContext, lf) == 408 * sizeof(void *), "itx table: 19 x 17 slots");

extern "C" {

// ---- itx ----
#define MI_DEF_ITX(tx, txtp, name)                                                                   \
    void mi_inv_txfm_add_##name(void *dst, ptrdiff_t stride, void *coeff, int eob, int bitdepth_max) { \
        (void)mi_dsp_itxfm_add(tx, txtp, dst, stride, coeff, eob, bitdepth_max);                       \
    }
MI_ITX_SLOTS(MI_DEF_ITX)
#undef MI_DEF_ITX

// ---- ipred ----
#define MI_DEF_IPRED(mode, name)                                                                        \
    void mi_ipred_##name(void *dst, ptrdiff_t stride, const void *topleft, int w, int h, int angle,     \
                         int max_width, int max_height, int bitdepth_max) {                             \
        (void)mi_dsp_intra_pred(mode, dst, stride, topleft, w, h, angle, max_width, max_height,         \
                                bitdepth_max);                                                          \
    }
MI_IPRED_SLOTS(MI_DEF_IPRED)
#undef MI_DEF_IPRED

#define MI_DEF_CFL(suffix, mode)                                                                         \
    void mi_ipred_cfl##suffix(void *dst, ptrdiff_t stride, const void *topleft, int w, int h,            \
                              const int16_t *ac, int alpha, int bitdepth_max) {                          \
        (void)mi_dsp_cfl_pred(mode, dst, stride, topleft, w, h, ac, alpha, bitdepth_max);                \
    }
MI_DEF_CFL(, 0)
MI_DEF_CFL(_left, 3)
MI_DEF_CFL(_top, 4)
MI_DEF_CFL(_128, 5)
#undef MI_DEF_CFL
// cfl_pred[1] / [2]: the reference's DefaultValue::DEFAULT (wrap_fn_ptr.rs:71-80), a
// non-null function that must never be reached (unimplemented!())
void mi_ipred_cfl_unimplemented(void *, ptrdiff_t, const void *, int, int, const int16_t *, int, int) {
    fprintf(stderr, "mi_dsp_table: cfl_pred slot without an implementation called\n");
    abort();
}

// Slots without a bitdepth argument: the pixel size is the variant's (16 bpc covers 10 and
// 12 bits, whose pixels these slots handle identically).
static inline int bdmax_of(int bpc16) { return bpc16 ? 4095 : 255; }
#define MI_DEF_BPC(bpc, is16)                                                                              \
    void mi_ipred_cfl_ac_420_##bpc(int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad,      \
                                   int cw, int ch) {                                                      \
        (void)mi_dsp_cfl_ac(1, ac, y, stride, w_pad, h_pad, cw, ch, bdmax_of(is16));                        \
    }                                                                                                     \
    void mi_ipred_cfl_ac_422_##bpc(int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad,      \
                                   int cw, int ch) {                                                      \
        (void)mi_dsp_cfl_ac(2, ac, y, stride, w_pad, h_pad, cw, ch, bdmax_of(is16));                        \
    }                                                                                                     \
    void mi_ipred_cfl_ac_444_##bpc(int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad,      \
                                   int cw, int ch) {                                                      \
        (void)mi_dsp_cfl_ac(3, ac, y, stride, w_pad, h_pad, cw, ch, bdmax_of(is16));                        \
    }                                                                                                     \
    void mi_pal_pred_##bpc(void *dst, ptrdiff_t stride, const void *pal, const uint8_t *idx, int w, int h) { \
        (void)mi_dsp_pal_pred(dst, stride, pal, idx, w, h, bdmax_of(is16));                                \
    }                                                                                                     \
    void mi_blend_##bpc(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h, const uint8_t *mask) { \
        (void)mi_dsp_mc_blend(dst, dst_stride, tmp, w, h, mask, bdmax_of(is16));                           \
    }                                                                                                     \
    void mi_blend_v_##bpc(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h) {                \
        (void)mi_dsp_mc_blend_v(dst, dst_stride, tmp, w, h, bdmax_of(is16));                               \
    }                                                                                                     \
    void mi_blend_h_##bpc(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h) {                \
        (void)mi_dsp_mc_blend_h(dst, dst_stride, tmp, w, h, bdmax_of(is16));                               \
    }                                                                                                     \
    void mi_emu_edge_##bpc(intptr_t bw, intptr_t bh, intptr_t iw, intptr_t ih, intptr_t x, intptr_t y,     \
                           void *dst, ptrdiff_t dst_stride, const void *ref, ptrdiff_t ref_stride) {       \
        (void)mi_dsp_mc_emu_edge((int)bw, (int)bh, (int)iw, (int)ih, (int)x, (int)y, dst, dst_stride, ref,  \
                                 ref_stride, bdmax_of(is16));                                              \
    }
MI_DEF_BPC(8bpc, 0)
MI_DEF_BPC(16bpc, 1)
#undef MI_DEF_BPC

// ---- mc ----
#define MI_DEF_MC(f, name)                                                                               \
    void mi_put_##name(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int w, int h, \
                       int mx, int my, int bitdepth_max) {                                                \
        (void)mi_dsp_mc_put(f, dst, dst_stride, src, src_stride, w, h, mx, my, bitdepth_max);             \
    }                                                                                                    \
    void mi_put_##name##_scaled(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,   \
                                int w, int h, int mx, int my, int dx, int dy, int bitdepth_max) {         \
        (void)mi_dsp_mc_scaled(0, f, dst, dst_stride, src, src_stride, w, h, mx, my, dx, dy, bitdepth_max); \
    }                                                                                                    \
    void mi_prep_##name(int16_t *tmp, const void *src, ptrdiff_t src_stride, int w, int h, int mx, int my, \
                        int bitdepth_max) {                                                              \
        (void)mi_dsp_mc_prep(f, tmp, src, src_stride, w, h, mx, my, bitdepth_max);                        \
    }                                                                                                    \
    void mi_prep_##name##_scaled(int16_t *tmp, const void *src, ptrdiff_t src_stride, int w, int h, int mx, \
                                 int my, int dx, int dy, int bitdepth_max) {                              \
        (void)mi_dsp_mc_scaled(1, f, tmp, 0, src, src_stride, w, h, mx, my, dx, dy, bitdepth_max);        \
    }
MI_FILTER2D_SLOTS(MI_DEF_MC)
#undef MI_DEF_MC

void mi_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
            int bitdepth_max) {
    (void)mi_dsp_mc_avg(dst, dst_stride, tmp1, tmp2, w, h, bitdepth_max);
}
void mi_w_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h, int weight,
              int bitdepth_max) {
    (void)mi_dsp_mc_w_avg(dst, dst_stride, tmp1, tmp2, w, h, weight, bitdepth_max);
}
void mi_mask(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
             const uint8_t *mask, int bitdepth_max) {
    (void)mi_dsp_mc_mask(dst, dst_stride, tmp1, tmp2, w, h, mask, bitdepth_max);
}
#define MI_DEF_WMASK(ss, layout)                                                                          \
    void mi_w_mask_##ss(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w,  \
                        int h, uint8_t *mask, int sign, int bitdepth_max) {                              \
        (void)mi_dsp_mc_w_mask(layout, dst, dst_stride, tmp1, tmp2, w, h, mask, sign, bitdepth_max);      \
    }
MI_DEF_WMASK(444, 3)
MI_DEF_WMASK(422, 2)
MI_DEF_WMASK(420, 1)
#undef MI_DEF_WMASK
void mi_warp_affine_8x8(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                        const int16_t *abcd, int mx, int my, int bitdepth_max) {
    (void)mi_dsp_mc_warp8x8(0, dst, dst_stride, src, src_stride, abcd, mx, my, bitdepth_max);
}
void mi_warp_affine_8x8t(int16_t *tmp, ptrdiff_t tmp_stride, const void *src, ptrdiff_t src_stride,
                         const int16_t *abcd, int mx, int my, int bitdepth_max) {
    (void)mi_dsp_mc_warp8x8(1, tmp, tmp_stride, src, src_stride, abcd, mx, my, bitdepth_max);
}
void mi_resize(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int dst_w, int h, int src_w,
               int dx, int mx0, int bitdepth_max) {
    (void)mi_dsp_mc_resize(dst, dst_stride, src, src_stride, dst_w, h, src_w, dx, mx0, bitdepth_max);
}

// ---- loop filter ----
#define MI_DEF_LPF(name, cls, dir)                                                                         \
    void mi_lpf_##name(void *dst, ptrdiff_t stride, const uint32_t *mask, const uint8_t (*lvl)[4],         \
                       ptrdiff_t lvl_stride, const void *lut, int w, int bitdepth_max) {                   \
        (void)mi_dsp_loop_filter_sb(cls, dir, dst, stride, mask, lvl, lvl_stride, lut, w, bitdepth_max);    \
    }
MI_DEF_LPF(h_sb_y, 0, 0)
MI_DEF_LPF(v_sb_y, 0, 1)
MI_DEF_LPF(h_sb_uv, 1, 0)
MI_DEF_LPF(v_sb_uv, 1, 1)
#undef MI_DEF_LPF

// ---- cdef ----
int mi_cdef_dir(const void *dst, ptrdiff_t stride, unsigned *var, int bitdepth_max) {
    const int d = mi_dsp_cdef_dir(dst, stride, var, bitdepth_max);
    return d < 0 ? 0 : d;
}
#define MI_DEF_CDEF(wh, fb)                                                                                \
    void mi_cdef_filter_##wh(void *dst, ptrdiff_t stride, const void *left, const void *top,               \
                             const void *bottom, int pri_strength, int sec_strength, int dir, int damping,  \
                             unsigned edges, int bitdepth_max) {                                           \
        (void)mi_dsp_cdef_filter(fb, dst, stride, left, top, bottom, pri_strength, sec_strength, dir,      \
                                 damping, (int)edges, bitdepth_max);                                       \
    }
MI_DEF_CDEF(8x8, 0)
MI_DEF_CDEF(4x8, 1)
MI_DEF_CDEF(4x4, 2)
#undef MI_DEF_CDEF

// ---- loop restoration ----
void mi_wiener_filter7(void *dst, ptrdiff_t stride, const void *left, const void *lpf, int w, int h,
                       const void *params, unsigned edges, int bitdepth_max) {
    (void)mi_dsp_lr_wiener(dst, stride, left, lpf, w, h, params, (int)edges, bitdepth_max);
}
// the reference fills both wiener slots with the same C function (looprestoration.rs:3549-3550);
// the 5-tap slot receives chroma taps whose outer coefficient is 0
void mi_wiener_filter5(void *dst, ptrdiff_t stride, const void *left, const void *lpf, int w, int h,
                       const void *params, unsigned edges, int bitdepth_max) {
    (void)mi_dsp_lr_wiener(dst, stride, left, lpf, w, h, params, (int)edges, bitdepth_max);
}
#define MI_DEF_SGR(name, kind)                                                                            \
    void mi_sgr_filter_##name(void *dst, ptrdiff_t stride, const void *left, const void *lpf, int w, int h, \
                              const void *params, unsigned edges, int bitdepth_max) {                     \
        (void)mi_dsp_lr_sgr(kind, dst, stride, left, lpf, w, h, params, (int)edges, bitdepth_max);         \
    }
MI_DEF_SGR(5x5, 0)
MI_DEF_SGR(3x3, 1)
MI_DEF_SGR(mix, 2)
#undef MI_DEF_SGR

// ---- film grain ----
void mi_generate_grain_y(void *buf, const MiFilmGrainData *data, int bitdepth_max) {
    (void)mi_dsp_fg_generate_grain_y(buf, data, bitdepth_max);
}
#define MI_DEF_FG(ss, layout)                                                                              \
    void mi_generate_grain_uv_##ss(void *buf, const void *buf_y, const MiFilmGrainData *data, intptr_t uv, \
                                   int bitdepth_max) {                                                    \
        (void)mi_dsp_fg_generate_grain_uv(layout, buf, buf_y, data, (int)uv, bitdepth_max);                \
    }                                                                                                     \
    void mi_fguv_32x32xn_##ss(void *dst_row, const void *src_row, ptrdiff_t stride,                        \
                              const MiFilmGrainData *data, size_t pw, const uint8_t *scaling,              \
                              const void *grain_lut, int bh, int row_num, const void *luma_row,           \
                              ptrdiff_t luma_stride, int uv_pl, int is_id, int bitdepth_max) {            \
        (void)mi_dsp_fguv_32x32xn(layout, dst_row, src_row, stride, data, pw, scaling, grain_lut, bh,      \
                                  row_num, luma_row, luma_stride, uv_pl, is_id, bitdepth_max);            \
    }
MI_DEF_FG(420, 1)
MI_DEF_FG(422, 2)
MI_DEF_FG(444, 3)
#undef MI_DEF_FG
void mi_fgy_32x32xn(void *dst_row, const void *src_row, ptrdiff_t stride, const MiFilmGrainData *data, size_t pw,
                    const uint8_t *scaling, const void *grain_lut, int bh, int row_num, int bitdepth_max) {
    (void)mi_dsp_fgy_32x32xn(dst_row, src_row, stride, data, pw, scaling, grain_lut, bh, row_num, bitdepth_max);
}

size_t mi_dsp_context_size(void) { return sizeof(MiDSPContext); }

int mi_fill_dsp_tables(void *dsp_ctx, int bpc) {
    if (!dsp_ctx || (bpc != 8 && bpc != 10 && bpc != 12)) return -EINVAL;
    MiDSPContext &c = *static_cast<MiDSPContext *>(dsp_ctx);
    memset(&c, 0, sizeof(c));
    const bool hbd = bpc > 8;
    // film grain (filmgrain.rs:1093-1110, new_c)
    c.fg.generate_grain_y = mi_generate_grain_y;
    c.fg.generate_grain_uv[0] = mi_generate_grain_uv_420;
    c.fg.generate_grain_uv[1] = mi_generate_grain_uv_422;
    c.fg.generate_grain_uv[2] = mi_generate_grain_uv_444;
    c.fg.fgy_32x32xn = mi_fgy_32x32xn;
    c.fg.fguv_32x32xn[0] = mi_fguv_32x32xn_420;
    c.fg.fguv_32x32xn[1] = mi_fguv_32x32xn_422;
    c.fg.fguv_32x32xn[2] = mi_fguv_32x32xn_444;
    // intra prediction (ipred.rs:2203-2255)
#define MI_SET_IPRED(mode, name) c.ipred.intra_pred[mode] = mi_ipred_##name;
    MI_IPRED_SLOTS(MI_SET_IPRED)
#undef MI_SET_IPRED
    c.ipred.cfl_ac[0] = hbd ? mi_ipred_cfl_ac_420_16bpc : mi_ipred_cfl_ac_420_8bpc;
    c.ipred.cfl_ac[1] = hbd ? mi_ipred_cfl_ac_422_16bpc : mi_ipred_cfl_ac_422_8bpc;
    c.ipred.cfl_ac[2] = hbd ? mi_ipred_cfl_ac_444_16bpc : mi_ipred_cfl_ac_444_8bpc;
    c.ipred.cfl_pred[0] = mi_ipred_cfl;
    c.ipred.cfl_pred[1] = c.ipred.cfl_pred[2] = mi_ipred_cfl_unimplemented;
    c.ipred.cfl_pred[3] = mi_ipred_cfl_left;
    c.ipred.cfl_pred[4] = mi_ipred_cfl_top;
    c.ipred.cfl_pred[5] = mi_ipred_cfl_128;
    c.ipred.pal_pred = hbd ? mi_pal_pred_16bpc : mi_pal_pred_8bpc;
    // motion compensation (mc.rs:2495-2556)
#define MI_SET_MC(f, name)                              \
    c.mc.mc[f] = mi_put_##name;                         \
    c.mc.mc_scaled[f] = mi_put_##name##_scaled;         \
    c.mc.mct[f] = mi_prep_##name;                       \
    c.mc.mct_scaled[f] = mi_prep_##name##_scaled;
    MI_FILTER2D_SLOTS(MI_SET_MC)
#undef MI_SET_MC
    c.mc.avg = mi_avg;
    c.mc.w_avg = mi_w_avg;
    c.mc.mask = mi_mask;
    c.mc.w_mask[0] = mi_w_mask_444;
    c.mc.w_mask[1] = mi_w_mask_422;
    c.mc.w_mask[2] = mi_w_mask_420;
    c.mc.blend = hbd ? mi_blend_16bpc : mi_blend_8bpc;
    c.mc.blend_v = hbd ? mi_blend_v_16bpc : mi_blend_v_8bpc;
    c.mc.blend_h = hbd ? mi_blend_h_16bpc : mi_blend_h_8bpc;
    c.mc.warp8x8 = mi_warp_affine_8x8;
    c.mc.warp8x8t = mi_warp_affine_8x8t;
    c.mc.emu_edge = hbd ? mi_emu_edge_16bpc : mi_emu_edge_8bpc;
    c.mc.resize = mi_resize;
    // inverse transforms (itx.rs:1072-1110)
#define MI_SET_ITX(tx, txtp, name) c.itx.itxfm_add[tx][txtp] = mi_inv_txfm_add_##name;
    MI_ITX_SLOTS(MI_SET_ITX)
#undef MI_SET_ITX
    // loop filter (loopfilter.rs:1079-1084): [luma, chroma][column edges, row edges]
    c.lf.loop_filter_sb[0][0] = mi_lpf_h_sb_y;
    c.lf.loop_filter_sb[0][1] = mi_lpf_v_sb_y;
    c.lf.loop_filter_sb[1][0] = mi_lpf_h_sb_uv;
    c.lf.loop_filter_sb[1][1] = mi_lpf_v_sb_uv;
    // CDEF (cdef.rs:1296-1302)
    c.cdef.dir = mi_cdef_dir;
    c.cdef.fb[0] = mi_cdef_filter_8x8;
    c.cdef.fb[1] = mi_cdef_filter_4x8;
    c.cdef.fb[2] = mi_cdef_filter_4x4;
    // loop restoration (looprestoration.rs:3545-3556)
    c.lr.wiener[0] = mi_wiener_filter7;
    c.lr.wiener[1] = mi_wiener_filter5;
    c.lr.sgr[0] = mi_sgr_filter_5x5;
    c.lr.sgr[1] = mi_sgr_filter_3x3;
    c.lr.sgr[2] = mi_sgr_filter_mix;
    c.initialized = true;
    return 0;
}

}  // extern "C"
