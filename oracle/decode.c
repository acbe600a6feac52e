/*
 * decode.c — the oracle's frame reconstruction driver: runs one front-end work list
 * (MiDecFrame, include/mi_av1dec.h) through the CPU restatement in the reference's order.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Order, as rav1d decodes a frame with one thread (decode.rs decode_frame_main ->
 * decode_tile_sbrow + filter_sbrow; recon.rs:4019-4211 filter_sbrow):
 *   reconstruction of every block (inter prediction of all inter blocks and their residuals --
 *   they read only reference pictures, so doing them first changes no pixel -- then the intra
 *   blocks in decode order: recon_b_intra's prediction, then itxfm_add per transform block)
 *   -> deblock (lf_apply.rs, sbrow order, in place) -> CDEF
 *   (cdef_apply.rs, reads the deblocked picture) -> loop restoration (lr_apply.rs, reads the
 *   CDEF output and the deblocked rows across stripe edges).
 * Film grain is applied by the caller to output pictures only (fg_apply.rs).
 */
#include <stdlib.h>
#include <string.h>

#include "mi_av1dec.h"
#include "oracle.h"

void oracle_cdef_frame(void *const dst[3], void *const src[3], const ptrdiff_t strides[3], int w,
                       int h, int layout, int bpc, const void *masks_, int sb128w, int damping_hdr,
                       const uint8_t *y_strength, const uint8_t *uv_strength);
void oracle_deblock_frame(void *const planes[3], const ptrdiff_t strides[3], int w, int h,
                          int layout, int bpc, const uint8_t *level, ptrdiff_t b4_stride,
                          const void *masks_, int sb128w, int sb128, const uint8_t *lut_e,
                          const uint8_t *lut_i, int filter_y, int filter_uv);
void oracle_lr_frame(void *const dst[3], void *const cdef[3], void *const deblocked[3],
                     const ptrdiff_t strides[3], int w, int h, int layout, int bpc, int sb128,
                     int restore_planes, const int unit_size_log2[2], const void *lr_mask,
                     int sb128w);

/* pic: the picture to reconstruct (128-aligned planes, cleared or not); scratch1/2: two more
 * pictures of the same geometry. On return the final (reference) picture is in out[], which
 * points at one of the three. */
void oracle_decode_frame_refs(const MiDecFrame *f, void *const pic[3], void *const scratch1[3],
                              void *const scratch2[3], const ptrdiff_t strides[3], void *const *refs,
                              const ptrdiff_t *ref_strides, const int *ref_wh, void **out)
{
    const int bpc = f->bpc, layout = f->layout;
    const int ss_ver = layout == 1;
    const int nplanes = layout ? 3 : 1;
    const size_t cb = bpc == 8 ? 2 : 4;
    const ptrdiff_t st2[2] = { strides[0], strides[1] };
    /* the arena is consumed by the transforms: work on a copy */
    void *coef = malloc(f->ncoef * cb + 16);
    memcpy(coef, f->coef, f->ncoef * cb);

    /* 1. inter prediction of every inter block (recon_b_inter, recon.rs:3162-3940): the units
     * read only reference pictures, so they run before any residual. Within a compound block
     * the luma SEG unit precedes the chroma units that read its mask. */
    if (f->n_mc || f->n_warp || f->n_scaled || f->n_combine_y || f->n_obmc_h || f->n_obmc_v) {
        int16_t *tmp = malloc(sizeof(int16_t) * (f->ntmp + 1));
        uint8_t *masks = malloc(f->nmasks + 1);
        if (f->nmasks) memcpy(masks, f->masks, f->nmasks);
        oracle_mc_frame(pic, st2, layout, bpc, refs, ref_strides, ref_wh, f->mc, f->n_mc, masks, tmp);
        oracle_mc_warp_frame(pic, st2, layout, bpc, refs, ref_strides, ref_wh, f->warp, f->n_warp, tmp);
        oracle_mc_scaled_frame(pic, st2, layout, bpc, f->w, f->h, refs, ref_strides, ref_wh, f->scaled, f->n_scaled,
                               tmp);
        oracle_mc_combine_frame(pic, st2, layout, bpc, f->combine_y, f->n_combine_y, tmp, masks);
        oracle_mc_combine_frame(pic, st2, layout, bpc, f->combine_uv, f->n_combine_uv, tmp, masks);
        /* obmc(): the above laps, then the left laps (recon.rs:2205-2309); a lap whose
         * reference differs in size goes through the scaled path */
        for (int k = 0; k < 2; k++) {
            const MiMcBlock *u = k ? f->obmc_v : f->obmc_h;
            const int n = k ? f->n_obmc_v : f->n_obmc_h;
            for (int i = 0; i < n; i++) {
                const int r = u[i].ref[0];
                if (ref_wh[r * 2] != f->w || ref_wh[r * 2 + 1] != f->h)
                    oracle_mc_scaled_frame(pic, st2, layout, bpc, f->w, f->h, refs, ref_strides, ref_wh, &u[i], 1, tmp);
                else
                    oracle_mc_frame(pic, st2, layout, bpc, refs, ref_strides, ref_wh, &u[i], 1, masks, tmp);
            }
        }
        free(tmp);
        free(masks);
    }
    /* 2. the residuals of inter blocks (read_coef_tree / recon_b_inter's chroma itxfm_add) */
    if (f->n_inter_tx) oracle_itx_frame(pic, strides, f->inter_tx, f->n_inter_tx, coef, (1 << bpc) - 1);
    /* 3. intra path in decode order (intra blocks of the frame, inter-intra blends) */
    if (f->n_intra)
        oracle_intra_recon(pic, st2, bpc, f->intra, f->intra_tx, f->n_intra, NULL, f->idx, f->pal, coef);
    free(coef);
    /* 2. deblocking, in place */
    if (f->filter_y)
        oracle_deblock_frame(pic, strides, f->w, f->h, layout, bpc, f->lf_level, f->b4_stride, f->lf_masks,
                             f->sb128w, f->sb128, f->lim_e, f->lim_i, f->filter_y, f->filter_uv);
    /* 3. CDEF: deblocked -> scratch1 */
    void *const *cdef_out = pic;
    if (f->cdef_on) {
        oracle_cdef_frame(scratch1, pic, strides, f->w, f->h, layout, bpc, f->lf_masks, f->sb128w,
                          f->cdef_damping, f->cdef_y, f->cdef_uv);
        cdef_out = scratch1;
    }
    void *const *deblocked = pic;
    /* 3b. super-resolution (recon.rs:4215-4285 filter_sbrow_resize; lf_apply.rs backup_lpf
     * resizes the deblocked rows loop restoration reads the same way): every picture has the
     * upscaled geometry; the CDEF output goes to scratch2, the deblocked picture to scratch1
     * (the CDEF output at coded width is no longer read), and LR writes into pic. */
    if (f->up_w != f->w) {
        const int ss_hor = layout == 1 || layout == 2;
        const int in_cw = (f->w + ss_hor) >> ss_hor, out_cw = (f->up_w + ss_hor) >> ss_hor;
        int step[2], start[2];
        step[0] = ((f->w << 14) + (f->up_w >> 1)) / f->up_w;          /* scale_fac, decode.rs:4644 */
        step[1] = ((in_cw << 14) + (out_cw >> 1)) / out_cw;
        for (int k = 0; k < 2; k++) {                                  /* get_upscale_x0, :4776 */
            const int iw = k ? in_cw : f->w, ow = k ? out_cw : f->up_w;
            const int err = ow * step[k] - (iw << 14);
            start[k] = ((-((ow - iw) << 13) + (ow >> 1)) / ow + 128 - err / 2) & 0x3fff;
        }
        const int bw4 = ((f->w + 7) >> 3) << 1;
        void *const *src_sets[2] = { cdef_out, pic };
        void *const *dst_sets[2] = { scratch2, scratch1 };
        for (int s2 = 0; s2 < (f->restore_planes ? 2 : 1); s2++)
            for (int p = 0; p < nplanes; p++) {
                const int sh = p ? ss_hor : 0, sv = p ? ss_ver : 0;
                oracle_mc_resize(dst_sets[s2][p], strides[p], src_sets[s2][p], strides[p], (f->up_w + sh) >> sh,
                                 (f->h + sv) >> sv, (4 * bw4 + sh) >> sh, step[p != 0], start[p != 0], bpc);
            }
        cdef_out = scratch2;
        deblocked = f->restore_planes ? scratch1 : scratch2;
    }
    /* 4. loop restoration: (CDEF output, deblocked) -> scratch2 (pic with super-resolution) */
    void *const *final = cdef_out;
    if (f->restore_planes) {
        void *const *lr_out = f->up_w != f->w ? pic : scratch2;
        oracle_lr_frame(lr_out, (void *const *)cdef_out, deblocked, strides, f->up_w, f->h, layout, bpc, f->sb128,
                        f->restore_planes, f->lr_unit_size, f->lr_mask, f->lr_sb128w);
        final = lr_out;
    }
    (void)ss_ver;
    for (int p = 0; p < 3; p++) out[p] = p < nplanes ? final[p] : NULL;
}

/* An intra frame (no references). */
void oracle_decode_frame(const MiDecFrame *f, void *const pic[3], void *const scratch1[3],
                         void *const scratch2[3], const ptrdiff_t strides[3], void **out)
{
    oracle_decode_frame_refs(f, pic, scratch1, scratch2, strides, NULL, NULL, NULL, out);
}
