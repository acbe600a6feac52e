/*
 * mi_av1dsp.h — C-ABI boundary of the MI355X-native AV1 decode-DSP path.
 *
 * Drop-in for rav1d's DSP function-pointer tables (Rav1dDSPContext, src/internal.rs:111-121;
 * C twin src/internal.h:61-69). Two surfaces:
 *
 *  1. Batched per-frame API (the performance path): the host front-end hands the device one
 *     descriptor list per frame and per stage, after pass-1 entropy (src/decode.rs:1203-1282,
 *     src/thread_task.rs:1048-1068). All buffers are device pointers; work is enqueued on the
 *     caller's HIP stream (passed as an opaque `void*`) and returns without synchronising.
 *
 *  2. Table-compatible per-call entry points (mi_dsp_*): exactly the reference's per-block
 *     signatures (trailing bitdepth_max always passed, as in rav1d). Buffers may be host or
 *     device memory; each call is a synchronous single-block device launch. They exist for
 *     drop-in parity testing, not speed (launch cost >> work).
 *
 * Conventions, as in the reference:
 *  - pixel = uint8_t (8 bpc) or uint16_t (10/12 bpc); coef = int16_t (8 bpc) or int32_t;
 *    strides are in BYTES (include/common/bitdepth.rs:113-125).
 *  - return 0 or a negative errno, matching Dav1dResult (src/error.rs:27-45):
 *    -EINVAL bad descriptor, -ENOMEM allocation, -EIO device fault/launch failure,
 *    -ENODEV no usable gfx950 device.
 *  - No HIP/torch types appear in this header.
 */
#ifndef MI_AV1DSP_H
#define MI_AV1DSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MI_AV1DSP_ABI_VERSION 1

/* ------------------------------------------------------------------------------------ */
/* Shared descriptors                                                                    */
/* ------------------------------------------------------------------------------------ */

/* A picture resident in device memory. Mirrors the plane/stride part of Dav1dPicture
 * (include/dav1d/picture.rs; C include/dav1d/picture.h:59-90). layout: Dav1dPixelLayout
 * (0 I400, 1 I420, 2 I422, 3 I444). stride[1] is shared by both chroma planes. */
typedef struct MiPicture {
    void     *data[3];
    ptrdiff_t stride[2];
    int32_t   w, h;          /* luma size in pixels */
    int32_t   layout;
    int32_t   bpc;           /* 8, 10 or 12 */
} MiPicture;

/* One transform block of the frame's coefficient arena (pass-2 input of itxfm_add:
 * src/recon.rs:1781-1788, 2674-2682, 3116, 4013). The arena stores each block's
 * coefficients column-major with column height min(h,32) — exactly the layout itxfm_add
 * reads (coeff[y + x*sh], src/itx.rs:128-142). 16 bytes.
 *
 * Packed blocks (flags & MI_TX_PACKED): every non-zero coefficient lies in the top-left
 * CW x CH corner (CW = MI_TX_PACKED_CW(flags) <= min(w,32), CH = MI_TX_PACKED_CH(flags) <=
 * min(h,32), multiples of 4), and the arena holds only that corner, ROW-major (coefficient
 * (x, y) at coef_off + y*CW + x, coef_off a multiple of 4); the rest of the block reads as
 * zero. A low-frequency block of a large transform then costs CW*CH arena entries instead of
 * min(w,32)*min(h,32), and a transform row is CW/4 vector loads. The front-end emits every
 * non-DC block of more than 16 coefficients packed. With MI_TX_I16 as well (10/12-bit arenas
 * only) the corner's coefficients are int16: coefficient (x, y) is
 * ((const int16_t *)(arena + coef_off))[y*CW + x] and the block spans CW*CH/2 int32 entries
 * (the front-end sets it when every coefficient of the corner fits). Other flag bits: 0. The
 * DSP-table entry points (itxfm_add) keep the reference's dense layout. */
#define MI_TX_PACKED 0x80u
#define MI_TX_I16 0x40u
#define MI_TX_PACKED_CW(f) (((((unsigned)(f)) >> 3) & 7u) * 4u + 4u)
#define MI_TX_PACKED_CH(f) ((((unsigned)(f)) & 7u) * 4u + 4u)
#define MI_TX_PACK(cw, ch) ((uint8_t)(MI_TX_PACKED | ((((cw) >> 2) - 1) << 3) | (((ch) >> 2) - 1)))
typedef struct MiTxBlock {
    uint32_t coef_off;       /* offset in coefficients (not bytes) into the arena */
    uint16_t x, y;           /* top-left pixel in `plane` */
    uint8_t  plane;          /* 0 Y, 1 U, 2 V */
    uint8_t  tx;             /* RectTxfmSize (src/levels.rs:46-82) */
    uint8_t  txtp;           /* TxfmType 0..15, or 16 = WHT_WHT (lossless) */
    uint8_t  flags;          /* 0, or MI_TX_PACK(cw, ch): the arena holds the packed corner */
    int32_t  eob;            /* end-of-block as passed to itxfm_add */
} MiTxBlock;

#define MI_N_RECT_TX_SIZES 19

/* Per-128x128 loop-filter / CDEF metadata: byte-identical to the reference's Av1Filter
 * (src/lf_mask.rs:40-51; C src/lf_mask.h:51-57), so the host can hand over f->lf.mask as is.
 * Edge masks must already carry the tile-boundary fixups of rav1d_loopfilter_sbrow_cols
 * (src/lf_apply.rs:625-705). 1348 bytes, 2-byte aligned. */
typedef struct MiAv1Filter {
    uint16_t filter_y[2][32][3][2];   /* [0 col edges, 1 row edges][pos][wd 4/8/16][half] */
    uint16_t filter_uv[2][32][2][2];  /* [dir][pos][wd 4/6][half] */
    int8_t   cdef_idx[4];             /* per 64x64, -1 = unset */
    uint16_t noskip_mask[16][2];      /* per 8x8, stored on a 4x8 basis */
} MiAv1Filter;

/* Frame-level deblocking inputs (Rav1dFrameData.lf, src/internal.rs:557-576). */
typedef struct MiLoopFilter {
    const uint8_t *level;        /* device: [u8;4] per 4x4 unit {Y col-edge, Y row-edge, U, V};
                                  * U/V slots are addressed at chroma 4x4 coordinates */
    ptrdiff_t b4_stride;         /* level entries per row */
    const MiAv1Filter *masks;    /* device: [sb128h][sb128w] */
    int32_t sb128w;
    int32_t filter_y;            /* frame_hdr.loopfilter.level_y[0] || level_y[1] */
    int32_t filter_uv;           /* level_u || level_v */
    uint8_t lim_e[64], lim_i[64];/* Av1FilterLUT.e / .i (rav1d_calc_eih) */
} MiLoopFilter;

/* Frame-level CDEF parameters (Dav1dFrameHeader.cdef, include/dav1d/headers.rs:2324;
 * C include/dav1d/headers.h Dav1dCdefParams) plus the per-64x64 indices/skip masks that live
 * in the Av1Filter array. */
typedef struct MiCdef {
    const MiAv1Filter *masks;    /* device: [sb128h][sb128w] (cdef_idx, noskip_mask) */
    int32_t sb128w;
    int32_t damping;             /* frame_hdr.cdef.damping (3..6) */
    uint8_t y_strength[8];       /* pri << 2 | sec, as coded */
    uint8_t uv_strength[8];
    /* Optional (NULL: grid order): the order the 64x64-unit workgroups run in, a device array
     * of mi_cdef_tile_order's length and contents. */
    const int32_t *order;
} MiCdef;

/* The order mi_cdef_frame's workgroups run best in: the 64x64 units by descending cost (a
 * primary strength: direction search and filter; a secondary strength only; nothing to filter:
 * a copy), longest first, each class dealt to the 8 XCDs in contiguous picture runs (workgroup
 * b runs on XCD b % 8) so that neighbouring units share an L2. A host call on a host copy of the Av1Filter array for a w x h
 * picture: writes the unit indices into `order` (capacity n) and returns their count, or
 * -EINVAL. */
int mi_cdef_tile_order(const MiAv1Filter *masks_host, int w, int h, int layout, const MiCdef *cdef, int32_t *order,
                       int n);

/* Loop-restoration unit parameters, byte-identical to Av1RestorationUnit / Av1Restoration
 * (src/lf_mask.rs:31-38, 55-58; C src/lf_mask.h:42-62). type: Dav1dRestorationType
 * (0 NONE, 2 WIENER, 3 + sgr_idx for SGRPROJ). */
typedef struct MiAv1RestorationUnit {
    uint8_t type;
    int8_t  filter_h[3];
    int8_t  filter_v[3];
    int8_t  sgr_weights[2];
} MiAv1RestorationUnit;
typedef struct MiAv1Restoration {
    MiAv1RestorationUnit lr[3][4];   /* [plane][64x64 quadrant of the 128x128] */
} MiAv1Restoration;                  /* 108 bytes */

typedef struct MiLr {
    const MiAv1Restoration *lr_mask; /* device: [sb128h][sb128w] (f->lf.lr_mask) */
    int32_t sb128w;
    int32_t restore_planes;          /* bit0 Y, bit1 U, bit2 V (f->lf.restore_planes) */
    int32_t unit_size_log2[2];       /* frame_hdr.restoration.unit_size[luma, chroma] */
    /* Optional (NULL: grid order): the order the (plane, stripe, tile) workgroups run in, a
     * device array of mi_lr_tile_order's length and contents. */
    const int32_t *order;
} MiLr;

/* The order mi_lr_frame's workgroups run best in: the restoration tiles by descending cost
 * (self-guided with both radii, with one, Wiener, copy), so that the longest start first and the
 * grid does not end on a tail of them (longest-processing-time-first). A host call on a host
 * copy of the lr_mask for a w x h picture of `layout`: writes the tile indices into `order`
 * (capacity n) and returns their count, or -EINVAL. */
int mi_lr_tile_order(const MiAv1Restoration *lr_mask_host, int w, int h, int layout, const MiLr *lr,
                     int32_t *order, int n);

/* Film-grain parameters, byte-identical to Dav1dFilmGrainData (include/dav1d/headers.h:
 * 315-333; Rust Rav1dFilmGrainData include/dav1d/headers.rs:1585-1610). */
typedef struct MiFilmGrainData {
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
} MiFilmGrainData;

/* One motion-compensated prediction unit: a block's rectangle in one plane (24 bytes).
 * Replaces the per-block arguments of recon's mc() (src/recon.rs:2025-2203; C
 * recon_tmpl.c:962-1011) plus the compound dispatch (recon_tmpl.c:1836-1921). */
#define MI_MC_AVG  0   /* COMP_INTER_AVG: avg(tmp[0], tmp[1]) */
#define MI_MC_WAVG 1   /* COMP_INTER_WEIGHTED_AVG: w_avg(tmp[0], tmp[1], weight) */
#define MI_MC_MASK 2   /* COMP_INTER_WEDGE (and chroma of SEG): mask(tmp[sign], tmp[!sign], mask) */
#define MI_MC_SEG  3   /* COMP_INTER_SEG, luma: w_mask(tmp[sign], tmp[!sign]); writes the chroma mask */
/* single-reference units (ref[1] < 0) with a non-default destination: */
#define MI_MC_OBMC_H 4 /* OBMC lap of the above neighbour (obmc(), recon.rs:2225-2266): put w x h, then
                          blend_h into cur: rows y < (param * 3) >> 2, mask obmc_masks[param + y];
                          param = the blend height v_mul * oh4, h = the lap height rounded up to a
                          power of two (the extra rows are not stored) */
#define MI_MC_OBMC_V 5 /* OBMC lap of the left neighbour (recon.rs:2267-2306): put w x h, then
                          blend_v into cur: columns x < (w * 3) >> 2, mask obmc_masks[w + x] */
#define MI_MC_PREP   6 /* prep (mct) into the int16 tmp arena at element mask_off, row pitch w: one
                          side of a compound whose other side is warped or scaled (mi_mc_combine) */
typedef struct MiMcBlock {
    uint16_t x, y;          /* top-left, plane pixels */
    uint8_t  w, h;          /* plane pixels, 2..128 (bw4 * h_mul, bh4 * v_mul) */
    uint8_t  plane;         /* 0..2 */
    uint8_t  filter2d;      /* enum Filter2d (src/levels.rs): 0..8 8-tap (h, v) pairs, 9 bilinear */
    int16_t  mvx[2], mvy[2];/* per reference, luma 1/8-pel units as coded (mv.x, mv.y) */
    int8_t   ref[2];        /* index into the refs[] array; ref[1] < 0: single prediction (put) */
    uint8_t  comp;          /* MI_MC_* for compound units */
    uint8_t  param;         /* bits 0-4: w_avg weight (jnt_weights), bit 7: mask_sign */
    uint32_t mask_off;      /* byte offset into the mask buffer (MASK: w*h read; SEG: written at
                               the chroma resolution, (w >> ss_hor) * (h >> ss_ver)) */
} MiMcBlock;

/* One intra-predicted block (24 bytes) for the batched intra entry. Mode = the reference's
 * intra_pred[] slot (src/levels.rs IntraPredMode implementation modes: 0 DC, 1 V, 2 H,
 * 3 LEFT_DC, 4 TOP_DC, 5 DC_128, 6 Z1, 7 Z2, 8 Z3, 9 SMOOTH, 10 SMOOTH_V, 11 SMOOTH_H,
 * 12 PAETH, 13 FILTER), MI_IPRED_CFL + dc slot for cfl_pred, or MI_IPRED_PAL for pal_pred. */
#define MI_IPRED_CFL 32   /* + 0 DC, 3 LEFT_DC, 4 TOP_DC, 5 DC_128 (cfl_pred[], ipred.rs:236) */
#define MI_IPRED_PAL 64   /* palette (8 pixels) at edge_off, indices (w*h bytes) at idx + aux_off */
typedef struct MiIpredBlock {
    uint32_t edge_off;      /* pixel index of the topleft sample in the edge buffer */
    uint32_t aux_off;       /* CfL: int16 index into ac (w*h entries); PAL: byte index into idx */
    uint16_t x, y;          /* destination, plane pixels */
    uint8_t  w, h;          /* 4..64 (FILTER <= 32) */
    uint8_t  plane;
    uint8_t  mode;
    uint16_t angle;         /* the intra_pred `angle` argument: angle | is_sm << 9 | edge filter << 10,
                               or the filter index for FILTER (ipred.rs:48-58, 866-868) */
    uint16_t max_w, max_h;  /* max_width / max_height (Z2 edge-filter limits) */
    int8_t   alpha;         /* CfL alpha */
    uint8_t  pad;
} MiIpredBlock;

/* One 8x8 block of a warped prediction (warp_affine, recon.rs:2311-2400): the arguments of
 * one warp8x8 / warp8x8t call with the source position instead of a pointer (40 bytes). */
typedef struct MiWarpBlock {
    uint16_t x, y;          /* destination top-left, plane pixels */
    uint8_t  plane;
    int8_t   ref;           /* index into refs[] */
    uint8_t  prep;          /* 0: warp8x8 into cur; 1: warp8x8t into tmp at tmp_off, pitch tmp_stride */
    uint8_t  pad0;
    int32_t  dx, dy;        /* warp_affine's dx, dy: the 8x8's source origin (window = dx-3 .. dx+11) */
    int32_t  mx, my;        /* filter phases as passed to warp8x8 */
    int16_t  abcd[4];       /* Rav1dWarpedMotionParams.abcd */
    uint32_t tmp_off;       /* int16 element offset of the block in tmp */
    uint16_t tmp_stride;    /* elements */
    uint16_t pad1;
} MiWarpBlock;

/* One compound combine from two prep intermediates in the tmp arena (the avg / w_avg / mask /
 * w_mask step of recon_b_inter, recon.rs:3292-3331, when a side was warped or scaled). 24 bytes. */
typedef struct MiMcCombine {
    uint16_t x, y;          /* destination, plane pixels */
    uint8_t  w, h;          /* plane pixels */
    uint8_t  plane;
    uint8_t  comp;          /* MI_MC_AVG .. MI_MC_SEG */
    uint8_t  param;         /* as MiMcBlock.param */
    uint8_t  pad[3];
    uint32_t tmp_off[2];    /* element offsets of tmp[0], tmp[1] (row pitch w) */
    uint32_t mask_off;      /* as MiMcBlock.mask_off */
} MiMcCombine;

/* One intra-predicted transform block whose edges the device gathers from the picture itself
 * (rav1d_prepare_intra_edges, src/ipred_prepare.rs:118-204, run in the kernel), 32 bytes.
 * Neighbour pixels must be final when the launch runs: one dependency level per launch. The
 * picture holds unfiltered reconstruction for the whole frame (deblocking runs after all
 * recon), so the reference's pre-filter top-SB-row backup (recon.rs:2532-2540) is the picture
 * row itself. */
#define MI_INTRA_HAVE_LEFT   1u   /* x > tile column start (recon.rs:2554) */
#define MI_INTRA_HAVE_TOP    2u   /* y > tile row start */
#define MI_INTRA_TOP_RIGHT   4u   /* EdgeFlags::I444_TOP_HAS_RIGHT (or the I420/I422 flag for chroma) */
#define MI_INTRA_BOTTOM_LEFT 8u   /* EdgeFlags::I444_LEFT_HAS_BOTTOM (or chroma flag) */
#define MI_INTRA_SMOOTH_NB  16u   /* sm_flag / sm_uv_flag of a neighbour (angle bit 9) */
#define MI_INTRA_EDGE_FILTER 32u  /* seq_hdr.intra_edge_filter (angle bit 10) */
#define MI_INTRA_II         64u   /* inter-intra: blend into the pixels with the mask at idx + aux_off */
#define MI_INTRA_CFL_AC    128u   /* CfL with the AC computed on the device (cfl_ac, ipred.rs:1326-1432)
                                     from the reconstructed luma under the block, instead of read
                                     from ac + aux_off: reserved = w_pad | h_pad << 8 | ss_hor << 16 |
                                     ss_ver << 17 (w, h = cw, ch of cfl_ac). The block's dependencies
                                     (mi_intra_recon deps / its level) must include the luma blocks
                                     that own the pixels it reads. */
typedef struct MiIntraBlock {
    uint16_t x, y;          /* plane pixels */
    uint8_t  w, h;          /* transform size, pixels (4..64) */
    uint8_t  plane;
    uint8_t  mode;          /* y_mode / uv_mode as coded (levels.rs IntraPredMode DC_PRED .. PAETH_PRED
                               = 0 .. 12), 13 = filter intra (FILTER_PRED), MI_IPRED_CFL (uv CfL, edges
                               as DC_PRED), MI_IPRED_PAL (palette) */
    int8_t   angle;         /* angle delta (-3 .. 3) of a directional mode */
    uint8_t  flags;         /* MI_INTRA_* */
    uint8_t  filt_idx;      /* filter-intra mode (FILTER) */
    int8_t   alpha;         /* CfL alpha */
    uint16_t tile_w, tile_h;/* tile column / row end, plane pixels (edge availability limits) */
    uint16_t max_w, max_h;  /* intra_pred's max_width / max_height */
    uint32_t aux_off;       /* CfL: int16 index into ac; PAL: byte index into idx; II: mask byte index */
    uint32_t pal_off;       /* PAL: pixel index of the block's 8-entry palette in `pal` */
    uint32_t reserved;      /* MI_INTRA_CFL_AC: w_pad | h_pad << 8 | ss_hor << 16 | ss_ver << 17; else 0 */
} MiIntraBlock;

#define MI_INTRA_IBC 96    /* MiIntraBlock.mode: intra block copy, the bilinear put (mc[FILTER_2D_BILINEAR],
                              mc.rs:1322-1338) from the current picture as recon's mc() does with
                              the frame itself as reference (recon.rs:3236-3290): reserved =
                              (uint16)mv.x | mv.y << 16 (luma 1/8 pel as coded), filt_idx = ss_hor |
                              ss_ver << 1 of the block's plane; max_w / max_h = the reference area
                              mc() clamps to for intrabc (f.bw * 4 >> ss_hor, f.bh * 4 >> ss_ver,
                              recon.rs:2052-2083: reads outside it replicate its border, as
                              emu_edge); the block's dependencies must cover the source rectangle
                              (plus one column / row when the chroma phase is half-pel) */
#define MI_INTRA_RESID 97  /* MiIntraBlock.mode: no prediction, the residual of a transform block of an
                              inter-intra block (recon_b_inter's itxfm_add after the blend,
                              recon.rs:3940-4045) added to the pixels already there; its dependencies
                              must cover its own rectangle (the MI_INTRA_II block) */
#define MI_IPRED_II 128    /* mode flag: inter-intra, blend the prediction into the existing
                              (inter) pixels with the mask at idx + aux_off (mc.blend,
                              recon.rs:3524-3543): only with slots 0-12 */

/* ------------------------------------------------------------------------------------ */
/* Context                                                                               */
/* ------------------------------------------------------------------------------------ */

typedef struct MiCtx MiCtx;

/* Create a context bound to `device` (HIP ordinal). One context per decoder
 * frame-context; calls on one context are serialised by the caller (src/internal.rs
 * Rav1dFrameContext), different contexts are independent. */
int  mi_ctx_create(int device, MiCtx **out);
void mi_ctx_destroy(MiCtx *ctx);
/* Last device-side error observed by the context (0 if none). */
int  mi_ctx_last_error(const MiCtx *ctx);
const char *mi_version(void);

/* ------------------------------------------------------------------------------------ */
/* Batched per-frame API                                                                 */
/* ------------------------------------------------------------------------------------ */

/* Inverse transform + add for a whole frame.
 * `blocks` (device) must be grouped by tx size: blocks of size s are
 * blocks[size_start[s] .. size_start[s+1]) (host array of 20 entries). Within a group,
 * sorting by txtp / eob==0 reduces wave divergence but is not required.
 * Blocks must not overlap (true of any AV1 frame). `coef` is the device arena.
 * flags: MI_ITX_KEEP_COEFS leaves the arena untouched; by default the consumed
 * coefficients are zeroed as the reference's itxfm_add does (src/itx.rs:152-158). */
#define MI_ITX_KEEP_COEFS 1u
int mi_itx_frame(MiCtx *ctx, const MiPicture *pic, const MiTxBlock *blocks,
                 const uint32_t size_start[MI_N_RECT_TX_SIZES + 1], void *coef,
                 unsigned flags, void *stream);

/* mi_itx_frame with the blocks of each size further grouped into MI_ITX_BANDS horizontal
 * picture bands: blocks of size s in band q are blocks[band_start[s][q] .. band_start[s][q+1]),
 * with band_start[s][MI_ITX_BANDS] == band_start[s+1][0]. Any grouping gives the same pixels;
 * grouping by position (band q = plane rows [q*h/8, (q+1)*h/8), as mi_itx_band_of) makes each
 * band run on one XCD, so a pixel line is fetched into and written back from one L2 whichever
 * transform sizes touch it. */
#define MI_ITX_BANDS 8
int mi_itx_frame_banded(MiCtx *ctx, const MiPicture *pic, const MiTxBlock *blocks,
                        const uint32_t band_start[MI_N_RECT_TX_SIZES][MI_ITX_BANDS + 1], void *coef,
                        unsigned flags, void *stream);
/* mi_itx_frame_banded whose bands each begin with a run of DC-only blocks (DCT_DCT, eob < 1):
 * blocks [band_start[s][q], dc_end[s][q]) of band q of size s, band_start[s][q] <= dc_end[s][q]
 * <= band_start[s][q + 1]. The runs take a DC path (many blocks per workgroup, whole line
 * segments); a block in a run that is not DC-only is skipped and reported by
 * mi_ctx_device_status (-EINVAL). Same pixels as mi_itx_frame over the same blocks. */
/* MI_ITX_DC_DEFER (mi_itx_frame_runs only): the DC runs' constants are not added to the
 * pixels; the context records them per 4x4 unit for the next mi_deblock_frame_dc, which adds
 * them to the pixels it stages, so the deblocked picture equals that of the undeferred call
 * while the reconstruction `pic` lacks them (for frames whose reconstruction nothing else reads:
 * no intra block predicts from it). Under stream capture the flag is ignored. */
#define MI_ITX_DC_DEFER 2u
int mi_itx_frame_runs(MiCtx *ctx, const MiPicture *pic, const MiTxBlock *blocks,
                      const uint32_t band_start[MI_N_RECT_TX_SIZES][MI_ITX_BANDS + 1],
                      const uint32_t dc_end[MI_N_RECT_TX_SIZES][MI_ITX_BANDS], void *coef, unsigned flags,
                      void *stream);

/* Intra prediction of n independent blocks (one wavefront step of a frame, or any set of
 * blocks whose edges are final): writes each block into `pic` from its gathered edges
 * (rav1d_prepare_intra_edges output, src/ipred_prepare.rs:118-204). `blocks`, `edges`
 * (pixels of pic's bit depth), `ac` (int16) and `idx` (bytes) are device arrays; ac / idx may
 * be NULL when no CfL / palette block is present. */
int mi_ipred_blocks(MiCtx *ctx, const MiPicture *pic, const MiIpredBlock *blocks, int n,
                    const void *edges, const int16_t *ac, const uint8_t *idx, void *stream);

/* Intra prediction of n independent transform blocks with device-side edge gathering from
 * `pic` (MiIntraBlock): the batched replacement of recon_b_intra's per-tx-block
 * prepare_intra_edges + intra_pred / cfl_pred / pal_pred (recon.rs:2402-3160). ac / idx / pal
 * are device arrays (may be NULL when unused). */
int mi_intra_blocks(MiCtx *ctx, const MiPicture *pic, const MiIntraBlock *blocks, int n,
                    const int16_t *ac, const uint8_t *idx, const void *pal, void *stream);

/* Whole-frame intra reconstruction in ONE persistent launch: every transform block's
 * prediction (as mi_intra_blocks) plus its residual (as mi_itx_frame), in dependency order,
 * for independent frames at once (the workgroups of one frame share one XCD, hence one L2).
 * Replaces recon_b_intra's per-block prepare_intra_edges / intra_pred / itxfm_add sequence (recon.rs:2402-3160) for whole frames. Up to 24 frames per call; frame f
 * is reconstructed by the workgroups on XCD f % 8. Per frame (device arrays):
 * blocks[n] in an order where every block comes after the blocks it depends on; tx[i] is the
 * residual of blocks[i] (same plane, position and size); deps[dep_start[i] ..
 * dep_start[i + 1]) are the indices (< i) of the blocks owning any pixel blocks[i]'s edges
 * read. flags: MI_ITX_KEEP_COEFS as mi_itx_frame; MI_IR_EDGE_GRANULES when every pixel any
 * block's edges read is reconstructed by this call (intra-only frames: no inter-intra or
 * MI_INTRA_RESID blocks, no inter pixels around the blocks): blocks then hand their right
 * column and bottom row to later blocks as tagged 8-byte records instead of done flags plus
 * picture reads, and only CfL and intra block copy blocks wait on their deps. A worker that
 * waits ~0.5 s for a dependency gives up (no hang); mi_ctx_device_status reports it. */
#define MI_IR_EDGE_GRANULES 2u
typedef struct MiIntraFrame {
    MiPicture pic;
    const MiIntraBlock *blocks;
    const MiTxBlock *tx;
    const int32_t *dep_start;
    const int32_t *deps;
    const int16_t *ac;
    const uint8_t *idx;
    const void *pal;
    void *coef;
    int32_t n;
} MiIntraFrame;
int mi_intra_recon(MiCtx *ctx, const MiIntraFrame *frames, int nframes, unsigned flags, void *stream);

/* Synchronise `stream` and report device-side failures of the context's launches since the
 * last call: 0; -EINVAL when a kernel skipped device descriptors the reference could never
 * issue (mi_itx_frame / mi_intra_recon: a transform type the size's table slot lacks, a size
 * outside its group, a rectangle outside its plane); -ETIMEDOUT when a dependency wait gave up;
 * -EIO when a block was never taken. */
int mi_ctx_device_status(MiCtx *ctx, void *stream);

/* Deblock a whole frame in place: all column edges (every plane), then all row edges.
 * Equivalent to the reference's per-sbrow cols/rows interleaving;
 * replaces rav1d_loopfilter_sbrow_cols/_rows (src/lf_apply.rs:597-834). */
int mi_deblock_frame(MiCtx *ctx, const MiPicture *pic, const MiLoopFilter *lf, void *stream);

/* Deblocking out of place: reads the reconstruction `src` (never written), writes the
 * deblocked picture to `dst` over the 128-aligned plane area (dav1d's default picture
 * geometry, src/picture.rs:98-115). One launch of 64x64 plane tiles, each filtering every
 * column edge and then every row edge that reaches it from an LDS copy with a 16/12-px halo;
 * bit-identical to mi_deblock_frame. Planes and strides must be 16-byte aligned. With
 * src == dst it runs mi_deblock_frame (in place). */
int mi_deblock_frame_to(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, const MiLoopFilter *lf,
                        void *stream);
/* mi_deblock_frame_to that adds, while staging, the DC runs the context's last
 * mi_itx_frame_runs(MI_ITX_DC_DEFER) recorded (src never written; with lf->filter_y == 0 the
 * output is src plus the DC). Without a pending deferral it is mi_deblock_frame_to. The picture
 * geometry must be the deferring call's and src != dst (-EINVAL otherwise). */
int mi_deblock_frame_dc(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, const MiLoopFilter *lf,
                        void *stream);

/* Motion compensation for a whole frame: writes the inter prediction of every unit into
 * `cur` (itx then adds the residual). `refs` (host array of nrefs pictures, device planes,
 * grain-free, same size as cur) are read with edge replication (emu_edge, mc_tmpl.c:798-845).
 * `blocks` (device) are bucketed by plane group g (0 luma, 1 chroma) and shape class
 * c = log2(w) * 8 + log2(h): the units of (g, c) are
 * blocks[class_start[g * MI_MC_NCLASS + c] .. class_start[g * MI_MC_NCLASS + c + 1]) (host
 * array, non-decreasing; all luma before all chroma). Luma runs first: chroma units of SEG
 * blocks read the mask their luma unit wrote. `masks` (device) holds MASK inputs and SEG
 * outputs. Scaled references, OBMC, warped and inter-intra units are not batched here yet. */
#define MI_MC_NCLASS 64
int mi_mc_frame(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
                const MiMcBlock *blocks, const uint32_t class_start[2 * MI_MC_NCLASS + 1],
                uint8_t *masks, int16_t *tmp, void *stream);
/* mi_mc_frame with flags. MI_MC_ONE_GRID: both plane groups run in one grid, so the small
 * chroma units fill the luma tail (4K10 synthetic frame: 62 us against 75 for the two
 * launches). The caller promises that no chroma unit of the call reads a mask written by a SEG
 * unit of the same call. For a frame without chroma MASK units this is a pure gain; when they
 * exist, moving them into a second call cost more than it saved (82-85 us), so the caller
 * keeps mi_mc_frame there. Unknown flags: -EINVAL. */
#define MI_MC_ONE_GRID 1u
int mi_mc_frame_ex(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
                   const MiMcBlock *blocks, const uint32_t class_start[2 * MI_MC_NCLASS + 1],
                   uint8_t *masks, int16_t *tmp, unsigned flags, void *stream);
/* mi_mc_frame as one grid whatever the units: a chroma MASK unit whose mask a SEG unit of the
 * same call writes carries MI_MC_AFTER_SEG in `param` (bit 6) and waits inside the launch for
 * that SEG unit's tiles (they publish the mask with agent-scope word stores and a flag per
 * tile; the luma waves precede the chroma ones in the grid, so a waiting wave only waits for
 * waves already started). SEG and MASK mask offsets must be multiples of 16 and mask_bytes
 * the size of the mask buffer. A wait that does not end is reported as -ETIMEDOUT, a flagged
 * unit whose mask offset lies past mask_bytes as -EINVAL (the kernel skips its flag access),
 * by mi_mc_sync_status or mi_ctx_device_status. While `stream` is being captured into a graph
 * the call runs as mi_mc_frame's two launches: an epoch fixed at capture would let a replay
 * see the flags of the previous replay. */
#define MI_MC_AFTER_SEG 0x40u
int mi_mc_frame_sync(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
                     const MiMcBlock *blocks, const uint32_t class_start[2 * MI_MC_NCLASS + 1],
                     uint8_t *masks, size_t mask_bytes, int16_t *tmp, void *stream);
/* 0, -ETIMEDOUT when a hand-off wait of an earlier mi_mc_frame_sync on the context timed out,
 * -EINVAL when a flagged unit's mask offset lay past mask_bytes (synchronises `stream`; clears
 * the status; mi_ctx_device_status reports the same codes) */
int mi_mc_sync_status(MiCtx *ctx, void *stream);
/* OBMC: the caller runs mi_mc_frame a second time with the above-neighbour laps
 * (MI_MC_OBMC_H units) and a third time with the left-neighbour laps (MI_MC_OBMC_V), as
 * obmc() blends above before left. `tmp` (device, int16) receives MI_MC_PREP units; may be
 * NULL without them. */

/* Scaled references (recon.rs:2124-2202): units whose reference differs in size from cur, put
 * (single) or MI_MC_PREP into tmp. Positions and steps follow f->svc (scale_fac,
 * decode.rs:4776) from the picture sizes. `blocks` is a device array of n units, any order. */
int mi_mc_scaled(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
                 const MiMcBlock *blocks, int n, int16_t *tmp, void *stream);

/* Warped motion (warp_affine, recon.rs:2311-2400): n 8x8 blocks (device array), edge
 * replication as emu_edge. */
int mi_mc_warp(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
               const MiWarpBlock *blocks, int n, int16_t *tmp, void *stream);

/* Compound combine of two tmp intermediates into cur (device arrays; SEG writes masks). */
int mi_mc_combine(MiCtx *ctx, const MiPicture *cur, const MiMcCombine *units, int n,
                  const int16_t *tmp, uint8_t *masks, void *stream);

/* Super-resolution upscale of a whole frame (rav1d_filter_sbrow_resize, recon.rs:4215-4285,
 * over all rows; mc.resize): src is the coded-width picture, dst the upscaled one (same height,
 * layout, bpc). Step and start per plane follow scale_fac / get_upscale_x0 (decode.rs:4644,
 * 4776, 4872-4878). */
int mi_superres_frame(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, void *stream);

/* CDEF for a whole frame, out of place: reads the deblocked picture `src` (never written)
 * and writes `dst` (blocks the reference skips are copied). Replaces rav1d_cdef_brow
 * (src/cdef_apply.rs:159-507). `src` and `dst` must have identical geometry. */
int mi_cdef_frame(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, const MiCdef *cdef,
                  void *stream);

/* Loop restoration for a whole frame: reads the CDEF output `cdef` inside each 64-row stripe
 * and the deblocked picture `deblocked` for the rows across stripe edges (the rows the
 * reference keeps in f->lf.lr_lpf_line, src/lf_apply.rs:24-141), writes `dst`. Planes not
 * in restore_planes, and units of type NONE, are copied. Replaces rav1d_lr_sbrow
 * (src/lr_apply.rs:261-329). All three pictures share one geometry. */
int mi_lr_frame(MiCtx *ctx, const MiPicture *cdef, const MiPicture *deblocked,
                const MiPicture *dst, const MiLr *lr, void *stream);

/* Film grain (output only; reference frames stay grain-free): out = in + grain. Replaces
 * rav1d_apply_grain (src/fg_apply.rs:272-284 = prep_grain + apply_grain_row per 32 rows).
 * mtrx_identity: seq_hdr.mtrx == DAV1D_MC_IDENTITY (restricted-range chroma clip).
 * The split form lets a caller run the pixel-independent prep (grain templates, scaling
 * LUTs, block offsets) on a side stream at frame start; apply uses the context's last prep. */
int mi_film_grain_frame(MiCtx *ctx, const MiPicture *in, const MiPicture *out,
                        const MiFilmGrainData *data, int mtrx_identity, void *stream);
int mi_film_grain_prep(MiCtx *ctx, const MiPicture *in, const MiFilmGrainData *data, void *stream);
int mi_film_grain_apply(MiCtx *ctx, const MiPicture *in, const MiPicture *out,
                        const MiFilmGrainData *data, int mtrx_identity, void *stream);

/* ------------------------------------------------------------------------------------ */
/* Table-compatible per-call entry points                                                */
/* ------------------------------------------------------------------------------------ */

/* itxfm_add[tx][txtp] (src/itx.rs:190-196; C src/itx.h:37-44). Replaces
 * inv_txfm_add_rust / dav1d_inv_txfm_add_<type>_<w>x<h>_<bpc>bpc_<isa>. Returns 0 or -errno
 * (the reference's fn returns void; a non-zero return here means nothing was written). */
int mi_dsp_itxfm_add(int tx, int txtp, void *dst, ptrdiff_t stride, void *coeff, int eob,
                     int bitdepth_max);

/* intra_pred[mode] (src/ipred.rs:48-58; C src/ipred.h:47-53) on one block: topleft points
 * into the caller's edge buffer (samples topleft[-(w+h)] .. topleft[w+h] are read). Host or
 * device pointers; synchronous. Replaces ipred_*_rust / dav1d_ipred_*_<bpc>bpc_<isa>. */
int mi_dsp_intra_pred(int mode, void *dst, ptrdiff_t stride, const void *topleft, int w, int h,
                      int angle, int max_width, int max_height, int bitdepth_max);

/* The remaining per-call entries of the intra, loop-filter and CDEF tables. Same contract as
 * above: host or device pointers, synchronous, 0 (or the documented value) / -errno. The
 * trailing bitdepth_max selects the pixel size where the reference's signature has none. */

/* cfl_pred[mode] (src/ipred.rs:108-117, C ipred_tmpl.c:71-84): mode 0 DC, 3 LEFT_DC, 4 TOP_DC,
 * 5 DC_128; ac: w * h int16 (cfl_ac's output). */
int mi_dsp_cfl_pred(int mode, void *dst, ptrdiff_t stride, const void *topleft, int w, int h, const int16_t *ac,
                    int alpha, int bitdepth_max);
/* pal_pred (src/ipred.rs:138-145, 1433-1452): idx one byte per pixel, w * h. */
int mi_dsp_pal_pred(void *dst, ptrdiff_t stride, const void *pal, const uint8_t *idx, int w, int h, int bitdepth_max);
/* cfl_ac[layout - 1] (src/ipred.rs:82-90, 1326-1432): layout 1 I420, 2 I422, 3 I444. */
int mi_dsp_cfl_ac(int layout, int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad, int cw, int ch,
                  int bitdepth_max);
/* loop_filter_sb[cls][dir] (src/loopfilter.rs:20-34, 745-985): cls 0 luma / 1 chroma, dir 0
 * column edges (h_sb*) / 1 row edges (v_sb*); vmask[3] (luma) or [2] (chroma) bit k = 4-px
 * unit k of the run; lvl points at the run's first [u8;4] level entry (already offset to
 * the slot used), b4_stride entries per row; lut = Av1FilterLUT (e[64], i[64], ...). */
int mi_dsp_loop_filter_sb(int cls, int dir, void *dst, ptrdiff_t stride, const uint32_t *vmask,
                          const uint8_t (*lvl)[4], ptrdiff_t b4_stride, const void *lut, int wh, int bitdepth_max);
/* cdef.fb[fb] (src/cdef.rs:35-56, 567-820): fb 0 8x8, 1 4x8, 2 4x4; left [h][2] pixels; top /
 * bottom point at the block's column 0 of the two rows above / below (stride as dst); edges =
 * CdefEdgeFlags (HAVE_LEFT 1, HAVE_RIGHT 2, HAVE_TOP 4, HAVE_BOTTOM 8). In place on dst. */
int mi_dsp_cdef_filter(int fb, void *dst, ptrdiff_t stride, const void *left, const void *top, const void *bottom,
                       int pri, int sec, int dir, int damping, int edges, int bitdepth_max);
/* cdef.dir (src/cdef.rs:921-1031): returns the direction 0..7 (or -errno), *var the variance. */
int mi_dsp_cdef_dir(const void *img, ptrdiff_t stride, unsigned *var, int bitdepth_max);

/* Rav1dMCDSPContext (src/mc.rs:1174-1338; C src/mc.h:38-108). mc[filter2d] / mct[filter2d]:
 * filter2d = Filter2d 0..8 (8-tap regular/smooth/sharp pairs) or 9 (bilinear); mx / my in
 * 1/16 pel; src at the block origin with the filter reach (3 before, 4 after) readable;
 * prep writes w * h int16 intermediates (PREP_BIAS applied). */
int mi_dsp_mc_put(int filter2d, void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int w, int h,
                  int mx, int my, int bitdepth_max);
int mi_dsp_mc_prep(int filter2d, int16_t *tmp, const void *src, ptrdiff_t src_stride, int w, int h, int mx, int my,
                   int bitdepth_max);
/* avg / w_avg / mask / w_mask[layout - 1] (layout 1 I420, 2 I422, 3 I444; mask written at the
 * chroma resolution) / blend / blend_v / blend_h (OBMC, obmc_masks) / emu_edge. */
int mi_dsp_mc_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                  int bitdepth_max);
int mi_dsp_mc_w_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h, int weight,
                    int bitdepth_max);
int mi_dsp_mc_mask(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                   const uint8_t *mask, int bitdepth_max);
int mi_dsp_mc_w_mask(int layout, void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w,
                     int h, uint8_t *mask, int sign, int bitdepth_max);
int mi_dsp_mc_blend(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h, const uint8_t *mask,
                    int bitdepth_max);
int mi_dsp_mc_blend_v(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h, int bitdepth_max);
int mi_dsp_mc_blend_h(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h, int bitdepth_max);
int mi_dsp_mc_emu_edge(int bw, int bh, int iw, int ih, int x, int y, void *dst, ptrdiff_t dst_stride, const void *ref,
                       ptrdiff_t ref_stride, int bitdepth_max);
/* warp8x8 (prep 0: pixels) / warp8x8t (prep 1: int16 intermediate, dst_stride in elements as
 * the reference's tmp_stride) (src/mc.rs:885-1030); src at the 8x8 block origin, rows and
 * columns -3 .. 11 readable; abcd = the block's warp steps. */
int mi_dsp_mc_warp8x8(int prep, void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                      const int16_t *abcd, int mx, int my, int bitdepth_max);
/* mc_scaled[filter2d] (prep 0: pixels into dst) / mct_scaled[filter2d] (prep 1: w * h int16
 * into dst, dst_stride ignored) (src/mc.rs:212, 351, 496, 608): mx, my in [0, 1024) (1/1024
 * pel), dx / dy the steps. */
int mi_dsp_mc_scaled(int prep, int filter2d, void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                     int w, int h, int mx, int my, int dx, int dy, int bitdepth_max);
/* resize (src/mc.rs:1114-1172): super-resolution upscaling of h rows. */
int mi_dsp_mc_resize(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int dst_w, int h,
                     int src_w, int dx, int mx0, int bitdepth_max);

/* lr.wiener[0|1] (src/looprestoration.rs:91-107, 299-370): one restoration unit of w <= 384
 * by h <= 64 filtered in place. left = LeftPixelRow [h][4] (read when edges & LR_HAVE_LEFT);
 * lpf = the loop-filtered rows, 0 and 1 above the unit and 6 and 7 below it, at `stride`
 * (read when LR_HAVE_TOP / LR_HAVE_BOTTOM, columns -3 .. w + 2 as the edges allow);
 * params = LooprestorationParams.filter [2][8] int16 as the reference builds it
 * (src/lr_apply.rs: 8-bit centre tap without its +128). */
int mi_dsp_lr_wiener(void *p, ptrdiff_t stride, const void *left, const void *lpf, int w, int h, const void *params,
                     int edges, int bitdepth_max);
/* lr.sgr[kind] (src/looprestoration.rs:710-912): kind 0 = 5x5 (s0, w0), 1 = 3x3 (s1, w1),
 * 2 = both; params = LooprestorationParams_sgr {u32 s0, s1; i16 w0, w1}; the rest as wiener. */
int mi_dsp_lr_sgr(int kind, void *p, ptrdiff_t stride, const void *left, const void *lpf, int w, int h,
                  const void *params, int edges, int bitdepth_max);

/* Film-grain table (src/filmgrain.rs:41-198). data = Dav1dFilmGrainData (MiFilmGrainData is
 * layout-identical); buf / buf_y / grain_lut = GrainLut<Entry>: rows of 82 entries, int8 at
 * 8 bits and int16 above; layout 1 = I420, 2 = I422, 3 = I444 (the generate_grain_uv /
 * fguv_32x32xn enum_map slot).
 * generate_grain_y (:298-343): the 73 x 82 luma template. */
int mi_dsp_fg_generate_grain_y(void *buf, const MiFilmGrainData *data, int bitdepth_max);
/* generate_grain_uv[layout] (:345-474): the chroma template of plane 1 + uv (its 38/73 x 44/82
 * corner), auto-regressed over the luma template buf_y. */
int mi_dsp_fg_generate_grain_uv(int layout, void *buf, const void *buf_y, const MiFilmGrainData *data, int uv,
                                int bitdepth_max);
/* fgy_32x32xn (:549-676): grain onto one strip of bh <= 32 rows and pw <= 8192 columns,
 * src_row -> dst_row (same stride); scaling = the plane's LUT (1 << bitdepth entries). */
int mi_dsp_fgy_32x32xn(void *dst_row, const void *src_row, ptrdiff_t stride, const MiFilmGrainData *data, size_t pw,
                       const uint8_t *scaling, const void *grain_lut, int bh, int row_num, int bitdepth_max);
/* fguv_32x32xn[layout] (:678-830): chroma plane 1 + uv_pl, bh in chroma rows; luma_row holds
 * the co-located luma (pw << ss_x columns, as the reference reads them). */
int mi_dsp_fguv_32x32xn(int layout, void *dst_row, const void *src_row, ptrdiff_t stride,
                        const MiFilmGrainData *data, size_t pw, const uint8_t *scaling, const void *grain_lut, int bh,
                        int row_num, const void *luma_row, ptrdiff_t luma_stride, int uv_pl, int is_id,
                        int bitdepth_max);

#ifdef __cplusplus
}
#endif
#endif /* MI_AV1DSP_H */
