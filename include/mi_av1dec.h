/*
 * mi_av1dec.h — C-ABI of the host front-end: AV1 OBUs in, pass-2 work lists out.
 *
 * This is the CPU side north_star keeps on the host (rav1d's OBU / msac / mode and
 * coefficient decoding: src/obu.rs:2662, src/msac.rs, src/decode.rs:1131-4067,
 * src/recon.rs:478-2023, src/lf_mask.rs:380-723), restated in C++ (rav1d_amd/host/) and built
 * as rav1d_amd/libmi_av1dec.so. Instead of reconstructing pixels it emits, per frame, the
 * descriptor lists of mi_av1dsp.h (MiIntraBlock / MiTxBlock, coefficient arena, Av1Filter
 * masks and levels, Av1Restoration units, film-grain data) that the gfx950 kernels execute.
 *
 * Threading: one MiDec per stream; calls on one MiDec are serialised by the caller.
 * Errors: 0 / positive counts, or a negative errno (-EINVAL bitstream error, -ENOMEM,
 * -ENOTSUP for a coding tool this front-end does not decode yet); mi_dec_error() explains.
 */
#ifndef MI_AV1DEC_H
#define MI_AV1DEC_H

#include <stddef.h>
#include <stdint.h>

#include "mi_av1dsp.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MI_AV1DEC_ABI_VERSION 2

/* The pass-2 work of one decoded frame. All pointers stay valid until the next
 * mi_dec_next() / mi_dec_destroy() on the same decoder. */
typedef struct MiDecFrame {
    int32_t w, h;                 /* coded luma size (frame_hdr.width[0], height) */
    int32_t up_w;                 /* luma width after super-resolution (width[1]); == w without */
    int32_t render_w, render_h;
    int32_t bpc, layout, sb128;
    /* intra path, decode order: blocks[i] predicted then tx[i] added (eob < 0: no residual);
     * deps[dep_start[i] .. dep_start[i + 1]) = earlier blocks owning pixels blocks[i] reads */
    const MiIntraBlock *intra;
    const MiTxBlock *intra_tx;
    int32_t n_intra;
    const int32_t *dep_start;     /* n_intra + 1 entries */
    const int32_t *deps;
    int32_t n_deps;
    /* residuals of inter blocks (added after motion compensation, before the intra path) */
    const MiTxBlock *inter_tx;
    int32_t n_inter_tx;
    /* coefficient arena: int16_t (8 bpc) or int32_t (10/12 bpc), ncoef entries. Entries
     * 0..15 are a reserved zero block: a transform block without residual (skip, or an
     * all-zero block) has eob < 0 and coef_off 0, so any consumer adds nothing. */
    const void *coef;
    size_t ncoef;
    const uint8_t *idx;           /* palette indices (MI_IPRED_PAL aux_off) */
    size_t nidx;
    const void *pal;              /* palette colours, pixels of bpc (MI_IPRED_PAL pal_off) */
    size_t npal;
    /* deblocking (MiLoopFilter inputs) */
    int32_t filter_y, filter_uv;
    const uint8_t *lf_level;      /* [rows][b4_stride][4] */
    int32_t b4_stride;
    const MiAv1Filter *lf_masks;  /* [sb128h][sb128w], tile fixups applied */
    int32_t sb128w, sb128h;
    uint8_t lim_e[64], lim_i[64];
    /* CDEF (seq_hdr.cdef) */
    int32_t cdef_on, cdef_damping;
    uint8_t cdef_y[8], cdef_uv[8];
    /* loop restoration */
    const MiAv1Restoration *lr_mask;   /* [sb128h][lr_sb128w] */
    int32_t lr_sb128w, restore_planes, lr_unit_size[2];
    /* inter prediction (recon_b_inter, recon.rs:3162-4045), run before the residuals: every count
     * is 0 in an intra frame. MiMcBlock / MiWarpBlock refs index the frame's seven references
     * (LAST .. ALTREF = MiDecEvent.ref_pic[0..6]). */
    const MiMcBlock *mc;              /* put / compound / MI_MC_PREP units, any order */
    int32_t n_mc;
    const MiMcBlock *obmc_h;          /* OBMC laps of above neighbours (blended first) */
    int32_t n_obmc_h;
    const MiMcBlock *obmc_v;          /* OBMC laps of left neighbours */
    int32_t n_obmc_v;
    const MiWarpBlock *warp;          /* warp8x8 / warp8x8t blocks */
    int32_t n_warp;
    const MiMcBlock *scaled;          /* units whose reference differs in size (put or MI_MC_PREP) */
    int32_t n_scaled;
    const MiMcCombine *combine_y;     /* compounds with a warped / scaled side: luma ... */
    int32_t n_combine_y;
    const MiMcCombine *combine_uv;    /* ... then chroma (its MASK units read what luma SEG wrote) */
    int32_t n_combine_uv;
    const uint8_t *masks;             /* wedge masks (MASK inputs) and room for SEG outputs */
    size_t nmasks;
    size_t ntmp;                      /* int16 elements of the arena the prep sides write */
    /* Optional: the intra queue mi_frame_run would plan (intra_plan.h), made off its critical
     * path (the front-end's frame jobs fill it): the n_intra blocks / transforms in queue order
     * (vertical strips, one per XCD, each by dependency level), dependencies as queue positions
     * (CSR, q_dep_start has n_intra + 1 entries), q_nstrips > 1: strip k = queue entries
     * [q_strip_start[k], q_strip_start[k + 1]); q_granules: edges handed over as granules (an
     * intra-only frame without inter-intra items). NULL q_intra: mi_frame_run plans. */
    const MiIntraBlock *q_intra;
    const MiTxBlock *q_intra_tx;
    const int32_t *q_dep_start;
    const int32_t *q_deps;
    int32_t q_n_deps;
    const int32_t *q_strip_start;
    int32_t q_nstrips;
    int32_t q_granules;
} MiDecFrame;

/* One decoder event: a frame to reconstruct into picture `pic_id` (frame != NULL; its inter
 * prediction reads pictures ref_pic[]), and/or a picture to output (show_pic >= 0, with film
 * grain when fg_present). Pictures listed in release[] are no longer referenced. */
typedef struct MiDecEvent {
    const MiDecFrame *frame;
    int32_t pic_id;
    int32_t ref_pic[7];
    int32_t show_pic;
    int32_t fg_present;
    MiFilmGrainData fg;
    const int32_t *release;
    int32_t n_release;
    int32_t mtrx_identity;   /* seq_hdr.mtrx == DAV1D_MC_IDENTITY (the grain's chroma clip, fg_apply.rs) */
} MiDecEvent;

/* ---- device execution of a decoded frame (these two live in librav1d_amd.so) ----
 *
 * The pictures one frame's pass 2 writes (device planes, all of one geometry):
 * recon = prediction + residual, deblocked (recon -> deblocked), cdef (deblocked -> cdef),
 * restored ((cdef, deblocked) -> restored). Stages the frame header switches off are skipped,
 * not copied: *final receives the index (0 recon .. 3 restored) of the picture holding the
 * frame's reference-quality output (the picture rav1d leaves in f.sr_cur after
 * filter_sbrow: recon.rs:4019-4211). */
typedef struct MiFramePictures {
    MiPicture recon, deblocked, cdef, restored;
    MiPicture refs[7];    /* the reference pictures of an inter frame (MiDecEvent.ref_pic order,
                             each the reference's final picture); unused for intra frames */
} MiFramePictures;

/* Enqueue one frame's reconstruction and in-loop filters on `stream` (recon_b_intra over the
 * intra work list in one persistent launch, blocks reordered by dependency level; then
 * mi_deblock_frame_to / mi_cdef_frame / mi_lr_frame). The host arrays of `f` are copied during
 * the call (pinned staging + async upload), so `f` may be released on return. Calls on one
 * context must use one stream. 0 or -errno (-EINVAL malformed work list, -ENOMEM, -EIO). */
int mi_frame_run(MiCtx *ctx, const MiDecFrame *f, const MiFramePictures *pics, int *final, void *stream);

/* The host-side checks mi_frame_run applies before enqueuing anything, without a device: 0, or
 * -EINVAL with *why (if non-NULL) naming the failed check. */
int mi_frame_validate(const MiDecFrame *f, const MiFramePictures *pics, const char **why);
/* Diagnostic: mean host time (ms) of mi_frame_run's planning pass over `f` (intra queue order,
 * dependency lists, inter unit buckets, residual bands), reps times; no device work. -1.0 when
 * the work list fails mi_frame_validate's checks (the pictures are not checked). */
double mi_frame_plan_ms(const MiDecFrame *f, int reps);

/* Wait for the work enqueued on `stream` and report device-side failures of the frame(s):
 * 0; -EINVAL when a kernel rejected (skipped) a descriptor no valid stream produces; -EIO
 * when a block's dependency wait gave up or a block was never reconstructed (the pictures
 * are then not valid). rav1d reports such a frame as a decode error (Dav1dResult,
 * src/error.rs). */
int mi_frame_end(MiCtx *ctx, void *stream);

/* Per-stage timing of mi_frame_run on one context (the §8(d) breakdown of a stream decode).
 * With timing on, every mi_frame_run records five HIP events on its stream; mi_ctx_timing
 * waits for them, sums the stages over the frames run since the last read, and resets.
 * Timing adds no synchronisation to mi_frame_run itself. */
typedef struct MiFrameTiming {
    int32_t frames;        /* frames run since the last read */
    int32_t reserved;
    double host_ms;        /* host time inside mi_frame_run: checks, dependency-level sort,
                              bucketing, staging copy (and any wait for the staging buffer) */
    double upload_ms;      /* device time of the descriptor + coefficient upload (H2D) */
    double inter_ms;       /* MC, warp, scaled, combine, OBMC laps, inter residuals */
    double intra_ms;       /* the persistent intra reconstruction launch */
    double filter_ms;      /* deblock, CDEF, super-resolution, loop restoration */
    int64_t upload_bytes;  /* bytes uploaded */
    double stage_ms;       /* of host_ms: the staging copy into pinned memory, with any wait for
                              the previous frame's upload to leave the staging buffer */
    double strips_ms;      /* of host_ms: the dependency levels and the XCD strip split */
} MiFrameTiming;
int mi_ctx_set_timing(MiCtx *ctx, int on);
int mi_ctx_timing(MiCtx *ctx, MiFrameTiming *out);

typedef struct MiDec MiDec;

int  mi_dec_create(MiDec **out);
void mi_dec_destroy(MiDec *d);
/* Frame threads (rav1d's Dav1dSettings.n_frame_threads, src/lib.rs): with n > 1, intra frames
 * are entropy-decoded on up to n worker threads while mi_dec_send parses on; mi_dec_next
 * still returns events in decode order and waits for the oldest frame's worker, so a caller
 * that wants the overlap sends a few temporal units ahead before draining. A worker's failure
 * is returned by the mi_dec_next of its frame. Default 1 (synchronous). 0 or -EINVAL. */
int  mi_dec_set_threads(MiDec *d, int n);
/* Dav1dSettings.inloop_filters (include/dav1d/dav1d.rs:17-35, src/lib.rs:136,218; the CLI's
 * --inloopfilters): the in-loop filters the frames this decoder emits ask mi_frame_run to
 * apply. A filter left out is skipped as rav1d's filter_sbrow_* skip it (recon.rs:4054, 4162,
 * 4178, 4290): the frame's filter_y / cdef_on / restore_planes are cleared, super-resolution
 * still runs, and the unfiltered picture is the reference later frames predict from. The bit
 * values are rav1d's. Default MI_INLOOPFILTER_ALL. 0 or -EINVAL. */
#define MI_INLOOPFILTER_NONE 0
#define MI_INLOOPFILTER_DEBLOCK (1 << 1)
#define MI_INLOOPFILTER_CDEF (1 << 2)
#define MI_INLOOPFILTER_RESTORATION (1 << 3)
#define MI_INLOOPFILTER_ALL (MI_INLOOPFILTER_DEBLOCK | MI_INLOOPFILTER_CDEF | MI_INLOOPFILTER_RESTORATION)
int  mi_dec_set_inloop_filters(MiDec *d, int flags);
/* Feed one temporal unit (any whole number of OBUs). */
int  mi_dec_send(MiDec *d, const uint8_t *data, size_t size);
/* Next event: 1 and *ev filled, 0 when none is pending, or -errno. */
int  mi_dec_next(MiDec *d, MiDecEvent *ev);
const char *mi_dec_error(const MiDec *d);

#ifdef __cplusplus
}
#endif
#endif /* MI_AV1DEC_H */
