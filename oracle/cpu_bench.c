/*
 * cpu_bench.c — the CPU baseline timer: the oracle's whole-frame pipeline (MC -> itx ->
 * deblock -> CDEF -> LR, the order rav1d runs for an inter frame: recon_b_inter then
 * filter_sbrow, recon.rs:3162-4211) driven from C, no Python or numpy inside the timed loop.
 * TEST INFRASTRUCTURE ONLY (see oracle.h): bench.py's cpu_baseline leg is its only caller.
 *
 * Threads run independent frames (one private set of pictures, coefficient arena and mask
 * scratch per thread, the same descriptors), which is how a host decodes independent streams
 * and the CPU analogue of the GPU replicas. Each thread does `frames` frames; the result is
 * the wall time of the slowest thread.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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

/* One frame's inputs (all host arrays; planes 128-aligned with strides[]). */
typedef struct OracleBenchJob {
    int w, h, bpc, layout;
    ptrdiff_t strides[3];
    size_t plane_bytes[3];
    const void *refs[2][3];            /* reference pictures (same geometry) */
    int nrefs;
    const void *units;                 /* MiMcBlock[n_units] */
    int n_units;
    const uint8_t *masks;              /* MC mask buffer */
    size_t masks_bytes;
    const void *tx;                    /* MiTxBlock[n_tx] */
    int n_tx;
    const void *coef;
    size_t coef_bytes;
    const uint8_t *lf_level;
    ptrdiff_t b4_stride;
    const void *lf_masks;              /* Av1Filter[sb128h][sb128w] */
    int sb128w;
    const uint8_t *lim_e, *lim_i;
    int filter_y, filter_uv;
    int cdef_damping;
    const uint8_t *cdef_y, *cdef_uv;
    int restore_planes;
    int unit_size_log2[2];
    const void *lr_mask;
    int lr_sb128w;
} OracleBenchJob;

typedef struct {
    const OracleBenchJob *j;
    pthread_barrier_t *start;
    int frames;
    double seconds;
} Worker;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *run(void *arg) {
    Worker *wk = arg;
    const OracleBenchJob *j = wk->j;
    const int np = j->layout ? 3 : 1;
    void *pic[4][3];
    for (int k = 0; k < 4; k++)
        for (int p = 0; p < 3; p++) pic[k][p] = p < np ? calloc(1, j->plane_bytes[p]) : NULL;
    for (int k = 0; k < 4; k++)
        for (int p = np; p < 3; p++) pic[k][p] = pic[k][0];
    void *coef = malloc(j->coef_bytes + 64);
    uint8_t *masks = malloc(j->masks_bytes + 64);
    int16_t *tmp = malloc(64);
    void *refs[6];
    ptrdiff_t ref_strides[4];
    int ref_wh[4];
    for (int r = 0; r < j->nrefs; r++) {
        for (int p = 0; p < 3; p++) refs[3 * r + p] = (void *)j->refs[r][p < np ? p : 0];
        ref_strides[2 * r] = j->strides[0];
        ref_strides[2 * r + 1] = j->strides[1];
        ref_wh[2 * r] = j->w;
        ref_wh[2 * r + 1] = j->h;
    }
    const ptrdiff_t cs[2] = { j->strides[0], j->strides[1] };
    /* buffers are touched before the clock starts: page faults take the process-wide mm lock */
    memcpy(coef, j->coef, j->coef_bytes);
    memcpy(masks, j->masks, j->masks_bytes);
    for (int k = 0; k < 4; k++)
        for (int p = 0; p < np; p++) memset(pic[k][p], 0, j->plane_bytes[p]);
    pthread_barrier_wait(wk->start);
    const double t0 = now();
    for (int f = 0; f < wk->frames; f++) {
        /* pass-2 inputs of this frame: the coefficient arena (itx consumes it) and masks */
        memcpy(coef, j->coef, j->coef_bytes);
        memcpy(masks, j->masks, j->masks_bytes);
        if (j->n_units)
            oracle_mc_frame(pic[0], cs, j->layout, j->bpc, refs, ref_strides, ref_wh, j->units, j->n_units,
                            masks, tmp);
        oracle_itx_frame(pic[0], j->strides, j->tx, j->n_tx, coef, (1 << j->bpc) - 1);
        oracle_deblock_frame(pic[0], j->strides, j->w, j->h, j->layout, j->bpc, j->lf_level, j->b4_stride,
                             j->lf_masks, j->sb128w, 1, j->lim_e, j->lim_i, j->filter_y, j->filter_uv);
        oracle_cdef_frame(pic[1], pic[0], j->strides, j->w, j->h, j->layout, j->bpc, j->lf_masks, j->sb128w,
                          j->cdef_damping, j->cdef_y, j->cdef_uv);
        oracle_lr_frame(pic[2], pic[1], pic[0], j->strides, j->w, j->h, j->layout, j->bpc, 1, j->restore_planes,
                        j->unit_size_log2, j->lr_mask, j->lr_sb128w);
    }
    wk->seconds = now() - t0;
    for (int k = 0; k < 4; k++)
        for (int p = 0; p < np; p++) free(pic[k][p]);
    free(coef);
    free(masks);
    free(tmp);
    return NULL;
}

/* Wall seconds for `threads` threads each decoding `frames` frames of `job` (the slowest
 * thread's time), or a negative value on failure. */
double oracle_bench_frames(const OracleBenchJob *job, int threads, int frames) {
    if (!job || threads < 1 || threads > 1024 || frames < 1) return -1;
    Worker *wk = calloc(threads, sizeof(Worker));
    pthread_t *th = calloc(threads, sizeof(pthread_t));
    pthread_barrier_t start;
    pthread_barrier_init(&start, NULL, threads);
    for (int i = 0; i < threads; i++) {
        wk[i].j = job;
        wk[i].start = &start;
        wk[i].frames = frames;
        if (pthread_create(&th[i], NULL, run, &wk[i])) {
            /* the barrier counts `threads`: never leave it short (abort the measurement) */
            abort();
        }
    }
    double t = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        if (wk[i].seconds > t) t = wk[i].seconds;
    }
    pthread_barrier_destroy(&start);
    free(wk);
    free(th);
    return t;
}
