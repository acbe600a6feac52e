// ctx.h — MiCtx, the per-stream device context behind include/mi_av1dsp.h (one per decoder
// frame context; calls on one context are serialised by the caller and use one stream).
#pragma once
#include "common.h"

#include <vector>

struct MiCtx {
    int device = 0;
    int last_error = 0;
    // film-grain scratch (grain templates, scaling LUTs, block offsets)
    int16_t *fg_lut = nullptr;
    uint8_t *fg_scaling = nullptr;
    uint8_t *fg_offsets = nullptr;
    size_t fg_offsets_bytes = 0;
    // persistent intra reconstruction: per-block done epochs, queue heads, error word
    uint32_t *ir_done = nullptr;
    size_t ir_done_n = 0;
    int *ir_words = nullptr;      // [0..63] queue heads, [64] error, [72..79] XCD worker ranks
    uint32_t ir_epoch = 0;        // never reset: done words and edge granules hold old epochs
    unsigned long long *ir_gran = nullptr;   // edge granules (ipred.hip GranCtx), zeroed when allocated
    size_t ir_gran_n = 0;
    unsigned long long *ir_tl = nullptr;     // MI_IR_TIMELINE stamps (diagnostics)
    size_t ir_tl_n = 0;
    // one-grid MC with in-launch hand-off (mi_mc_frame_sync): per-tile flags of SEG masks,
    // epoch (never reset: the flags hold old epochs), error word
    uint32_t *mc_flags = nullptr;
    size_t mc_flags_n = 0;
    uint32_t mc_epoch = 0;
    int *mc_err = nullptr;
    // deferred DC runs (mi_itx_frame_runs MI_ITX_DC_DEFER -> mi_deblock_frame_dc): the map
    // (zeroed when allocated and when its 16-bit tag wraps), its geometry and the pending tag
    uint32_t *dc_map = nullptr;
    size_t dc_map_n = 0;
    int dc_w = 0, dc_h = 0, dc_layout = -1;
    uint32_t dc_tag = 0, dc_pending = 0;
    // frame executor (frame_exec.cpp): device copy of one frame's descriptors, staged through
    // pinned host memory; `fx_ev` marks when the staging buffer may be rewritten
    uint8_t *fx_dev = nullptr, *fx_host = nullptr;
    size_t fx_dev_bytes = 0, fx_host_bytes = 0;
    hipEvent_t fx_ev = nullptr;
    bool fx_ev_pending = false;
    // per-stage timing of mi_frame_run (mi_ctx_set_timing): 5 events per frame (before the
    // upload, after it, after inter prediction + residuals, after intra, at the end)
    bool tm_on = false;
    std::vector<hipEvent_t> tm_ev;
    double tm_host_ms = 0, tm_stage_ms = 0, tm_strips_ms = 0;
    int64_t tm_bytes = 0;
    int tm_frames = 0;
    void tm_clear() {
        for (hipEvent_t e : tm_ev) (void)hipEventDestroy(e);
        tm_ev.clear();
        tm_host_ms = tm_stage_ms = tm_strips_ms = 0;
        tm_bytes = 0;
        tm_frames = 0;
    }
    ~MiCtx() {
        tm_clear();
        if (fx_ev) (void)hipEventDestroy(fx_ev);
        if (fx_dev) (void)hipFree(fx_dev);
        if (fx_host) (void)hipHostFree(fx_host);
        if (ir_done) (void)hipFree(ir_done);
        if (mc_flags) (void)hipFree(mc_flags);
        if (mc_err) (void)hipFree(mc_err);
        if (dc_map) (void)hipFree(dc_map);
        if (ir_words) (void)hipFree(ir_words);
        if (ir_gran) (void)hipFree(ir_gran);
        if (ir_tl) (void)hipFree(ir_tl);
        if (fg_lut) (void)hipFree(fg_lut);
        if (fg_scaling) (void)hipFree(fg_scaling);
        if (fg_offsets) (void)hipFree(fg_offsets);
    }
};

struct MiIntraFrame;
namespace mi_internal {
// mi_intra_recon over frames, or (nstrips > 1, one frame) over the frame's strips: queue q =
// blocks [strip_start[q], strip_start[q + 1]) on XCD q (capi.cpp)
// granules: edges handed over as data-tagged granules (ipred.hip); then deps need list only the
// blocks whose pixels are read beyond the edges (CfL luma, intra block copy sources)
int intra_recon(MiCtx *ctx, const MiIntraFrame *frames, int nframes, const int32_t *strip_start, int nstrips,
                unsigned flags, void *stream, bool granules = false);
}
