// plan.cpp — the MiDecFrame view of a FrameWork (what mi_dec_next hands out) and the frame's
// intra queue, planned on the front-end's frame thread: the queue mi_frame_run would otherwise
// plan on its own host pass (csrc/intra_plan.h; frame_exec.cpp plan_frame), now off the
// device's critical path (MiDecFrame.q_*).
#include <algorithm>

#include "decoder.h"
#include "../csrc/intra_plan.h"

namespace av1 {

void frame_view(const FrameWork &w, MiDecFrame &f) {
    memset(&f, 0, sizeof(f));
    f.w = w.w;
    f.h = w.h;
    f.up_w = w.up_w;
    f.render_w = w.render_w;
    f.render_h = w.render_h;
    f.bpc = w.bpc;
    f.layout = w.layout;
    f.sb128 = w.sb128;
    f.intra = w.intra.data();
    f.intra_tx = w.intra_tx.data();
    f.n_intra = (int32_t)w.intra.size();
    f.dep_start = w.dep_start.data();
    f.deps = w.deps.data();
    f.n_deps = (int32_t)w.deps.size();
    f.inter_tx = w.inter_tx.data();
    f.n_inter_tx = (int32_t)w.inter_tx.size();
    f.coef = w.coef.data();
    f.ncoef = w.ncoef;
    f.idx = w.idx.data();
    f.nidx = w.idx.size();
    f.pal = w.pal.data();
    f.npal = w.pal.size() / (w.bpc == 8 ? 1 : 2);
    f.filter_y = w.filter_y;
    f.filter_uv = w.filter_uv;
    f.lf_level = w.lf_level.data();
    f.b4_stride = w.b4_stride;
    f.lf_masks = w.lf_masks.data();
    f.sb128w = w.sb128w;
    f.sb128h = w.sb128h;
    memcpy(f.lim_e, w.lim_e, 64);
    memcpy(f.lim_i, w.lim_i, 64);
    f.cdef_on = w.cdef_on;
    f.cdef_damping = w.cdef_damping;
    memcpy(f.cdef_y, w.cdef_y, 8);
    memcpy(f.cdef_uv, w.cdef_uv, 8);
    f.lr_mask = w.lr_mask.data();
    f.lr_sb128w = w.sr_sb128w;
    f.restore_planes = w.restore_planes;
    f.lr_unit_size[0] = w.lr_unit_size[0];
    f.lr_unit_size[1] = w.lr_unit_size[1];
    f.mc = w.mc.data();
    f.n_mc = (int32_t)w.mc.size();
    f.obmc_h = w.obmc_h.data();
    f.n_obmc_h = (int32_t)w.obmc_h.size();
    f.obmc_v = w.obmc_v.data();
    f.n_obmc_v = (int32_t)w.obmc_v.size();
    f.warp = w.warp.data();
    f.n_warp = (int32_t)w.warp.size();
    f.scaled = w.scaled.data();
    f.n_scaled = (int32_t)w.scaled.size();
    f.combine_y = w.combine_y.data();
    f.n_combine_y = (int32_t)w.combine_y.size();
    f.combine_uv = w.combine_uv.data();
    f.n_combine_uv = (int32_t)w.combine_uv.size();
    f.masks = w.masks.data();
    f.nmasks = w.masks.size();
    f.ntmp = w.ntmp;
    if (w.q) {
        const mi_plan::IntraQueue &q = *w.q;
        f.q_intra = q.blocks.data();
        f.q_intra_tx = q.tx.data();
        f.q_dep_start = q.dep_start.data();
        f.q_deps = q.deps.data();
        f.q_n_deps = (int32_t)q.dep_start[f.n_intra];
        f.q_nstrips = q.strip_start.empty() ? 1 : (int32_t)q.strip_start.size() - 1;
        f.q_strip_start = q.strip_start.empty() ? nullptr : q.strip_start.data();
        f.q_granules = q.granules;
    }
}

void plan_intra_queue(FrameWork &w, WorkerPool *pool) {
    w.q.reset();
    MiDecFrame f;
    frame_view(w, f);
    auto q = std::make_shared<mi_plan::IntraQueue>();
    const int nt = pool ? std::min(8, pool->workers() + 1) : 1;
    // fn(lo, hi, t) over up to nt contiguous ranges of [0, n) (range t a task of the pool), at
    // least min_n items each
    mi_plan::plan_intra(&f, *q, [nt, pool](int n, int min_n, auto &&fn) {
        int parts = n / (min_n > 0 ? min_n : 1);
        parts = parts < 1 ? 1 : parts > nt ? nt : parts;
        if (parts == 1) {
            fn(0, n, 0);
            return 1;
        }
        pool->run(parts, [&](int t) { fn((int)((int64_t)n * t / parts), (int)((int64_t)n * (t + 1) / parts), t); });
        return parts;
    });
    w.q = std::move(q);
}

}  // namespace av1
