// api.cpp — the C-ABI of the front-end (include/mi_av1dec.h).
#include <cerrno>
#include <new>

#include "decoder.h"
#include "mi_av1dec.h"

struct MiDec {
    av1::Decoder dec;
    av1::DecEvent cur;
    MiDecFrame frame;
    std::vector<int32_t> release;
    std::string err;
    int inloop = MI_INLOOPFILTER_ALL;
};

extern "C" {

int mi_dec_create(MiDec **out) {
    if (!out) return -EINVAL;
    MiDec *d = new (std::nothrow) MiDec;
    if (!d) return -ENOMEM;
    *out = d;
    return 0;
}

void mi_dec_destroy(MiDec *d) { delete d; }

int mi_dec_set_threads(MiDec *d, int n) {
    if (!d || n < 1) return -EINVAL;
    d->dec.set_threads(n);
    return 0;
}

int mi_dec_set_inloop_filters(MiDec *d, int flags) {
    if (!d || (flags & ~MI_INLOOPFILTER_ALL)) return -EINVAL;
    d->inloop = flags;
    return 0;
}

const char *mi_dec_error(const MiDec *d) { return d ? d->dec.error.c_str() : "null decoder"; }

int mi_dec_send(MiDec *d, const uint8_t *data, size_t size) {
    if (!d || (!data && size)) return -EINVAL;
    try {
        const int r = d->dec.send(data, size);
        if (r < 0 && d->dec.error.find("not supported") != std::string::npos) return -ENOTSUP;
        return r;
    } catch (const std::bad_alloc &) {
        d->dec.error = "out of memory";
        return -ENOMEM;
    } catch (const std::exception &e) {
        // e.g. std::system_error from a frame thread that could not be started: no C++
        // exception crosses the C ABI
        d->dec.error = e.what();
        return -EAGAIN;
    }
}

int mi_dec_next(MiDec *d, MiDecEvent *ev) {
    if (!d || !ev) return -EINVAL;
    int r;
    try {
        r = d->dec.pop(d->cur);
    } catch (const std::exception &e) {
        d->dec.error = e.what();
        return -EAGAIN;
    }
    if (r <= 0) {
        if (r < 0 && d->dec.error.find("not supported") != std::string::npos) return -ENOTSUP;
        return r;
    }
    const av1::DecEvent &e = d->cur;
    memset(ev, 0, sizeof(*ev));
    ev->pic_id = e.pic_id;
    for (int i = 0; i < 7; i++) ev->ref_pic[i] = e.ref_pic[i];
    ev->show_pic = e.show_pic;
    ev->fg_present = e.fg_present;
    ev->fg = e.fg;
    ev->mtrx_identity = e.mtrx_identity;
    d->release.assign(e.release.begin(), e.release.end());
    ev->release = d->release.data();
    ev->n_release = (int32_t)d->release.size();
    if (e.work) {
        const av1::FrameWork &w = *e.work;
        MiDecFrame &f = d->frame;
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
        // Dav1dSettings.inloop_filters: a filter switched off is skipped for the whole frame
        const bool dbl = d->inloop & MI_INLOOPFILTER_DEBLOCK;
        f.filter_y = dbl ? w.filter_y : 0;
        f.filter_uv = dbl ? w.filter_uv : 0;
        f.lf_level = w.lf_level.data();
        f.b4_stride = w.b4_stride;
        f.lf_masks = w.lf_masks.data();
        f.sb128w = w.sb128w;
        f.sb128h = w.sb128h;
        memcpy(f.lim_e, w.lim_e, 64);
        memcpy(f.lim_i, w.lim_i, 64);
        f.cdef_on = (d->inloop & MI_INLOOPFILTER_CDEF) ? w.cdef_on : 0;
        f.cdef_damping = w.cdef_damping;
        memcpy(f.cdef_y, w.cdef_y, 8);
        memcpy(f.cdef_uv, w.cdef_uv, 8);
        f.lr_mask = w.lr_mask.data();
        f.lr_sb128w = w.sr_sb128w;
        f.restore_planes = (d->inloop & MI_INLOOPFILTER_RESTORATION) ? w.restore_planes : 0;
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
        ev->frame = &f;
    }
    return 1;
}

}  // extern "C"
