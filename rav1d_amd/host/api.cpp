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
        MiDecFrame &f = d->frame;
        av1::frame_view(*e.work, f);
        // Dav1dSettings.inloop_filters: a filter switched off is skipped for the whole frame
        if (!(d->inloop & MI_INLOOPFILTER_DEBLOCK)) f.filter_y = f.filter_uv = 0;
        if (!(d->inloop & MI_INLOOPFILTER_CDEF)) f.cdef_on = 0;
        if (!(d->inloop & MI_INLOOPFILTER_RESTORATION)) f.restore_planes = 0;
        ev->frame = &f;
    }
    return 1;
}

}  // extern "C"
