// frame_exec.cpp — mi_frame_run / mi_frame_end (include/mi_av1dec.h): one front-end work list
// (MiDecFrame) executed on the device.
//
// The reference reconstructs a frame superblock row by superblock row, interleaving
// decode_tile_sbrow and filter_sbrow (decode.rs:4526-4550; recon.rs:4019-4211). With the
// whole frame's work list known up front the device runs it as four whole-frame stages on
// one stream: intra reconstruction (one persistent launch over the blocks in dependency-level
// order), deblocking recon -> deblocked, CDEF deblocked -> cdef, loop restoration
// (cdef, deblocked) -> restored (out-of-place buffers stand in for the
// reference's line backups).
//
// The work list is validated on the host before anything is enqueued (-EINVAL, never a
// device fault), then copied into one pinned staging blob and uploaded with a single async
// copy.
#include <errno.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "ctx.h"
#include "../../include/mi_av1dec.h"

namespace {

// Legal TxfmType values per RectTxfmSize (itx.rs:400-457): the 4/8/16-class rectangles and
// 8x8 and below carry all 16 (4x4 also WHT_WHT = 16), 16x16 the first 12, the 32 class
// DCT_DCT + IDTX, the 64 class DCT_DCT only.
bool legal_txtp(int tx, int txtp) {
    if (tx < 0 || tx >= MI_N_RECT_TX_SIZES || txtp < 0) return false;
    const mi::TxDim d = mi::tx_dim(tx);
    const int m = std::max(d.w, d.h);
    if (txtp == 16) return tx == 0;
    if (m == 64) return txtp == 0;
    if (m == 32) return txtp == 0 || txtp == 9;
    if (d.w == 16 && d.h == 16) return txtp < 12;
    return txtp < 16;
}

int tx_of(int w, int h) {
    for (int t = 0; t < MI_N_RECT_TX_SIZES; t++)
        if (mi::tx_dim(t).w == w && mi::tx_dim(t).h == h) return t;
    return -1;
}

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

struct Section {
    const void *src;
    size_t bytes;
    size_t off;
};

int validate(const MiDecFrame *f, const MiFramePictures *p) {
    if (f->bpc != 8 && f->bpc != 10 && f->bpc != 12) return -EINVAL;
    if (f->layout < 0 || f->layout > 3 || f->w <= 0 || f->h <= 0) return -EINVAL;
    // super-resolution (up_w > w): every picture has the upscaled geometry
    if (f->up_w < f->w || f->up_w > 2 * f->w + 16) return -EINVAL;
    const MiPicture *pics[4] = { &p->recon, &p->deblocked, &p->cdef, &p->restored };
    for (const MiPicture *q : pics)
        if (q->bpc != f->bpc || q->layout != f->layout || q->w != f->up_w || q->h != f->h || !q->data[0] ||
            (f->layout && (!q->data[1] || !q->data[2])) || q->stride[0] != p->recon.stride[0] ||
            q->stride[1] != p->recon.stride[1])
            return -EINVAL;
    const int ss_hor = f->layout == 1 || f->layout == 2, ss_ver = f->layout == 1;
    const int nplanes = f->layout ? 3 : 1;
    const int aw = (f->w + 127) & ~127, ah = (f->h + 127) & ~127, aw_up = (f->up_w + 127) & ~127;
    const size_t pb = f->bpc == 8 ? 1 : 2;
    for (int pl = 0; pl < nplanes; pl++)
        if ((size_t)std::abs(p->recon.stride[pl ? 1 : 0]) < (size_t)(aw_up >> (pl ? ss_hor : 0)) * pb) return -EINVAL;
    if (f->n_intra < 0 || (f->n_intra && (!f->intra || !f->intra_tx || !f->dep_start))) return -EINVAL;
    if (f->n_intra && f->ncoef < 16) return -EINVAL;
    if (f->dep_start && (f->dep_start[0] != 0 || f->dep_start[f->n_intra] != f->n_deps)) return -EINVAL;
    for (int i = 0; i < f->n_intra; i++) {
        const MiIntraBlock &b = f->intra[i];
        const MiTxBlock &t = f->intra_tx[i];
        if (b.plane >= nplanes || t.plane != b.plane || t.x != b.x || t.y != b.y) return -EINVAL;
        const int tx = tx_of(b.w, b.h);
        if (tx < 0 || t.tx != tx) return -EINVAL;
        const int sh = b.plane ? ss_hor : 0, sv = b.plane ? ss_ver : 0;
        if (b.x + b.w > (aw >> sh) || b.y + b.h > (ah >> sv)) return -EINVAL;
        if (t.eob >= 0) {
            if (!legal_txtp(tx, t.txtp)) return -EINVAL;
            const mi::TxDim d = mi::tx_dim(tx);
            if ((size_t)t.coef_off + (size_t)std::min(d.w, 32) * std::min(d.h, 32) > f->ncoef) return -EINVAL;
        } else if (t.coef_off + 16 > f->ncoef || t.txtp != 0) {
            return -EINVAL;
        }
        const int mode = b.mode & ~MI_IPRED_II;
        if (mode == MI_IPRED_PAL) {
            if ((size_t)b.aux_off + (size_t)b.w * b.h > f->nidx || (size_t)b.pal_off + 8 > f->npal) return -EINVAL;
        } else if (mode == MI_INTRA_IBC) {
            // the reference area the copy clamps its taps to lies inside the picture
            if (b.filt_idx != (sh | (sv << 1)) || !b.max_w || !b.max_h || b.max_w > (aw >> sh) ||
                b.max_h > (ah >> sv) || (b.mode & MI_IPRED_II))
                return -EINVAL;
        } else if (mode != MI_IPRED_CFL && mode > 13) {
            return -EINVAL;
        }
        if ((b.mode & MI_IPRED_II) || (b.flags & MI_INTRA_II)) return -EINVAL;   // inter-intra: inter frames
        for (int d = f->dep_start[i]; d < f->dep_start[i + 1]; d++)
            if (d < 0 || d >= f->n_deps || f->deps[d] < 0 || f->deps[d] >= i) return -EINVAL;
        if (f->dep_start[i + 1] < f->dep_start[i]) return -EINVAL;
    }
    const int sb128w = (f->w + 127) >> 7, sb128h = (f->h + 127) >> 7;
    if (f->filter_y && (!f->lf_level || !f->lf_masks || f->sb128w != sb128w || f->sb128h != sb128h ||
                        f->b4_stride < sb128w * 32))
        return -EINVAL;
    if (f->cdef_on && (!f->lf_masks || f->sb128w != sb128w || f->sb128h != sb128h)) return -EINVAL;
    if (f->restore_planes && (!f->lr_mask || f->lr_sb128w != ((f->up_w + 127) >> 7))) return -EINVAL;
    if (f->n_inter_tx) return -EINVAL;     // inter frames: not produced by the front-end yet
    return 0;
}

int stage_upload(MiCtx *ctx, std::vector<Section> &secs, hipStream_t s) {
    size_t total = 0;
    for (Section &x : secs) {
        x.off = total;
        total += align256(x.bytes);
    }
    total = std::max<size_t>(total, 256);
    // the previous frame's upload must have left the staging buffer
    if (ctx->fx_ev_pending) {
        if (hipEventSynchronize(ctx->fx_ev) != hipSuccess) return -EIO;
        ctx->fx_ev_pending = false;
    }
    if (total > ctx->fx_host_bytes) {
        if (ctx->fx_host) (void)hipHostFree(ctx->fx_host);
        ctx->fx_host = nullptr;
        ctx->fx_host_bytes = 0;
        const size_t n = total + total / 2;
        if (hipHostMalloc((void **)&ctx->fx_host, n, hipHostMallocDefault) != hipSuccess) return -ENOMEM;
        ctx->fx_host_bytes = n;
    }
    if (total > ctx->fx_dev_bytes) {
        // earlier frames' kernels on this stream may still read the old buffer
        if (hipStreamSynchronize(s) != hipSuccess) return -EIO;
        if (ctx->fx_dev) (void)hipFree(ctx->fx_dev);
        ctx->fx_dev = nullptr;
        ctx->fx_dev_bytes = 0;
        const size_t n = total + total / 2;
        if (hipMalloc((void **)&ctx->fx_dev, n) != hipSuccess) return -ENOMEM;
        ctx->fx_dev_bytes = n;
    }
    for (const Section &x : secs)
        if (x.bytes) memcpy(ctx->fx_host + x.off, x.src, x.bytes);
    if (!ctx->fx_ev && hipEventCreateWithFlags(&ctx->fx_ev, hipEventDisableTiming) != hipSuccess) return -EIO;
    if (hipMemcpyAsync(ctx->fx_dev, ctx->fx_host, total, hipMemcpyHostToDevice, s) != hipSuccess) return -EIO;
    if (hipEventRecord(ctx->fx_ev, s) != hipSuccess) return -EIO;
    ctx->fx_ev_pending = true;
    return 0;
}

} // namespace

extern "C" {

int mi_frame_run(MiCtx *ctx, const MiDecFrame *f, const MiFramePictures *pics, int *final, void *stream) {
    if (!ctx || !f || !pics || !final) return -EINVAL;
    int r = validate(f, pics);
    if (r) return ctx->last_error = r;
    hipStream_t s = (hipStream_t)stream;
    const size_t cb = f->bpc == 8 ? 2 : 4, pb = f->bpc == 8 ? 1 : 2;
    const int n = f->n_intra;

    // dependency levels (deps always point backwards): level order lets the persistent
    // kernel's workers run every block of a level side by side
    std::vector<MiIntraBlock> blocks(n);
    std::vector<MiTxBlock> tx(n);
    std::vector<int32_t> dep_start(n + 1), deps(std::max(1, f->n_deps));
    if (n) {
        std::vector<int32_t> level(n), pos(n);
        int maxl = 0;
        for (int i = 0; i < n; i++) {
            int l = 0;
            for (int d = f->dep_start[i]; d < f->dep_start[i + 1]; d++) l = std::max(l, level[f->deps[d]] + 1);
            level[i] = l;
            maxl = std::max(maxl, l);
        }
        std::vector<int32_t> cnt(maxl + 2, 0);
        for (int i = 0; i < n; i++) cnt[level[i] + 1]++;
        for (int l = 0; l <= maxl; l++) cnt[l + 1] += cnt[l];
        for (int i = 0; i < n; i++) pos[i] = cnt[level[i]]++;
        std::vector<int32_t> inv(n);
        for (int i = 0; i < n; i++) inv[pos[i]] = i;
        int nd = 0;
        for (int k = 0; k < n; k++) {
            const int i = inv[k];
            blocks[k] = f->intra[i];
            tx[k] = f->intra_tx[i];
            dep_start[k] = nd;
            for (int d = f->dep_start[i]; d < f->dep_start[i + 1]; d++) deps[nd++] = pos[f->deps[d]];
        }
        dep_start[n] = nd;
    }
    const int sb128h = (f->h + 127) >> 7;
    std::vector<Section> secs = {
        { blocks.data(), blocks.size() * sizeof(MiIntraBlock), 0 },
        { tx.data(), tx.size() * sizeof(MiTxBlock), 0 },
        { dep_start.data(), dep_start.size() * 4, 0 },
        { deps.data(), deps.size() * 4, 0 },
        { f->coef, f->ncoef * cb, 0 },
        { f->idx, f->nidx, 0 },
        { f->pal, f->npal * pb, 0 },
        { f->lf_level, f->filter_y ? (size_t)f->b4_stride * sb128h * 32 * 4 : 0, 0 },
        { f->lf_masks, (f->filter_y || f->cdef_on) ? (size_t)f->sb128w * sb128h * sizeof(MiAv1Filter) : 0, 0 },
        { f->lr_mask, f->restore_planes ? (size_t)f->lr_sb128w * sb128h * sizeof(MiAv1Restoration) : 0, 0 },
    };
    if ((r = stage_upload(ctx, secs, s))) return ctx->last_error = r;
    uint8_t *dev = ctx->fx_dev;
    auto D = [&](int i) -> void * { return secs[i].bytes ? dev + secs[i].off : nullptr; };

    // 1. intra reconstruction (prediction + residual per transform block)
    if (n) {
        MiIntraFrame fr;
        memset(&fr, 0, sizeof(fr));
        fr.pic = pics->recon;
        fr.pic.w = f->w;                 // coded width (super-resolution upscales after CDEF)
        fr.blocks = (const MiIntraBlock *)D(0);
        fr.tx = (const MiTxBlock *)D(1);
        fr.dep_start = (const int32_t *)D(2);
        fr.deps = (const int32_t *)D(3);
        fr.coef = D(4);
        fr.idx = (const uint8_t *)D(5);
        fr.pal = D(6);
        fr.n = n;
        if ((r = mi_intra_recon(ctx, &fr, 1, 0, stream))) return r;
    }
    // the coded-width views of the pictures (stages before super-resolution)
    MiPicture cp[4] = { pics->recon, pics->deblocked, pics->cdef, pics->restored };
    for (MiPicture &q : cp) q.w = f->w;
    const MiPicture *cur = &cp[0];
    int idx = 0;
    // 2. deblocking (lf_apply.rs:597-834), recon -> deblocked
    if (f->filter_y) {
        MiLoopFilter lf;
        memset(&lf, 0, sizeof(lf));
        lf.level = (const uint8_t *)D(7);
        lf.b4_stride = f->b4_stride;
        lf.masks = (const MiAv1Filter *)D(8);
        lf.sb128w = f->sb128w;
        lf.filter_y = f->filter_y;
        lf.filter_uv = f->filter_uv;
        memcpy(lf.lim_e, f->lim_e, 64);
        memcpy(lf.lim_i, f->lim_i, 64);
        if ((r = mi_deblock_frame_to(ctx, cur, &cp[1], &lf, stream))) return r;
        cur = &cp[1];
        idx = 1;
    }
    const MiPicture *deblocked = cur;
    int dbl_idx = idx;
    // 3. CDEF (cdef_apply.rs:159-507), deblocked -> cdef
    if (f->cdef_on) {
        MiCdef cd;
        memset(&cd, 0, sizeof(cd));
        cd.masks = (const MiAv1Filter *)D(8);
        cd.sb128w = f->sb128w;
        cd.damping = f->cdef_damping;
        memcpy(cd.y_strength, f->cdef_y, 8);
        memcpy(cd.uv_strength, f->cdef_uv, 8);
        if ((r = mi_cdef_frame(ctx, cur, &cp[2], &cd, stream))) return r;
        cur = &cp[2];
        idx = 2;
    }
    // 3b. super-resolution (recon.rs:4215-4285 filter_sbrow_resize for the CDEF output;
    // lf_apply.rs backup_lpf resizes the deblocked rows loop restoration reads across stripe
    // edges the same way): both upscaled into pictures no later stage still reads at coded width
    const MiPicture *slot[4] = { &pics->recon, &pics->deblocked, &pics->cdef, &pics->restored };
    if (f->up_w != f->w) {
        // free slots: everything except cur (C) and deblocked (D)
        int fr_[4], nf = 0;
        for (int k = 0; k < 4; k++)
            if (k != idx && k != dbl_idx) fr_[nf++] = k;
        const int cu = fr_[0];
        if ((r = mi_superres_frame(ctx, cur, slot[cu], stream))) return r;
        int du = cu;
        if (f->restore_planes) {
            du = fr_[1];
            if (deblocked != cur && (r = mi_superres_frame(ctx, deblocked, slot[du], stream))) return r;
            if (deblocked == cur) du = cu;
        }
        // loop restoration writes into a slot holding neither input: the coded-width CDEF output
        // (or, without CDEF, the coded-width deblocked picture) is no longer read
        cur = slot[cu];
        deblocked = slot[du];
        idx = cu;
        dbl_idx = du;
    }
    // 4. loop restoration (lr_apply.rs:261-329), (cdef, deblocked) -> restored
    if (f->restore_planes) {
        MiLr lr;
        memset(&lr, 0, sizeof(lr));
        lr.lr_mask = (const MiAv1Restoration *)D(9);
        lr.sb128w = f->lr_sb128w;
        lr.restore_planes = f->restore_planes;
        lr.unit_size_log2[0] = f->lr_unit_size[0];
        lr.unit_size_log2[1] = f->lr_unit_size[1];
        int out = 3;
        if (f->up_w != f->w)
            for (int k = 0; k < 4; k++)
                if (k != idx && k != dbl_idx) { out = k; break; }
        if ((r = mi_lr_frame(ctx, cur, deblocked, slot[out], &lr, stream))) return r;
        idx = out;
    }
    *final = idx;
    return 0;
}

int mi_frame_end(MiCtx *ctx, void *stream) {
    if (!ctx) return -EINVAL;
    const int r = mi_ctx_device_status(ctx, stream);
    // a kernel rejected descriptors: -EINVAL; a stalled or untaken block: -EIO
    return r ? (ctx->last_error = r == -EINVAL ? -EINVAL : -EIO) : 0;
}

}  // extern "C"
