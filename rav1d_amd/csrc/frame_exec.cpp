// frame_exec.cpp — mi_frame_run / mi_frame_end (include/mi_av1dec.h): one front-end work list
// (MiDecFrame) executed on the device.
//
// The reference reconstructs a frame superblock row by superblock row, interleaving
// decode_tile_sbrow and filter_sbrow (decode.rs:4526-4550; recon.rs:4019-4211). With the
// whole frame's work list known up front the device runs it as whole-frame stages on one
// stream: inter prediction of every inter block (MC, warp, scaled references, compound
// combines, OBMC laps: they read only reference pictures) and the inter residuals, then intra
// reconstruction (one persistent launch over the intra and inter-intra blocks in
// dependency-level order), deblocking recon -> deblocked, CDEF deblocked -> cdef, loop
// restoration (cdef, deblocked) -> restored (out-of-place buffers stand in for
// the reference's line backups).
//
// The work list is validated on the host before anything is enqueued (-EINVAL, never a
// device fault), then copied into one pinned staging blob and uploaded with a single async
// copy.
#include <errno.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>
#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "ctx.h"
#include "intra_plan.h"
#include "../../include/mi_av1dec.h"

namespace {

// A small pool of host threads for the planning pass of large frames (created on first use,
// never torn down). One job at a time: a caller that finds the pool busy (another context's
// frame_run on another host thread) runs its ranges inline. In a forked child the workers do
// not exist, so a process other than the pool's creator always runs inline; a range whose
// worker threw (bad_alloc) is re-run on the calling thread, where the exception reaches the
// caller as it would in a serial pass.
class PlanPool {
  public:
    explicit PlanPool(int n) : n_(n), pid_(getpid()) {
        for (int t = 1; t < n_; t++) std::thread([this, t] { worker(t); }).detach();
    }
    int size() const { return getpid() == pid_ ? n_ : 1; }
    // fn(t) for t in [0, n_) (t = 0 on the calling thread); false: the pool is busy
    bool run(const std::function<void(int)> &fn) {
        if (getpid() != pid_) return false;
        std::unique_lock<std::mutex> use(use_, std::try_to_lock);
        if (!use.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            left_ = n_ - 1;
            failed_.assign(n_, 0);
            gen_++;
        }
        cv_.notify_all();
        fn(0);
        std::vector<char> failed;
        {
            std::unique_lock<std::mutex> g(m_);
            done_.wait(g, [this] { return left_ == 0; });
            job_ = nullptr;
            failed.swap(failed_);
        }
        for (int t = 1; t < n_; t++)
            if (failed[t]) fn(t);
        return true;
    }

  private:
    void worker(int t) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)> *job;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                job = job_;
            }
            bool ok = true;
            try {
                (*job)(t);
            } catch (...) {
                ok = false;
            }
            std::lock_guard<std::mutex> g(m_);
            if (!ok) failed_[t] = 1;
            if (--left_ == 0) done_.notify_one();
        }
    }
    const int n_;
    const pid_t pid_;
    std::vector<char> failed_;
    std::mutex use_, m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    uint64_t gen_ = 0;
    int left_ = 0;
};

PlanPool *plan_pool() {
    static PlanPool *pool = new PlanPool(std::max(1, std::min((int)std::thread::hardware_concurrency(), 8)));
    return pool;
}

// fn(lo, hi, t) over [0, n) in contiguous ranges, one per pool thread; below `min_n` items (or
// with the pool busy) on the calling thread alone. Returns the number of ranges.
template <typename Fn>
int parallel_ranges(int n, int min_n, Fn &&fn) {
    PlanPool *pool = plan_pool();
    const int nt = n < min_n ? 1 : pool->size();
    if (nt > 1) {
        const std::function<void(int)> job = [&](int t) {
            fn((int)((int64_t)n * t / nt), (int)((int64_t)n * (t + 1) / nt), t);
        };
        if (pool->run(job)) return nt;
    }
    fn(0, n, 0);
    return 1;
}

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
    const void *src;      // nullptr: device scratch, not uploaded (after every uploaded section)
    size_t bytes;
    size_t off;
};

int ilog2(int v) { return 31 - __builtin_clz((unsigned)v); }

// MiMcBlock units bucketed as mi_mc_frame takes them: plane group (luma, chroma), then shape
// class log2(w) * 8 + log2(h)
void bucket_mc(const MiMcBlock *u, int n, std::vector<MiMcBlock> &out, uint32_t cs[2 * MI_MC_NCLASS + 1]) {
    std::vector<uint32_t> cnt(2 * MI_MC_NCLASS + 1, 0);
    auto key = [](const MiMcBlock &b) { return (b.plane ? MI_MC_NCLASS : 0) + ilog2(b.w) * 8 + ilog2(b.h); };
    for (int i = 0; i < n; i++) cnt[key(u[i]) + 1]++;
    for (int k = 0; k < 2 * MI_MC_NCLASS; k++) cnt[k + 1] += cnt[k];
    for (int k = 0; k <= 2 * MI_MC_NCLASS; k++) cs[k] = cnt[k];
    out.resize(n);
    for (int i = 0; i < n; i++) out[cnt[key(u[i])]++] = u[i];
}

// the check a rejected work list failed (mi_frame_validate's `why`)
thread_local const char *g_why = nullptr;
#define STR2(x) #x
#define STR(x) STR2(x)
#define BAD() (g_why = "frame_exec.cpp:" STR(__LINE__), -EINVAL)

// the coefficients a transform block reads from the arena: a DC-only block (DCT_DCT, eob < 1)
// its DC alone (the front-end stores only that), a packed block its CW x CH corner
// (MI_TX_PACKED; half as many int32 entries with MI_TX_I16), any other the min(w,32) x min(h,32) run; illegal flags: more than any arena
size_t coef_span(const mi::TxDim &d, int txtp, int eob, uint8_t flags, uint32_t coef_off, bool hbd) {
    const int sw = std::min(d.w, 32), sh = std::min(d.h, 32);
    if (!mi::tx_flags_ok(flags, sw, sh, coef_off, hbd)) return SIZE_MAX / 2;
    if (txtp == 0 && eob < 1) return 1;
    const mi::TxCoefShape cs = mi::tx_coef_shape(flags, sw, sh);
    return (size_t)cs.cw * cs.ch / (flags & MI_TX_I16 ? 2 : 1);
}
#define BADF() (g_why = "frame_exec.cpp:" STR(__LINE__), false)

bool pow2_in(int v, int lo, int hi) { return v >= lo && v <= hi && !(v & (v - 1)); }

bool inter_present(const MiDecFrame *f) { return mi_plan::inter_present(f); }

// The reference pictures an inter frame's units read (same bit depth and layout, planes present)
// and which of them differ in size from the frame (the scaled-reference path).
int validate_refs(const MiDecFrame *f, const MiFramePictures *p, bool scaled[7]) {
    for (int r = 0; r < 7; r++) {
        const MiPicture &q = p->refs[r];
        scaled[r] = false;
        if (!q.data[0]) continue;
        if (q.bpc != f->bpc || q.layout != f->layout || q.w <= 0 || q.h <= 0 || (f->layout && (!q.data[1] || !q.data[2])))
            return BAD();
        // svc scale factors (decode.rs:4776): 2x down to 1/16 x
        if (2 * f->w < q.w || 2 * f->h < q.h || f->w > 16 * q.w || f->h > 16 * q.h) return BAD();
        scaled[r] = q.w != f->w || q.h != f->h || q.stride[0] != p->recon.stride[0] || q.stride[1] != p->recon.stride[1];
    }
    return 0;
}

int validate_inter(const MiDecFrame *f, const MiFramePictures *p, const bool scaled[7]) {
    const int ss_hor = f->layout == 1 || f->layout == 2, ss_ver = f->layout == 1;
    const int nplanes = f->layout ? 3 : 1;
    const int aw = (f->w + 127) & ~127, ah = (f->h + 127) & ~127;
    auto ref_ok = [&](int r) { return r >= 0 && r < 7 && p->refs[r].data[0]; };
    // a unit's rectangle, references, and the mask / tmp bytes it touches
    auto unit_ok = [&](const MiMcBlock &u, bool allow_scaled, bool lap) {
        if (u.plane >= nplanes || !pow2_in(u.w, 2, 128) || !pow2_in(u.h, 2, 128)) return BADF();
        const int sh = u.plane ? ss_hor : 0, sv = u.plane ? ss_ver : 0;
        if (u.x + u.w > (aw >> sh) || u.y + u.h > (ah >> sv)) return BADF();
        if (u.filter2d > 9 || !ref_ok(u.ref[0]) || (!allow_scaled && scaled[u.ref[0]])) return BADF();
        if (lap) return (u.comp == MI_MC_OBMC_H || u.comp == MI_MC_OBMC_V) && u.ref[1] < 0 &&
                        (u.comp == MI_MC_OBMC_V || (u.param >= 2 && u.param <= u.h * 2 && u.param <= 64));
        if (u.ref[1] >= 0) {
            if (!ref_ok(u.ref[1]) || scaled[u.ref[1]] || u.comp > MI_MC_SEG) return BADF();
            if (u.comp == MI_MC_MASK && (size_t)u.mask_off + (size_t)u.w * u.h > f->nmasks) return BADF();
            if (u.comp == MI_MC_SEG) {
                const int ms = f->layout ? ss_hor : 0, mv = f->layout ? ss_ver : 0;
                if ((size_t)u.mask_off + (size_t)(u.w >> ms) * (u.h >> mv) > f->nmasks) return BADF();
            }
            if (u.comp == MI_MC_WAVG && (u.param & 31) > 16) return BADF();
            return true;
        }
        if (u.comp == MI_MC_PREP) return (size_t)u.mask_off + (size_t)u.w * u.h <= f->ntmp;
        return u.comp == 0;
    };
    struct L { const MiMcBlock *u; int n; bool scaled_ok, lap; };
    const L lists[4] = { { f->mc, f->n_mc, false, false }, { f->scaled, f->n_scaled, true, false },
                         { f->obmc_h, f->n_obmc_h, true, true }, { f->obmc_v, f->n_obmc_v, true, true } };
    for (const L &l : lists) {
        if (l.n < 0 || (l.n && !l.u)) return BAD();
        for (int i = 0; i < l.n; i++) {
            if (!unit_ok(l.u[i], l.scaled_ok, l.lap)) return BAD();
            if (l.scaled_ok && !l.lap && (l.u[i].ref[1] >= 0 || (l.u[i].comp != 0 && l.u[i].comp != MI_MC_PREP)))
                return BAD();
        }
    }
    if (f->n_warp < 0 || (f->n_warp && !f->warp)) return BAD();
    for (int i = 0; i < f->n_warp; i++) {
        const MiWarpBlock &w = f->warp[i];
        const int sh = w.plane ? ss_hor : 0, sv = w.plane ? ss_ver : 0;
        if (w.plane >= nplanes || !ref_ok(w.ref) || scaled[w.ref] || w.prep > 1) return BAD();
        if (w.x + 8 > (aw >> sh) || w.y + 8 > (ah >> sv)) return BAD();
        // every filter phase warp8x8 forms (mx + y * beta + x * alpha over the 15 x 8 intermediate
        // samples, my + y * delta + x * gamma over the 8 x 8 outputs) indexes the 193-entry table
        auto phases_ok = [](int64_t m, int64_t sy, int ny, int64_t sx) {
            for (int cy = 0; cy < 2; cy++)
                for (int cx = 0; cx < 2; cx++) {
                    const int64_t t = m + (cy ? ny : 0) * sy + (cx ? 7 : 0) * sx;
                    const int64_t i = 64 + ((t + 512) >> 10);
                    if (i < 0 || i > 192) return false;
                }
            return true;
        };
        if (!phases_ok(w.mx, w.abcd[1], 14, w.abcd[0]) || !phases_ok(w.my, w.abcd[3], 7, w.abcd[2])) return BAD();
        if (w.prep && (w.tmp_stride < 8 || (size_t)w.tmp_off + (size_t)7 * w.tmp_stride + 8 > f->ntmp)) return BAD();
    }
    for (int k = 0; k < 2; k++) {
        const MiMcCombine *c = k ? f->combine_uv : f->combine_y;
        const int n = k ? f->n_combine_uv : f->n_combine_y;
        if (n < 0 || (n && !c)) return BAD();
        for (int i = 0; i < n; i++) {
            const MiMcCombine &u = c[i];
            const int sh = u.plane ? ss_hor : 0, sv = u.plane ? ss_ver : 0;
            if (u.plane >= nplanes || (k == 0) != (u.plane == 0) || !pow2_in(u.w, 2, 128) || !pow2_in(u.h, 2, 128) ||
                u.comp > MI_MC_SEG || u.x + u.w > (aw >> sh) || u.y + u.h > (ah >> sv))
                return BAD();
            for (int t = 0; t < 2; t++)
                if ((size_t)u.tmp_off[t] + (size_t)u.w * u.h > f->ntmp) return BAD();
            if (u.comp == MI_MC_MASK && (size_t)u.mask_off + (size_t)u.w * u.h > f->nmasks) return BAD();
            if (u.comp == MI_MC_SEG) {
                const int ms = f->layout ? ss_hor : 0, mv = f->layout ? ss_ver : 0;
                if ((size_t)u.mask_off + (size_t)(u.w >> ms) * (u.h >> mv) > f->nmasks) return BAD();
            }
        }
    }
    if ((f->nmasks && !f->masks) || f->ntmp > ((size_t)1 << 28)) return BAD();
    if (f->n_inter_tx < 0 || (f->n_inter_tx && !f->inter_tx)) return BAD();
    for (int i = 0; i < f->n_inter_tx; i++) {
        const MiTxBlock &t = f->inter_tx[i];
        if (t.plane >= nplanes || t.tx >= MI_N_RECT_TX_SIZES || t.eob < 0 || !legal_txtp(t.tx, t.txtp)) return BAD();
        const mi::TxDim d = mi::tx_dim(t.tx);
        const int sh = t.plane ? ss_hor : 0, sv = t.plane ? ss_ver : 0;
        if (t.x + d.w > (aw >> sh) || t.y + d.h > (ah >> sv)) return BAD();
        if ((size_t)t.coef_off + coef_span(d, t.txtp, t.eob, t.flags, t.coef_off, f->bpc > 8) > f->ncoef) return BAD();
    }
    return 0;
}

int validate(const MiDecFrame *f, const MiFramePictures *p) {
    if (f->bpc != 8 && f->bpc != 10 && f->bpc != 12) return BAD();
    if (f->layout < 0 || f->layout > 3 || f->w <= 0 || f->h <= 0) return BAD();
    // super-resolution (up_w > w): every picture has the upscaled geometry
    if (f->up_w < f->w || f->up_w > 2 * f->w + 16) return BAD();
    const int ss_hor = f->layout == 1 || f->layout == 2, ss_ver = f->layout == 1;
    const int nplanes = f->layout ? 3 : 1;
    const int aw = (f->w + 127) & ~127, ah = (f->h + 127) & ~127, aw_up = (f->up_w + 127) & ~127;
    const size_t pb = f->bpc == 8 ? 1 : 2;
    if (p) {   // (nullptr: the work list alone, as mi_frame_plan_ms checks it)
        const MiPicture *pics[4] = { &p->recon, &p->deblocked, &p->cdef, &p->restored };
        for (const MiPicture *q : pics)
            if (q->bpc != f->bpc || q->layout != f->layout || q->w != f->up_w || q->h != f->h || !q->data[0] ||
                (f->layout && (!q->data[1] || !q->data[2])) || q->stride[0] != p->recon.stride[0] ||
                q->stride[1] != p->recon.stride[1])
                return BAD();
        for (int pl = 0; pl < nplanes; pl++)
            if ((size_t)std::abs(p->recon.stride[pl ? 1 : 0]) < (size_t)(aw_up >> (pl ? ss_hor : 0)) * pb) return BAD();
        // loop restoration takes positive strides below 2^24 and planes below 4 GB (mi_lr_frame
        // makes the same check; made here too so that nothing is enqueued before it fails)
        if (f->restore_planes)
            for (int pl = 0; pl < nplanes; pl++) {
                const int64_t st = p->recon.stride[pl ? 1 : 0];
                const int64_t ph = pl ? (f->h + ss_ver) >> ss_ver : f->h;
                if (st <= 0 || st >= (1 << 24) || ph * st >= (1LL << 32)) return BAD();
            }
    }
    // every array a count refers to is present (they are copied from during the call)
    if (f->n_intra < 0 || (f->n_intra && (!f->intra || !f->intra_tx || !f->dep_start))) return BAD();
    if (f->n_deps < 0 || (f->n_deps && !f->deps) || (f->ncoef && !f->coef) || (f->nidx && !f->idx) ||
        (f->npal && !f->pal))
        return BAD();
    if ((f->n_intra || f->n_inter_tx) && f->ncoef < 16) return BAD();
    if (f->dep_start && (f->dep_start[0] != 0 || f->dep_start[f->n_intra] != f->n_deps)) return BAD();
    const bool inter = inter_present(f);
    // per-block checks on the planning pool (ranges of blocks; a failing range is re-checked
    // on the calling thread, whose g_why the caller reads)
    // one block with its transform (decode order, or the front-end's queue order)
    auto check_block = [&](const MiIntraBlock &b, const MiTxBlock &t) -> int {
        if (b.plane >= nplanes || t.plane != b.plane || t.x != b.x || t.y != b.y) return BAD();
        const int tx = tx_of(b.w, b.h);
        if (tx < 0 || t.tx != tx) return BAD();
        const int sh = b.plane ? ss_hor : 0, sv = b.plane ? ss_ver : 0;
        if (b.x + b.w > (aw >> sh) || b.y + b.h > (ah >> sv)) return BAD();
        if (t.eob >= 0) {
            if (!legal_txtp(tx, t.txtp)) return BAD();
            const mi::TxDim d = mi::tx_dim(tx);
            if ((size_t)t.coef_off + coef_span(d, t.txtp, t.eob, t.flags, t.coef_off, f->bpc > 8) > f->ncoef) return BAD();
        } else if (t.coef_off + 16 > f->ncoef || (t.txtp != 0 && t.txtp != 16)) {
            return BAD();
        }
        // edge availability: no left / top neighbour at the plane's first column / row; the
        // tile limits inside the plane
        if (((b.flags & MI_INTRA_HAVE_LEFT) && !b.x) || ((b.flags & MI_INTRA_HAVE_TOP) && !b.y)) return BAD();
        if (b.mode != MI_INTRA_RESID && b.mode != MI_IPRED_PAL &&
            (b.tile_w > (aw >> sh) || b.tile_h > (ah >> sv) || b.tile_w <= b.x || b.tile_h <= b.y))
            return BAD();
        const int mode = b.mode;
        if (mode == MI_IPRED_PAL) {
            if ((size_t)b.aux_off + (size_t)b.w * b.h > f->nidx || (size_t)b.pal_off + 8 > f->npal) return BAD();
        } else if (mode == MI_INTRA_IBC) {
            // the reference area the copy clamps its taps to lies inside the picture
            if (b.filt_idx != (sh | (sv << 1)) || !b.max_w || !b.max_h || b.max_w > (aw >> sh) || b.max_h > (ah >> sv))
                return BAD();
        } else if (mode == MI_IPRED_CFL) {
            // CfL (chroma only; the executor has no ac array: the AC comes from the luma under
            // the block) with padded sizes inside the block and the layout's subsampling
            if (!(b.flags & MI_INTRA_CFL_AC) || !b.plane) return BAD();
            const unsigned wp = b.reserved & 0xff, hp = (b.reserved >> 8) & 0xff;
            if (((b.reserved >> 16) & 1) != (unsigned)ss_hor || ((b.reserved >> 17) & 1) != (unsigned)ss_ver ||
                wp * 4 > b.w || hp * 4 > b.h || (b.reserved >> 18))
                return BAD();
        } else if (mode == 13) {
            if (b.filt_idx >= 5 || b.w > 32 || b.h > 32) return BAD();   // filter intra: 5 taps sets, <= 32x32
        } else if (mode >= 1 && mode <= 8) {
            if (b.angle < -3 || b.angle > 3) return BAD();
        } else if (mode != MI_INTRA_RESID && mode > 12) {
            return BAD();
        }
        if (b.flags & MI_INTRA_II) {
            // inter-intra: slots 0-12 with the blend mask in idx, in an inter frame
            if (mode > 12 || (size_t)b.aux_off + (size_t)b.w * b.h > f->nidx || !inter) return BAD();
        }
        return 0;
    };
    auto check = [&](int i) -> int {
        if (int e = check_block(f->intra[i], f->intra_tx[i])) return e;
        for (int d = f->dep_start[i]; d < f->dep_start[i + 1]; d++)
            if (d < 0 || d >= f->n_deps || f->deps[d] < 0 || f->deps[d] >= i) return BAD();
        if (f->dep_start[i + 1] < f->dep_start[i]) return BAD();
        return 0;
    };
    // the front-end's intra queue (MiDecFrame.q_*), when given, is what the kernels read: its
    // blocks get the per-block checks, and its dependencies must lie inside it and, within a
    // strip, point to earlier queue entries (the strip's workers take entries in order; a
    // dependency on another strip is waited for with a bounded wait). The decode-order lists
    // then keep only their structural checks.
    const bool q = f->q_intra != nullptr;
    const int n = f->n_intra;
    if (q) {
        if (!f->q_intra_tx || !f->q_dep_start || f->q_n_deps < 0 || (f->q_n_deps && !f->q_deps)) return BAD();
        if (f->q_dep_start[0] != 0 || f->q_dep_start[n] != f->q_n_deps) return BAD();
        if (f->q_nstrips > 1) {
            if (!f->q_strip_start || f->q_nstrips > 8 || f->q_strip_start[0] != 0 || f->q_strip_start[f->q_nstrips] != n)
                return BAD();
            for (int k = 0; k < f->q_nstrips; k++)
                if (f->q_strip_start[k + 1] < f->q_strip_start[k]) return BAD();
        }
    }
    const int nss = q && f->q_nstrips > 1 ? f->q_nstrips : 1;
    auto check_q = [&](int i) -> int {
        if (int e = check_block(f->q_intra[i], f->q_intra_tx[i])) return e;
        if (f->q_dep_start[i + 1] < f->q_dep_start[i]) return BAD();
        int lo = 0, hi = n;   // entry i's strip
        for (int k = 0; nss > 1 && k < nss; k++)
            if (i < f->q_strip_start[k + 1]) {
                lo = f->q_strip_start[k];
                hi = f->q_strip_start[k + 1];
                break;
            }
        for (int d = f->q_dep_start[i]; d < f->q_dep_start[i + 1]; d++) {
            const int j = f->q_deps[d];
            if (j < 0 || j >= n || j == i || (j > i && j >= lo && j < hi)) return BAD();
        }
        return 0;
    };
    std::atomic<int> bad{0};
    parallel_ranges(n, 32768, [&](int lo, int hi, int) {
        for (int i = lo; i < hi && !bad.load(std::memory_order_relaxed); i++)
            if (q ? check_q(i) : check(i)) bad.store(1, std::memory_order_relaxed);
    });
    if (bad.load())
        for (int i = 0; i < n; i++)
            if (int e = q ? check_q(i) : check(i)) return e;
    const int sb128w = (f->w + 127) >> 7, sb128h = (f->h + 127) >> 7;
    if (f->filter_y && (!f->lf_level || !f->lf_masks || f->sb128w != sb128w || f->sb128h != sb128h ||
                        f->b4_stride < sb128w * 32))
        return BAD();
    if (f->cdef_on && (!f->lf_masks || f->sb128w != sb128w || f->sb128h != sb128h)) return BAD();
    if (f->restore_planes && (!f->lr_mask || f->lr_sb128w != ((f->up_w + 127) >> 7))) return BAD();
    return 0;
}

int stage_upload(MiCtx *ctx, std::vector<Section> &secs, hipStream_t s, hipEvent_t before = nullptr,
                 int64_t *bytes = nullptr) {
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
    size_t upload = 0;
    // the sections' bytes in 1-MB pieces, copied on several threads (tens of MB for a 4K frame)
    struct Piece { size_t dst, len; const uint8_t *src; };
    std::vector<Piece> pieces;
    for (const Section &x : secs)
        if (x.bytes && x.src) {
            for (size_t o = 0; o < x.bytes; o += (1u << 20))
                pieces.push_back({ x.off + o, std::min<size_t>(1u << 20, x.bytes - o), (const uint8_t *)x.src + o });
            upload = std::max(upload, x.off + x.bytes);
        }
    parallel_ranges((int)pieces.size(), 4, [&](int lo, int hi, int) {
        for (int i = lo; i < hi; i++) memcpy(ctx->fx_host + pieces[i].dst, pieces[i].src, pieces[i].len);
    });
    if (!ctx->fx_ev && hipEventCreateWithFlags(&ctx->fx_ev, hipEventDisableTiming) != hipSuccess) return -EIO;
    if (before && hipEventRecord(before, s) != hipSuccess) return -EIO;
    if (bytes) *bytes = (int64_t)upload;
    if (upload && hipMemcpyAsync(ctx->fx_dev, ctx->fx_host, upload, hipMemcpyHostToDevice, s) != hipSuccess)
        return -EIO;
    if (hipEventRecord(ctx->fx_ev, s) != hipSuccess) return -EIO;
    ctx->fx_ev_pending = true;
    return 0;
}

} // namespace

namespace {

// the five stage events of one timed frame (mi_ctx_set_timing); released unless committed
struct StageEvents {
    hipEvent_t ev[5] = {};
    bool on = false;
    explicit StageEvents(bool timing) : on(timing) {
        if (on)
            for (hipEvent_t &e : ev)
                if (hipEventCreate(&e) != hipSuccess) e = nullptr;
    }
    void mark(int k, hipStream_t s) {
        if (ev[k]) (void)hipEventRecord(ev[k], s);
    }
    ~StageEvents() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

int frame_run(MiCtx *ctx, const MiDecFrame *f, const MiFramePictures *pics, int *final, void *stream,
              StageEvents &tev, int64_t *bytes);

}  // namespace

extern "C" {

int mi_frame_run(MiCtx *ctx, const MiDecFrame *f, const MiFramePictures *pics, int *final, void *stream) {
    if (!ctx || !f || !pics || !final) return -EINVAL;
    const auto t0 = std::chrono::steady_clock::now();
    StageEvents tev(ctx->tm_on);
    int64_t bytes = 0;
    const int r = frame_run(ctx, f, pics, final, stream, tev, &bytes);
    if (r == 0 && ctx->tm_on) {
        bool all = true;
        for (hipEvent_t e : tev.ev) all = all && e;
        if (all) {
            for (hipEvent_t &e : tev.ev) {
                ctx->tm_ev.push_back(e);
                e = nullptr;
            }
            ctx->tm_frames++;
            ctx->tm_bytes += bytes;
            ctx->tm_host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
    }
    return r;
}

int mi_ctx_set_timing(MiCtx *ctx, int on) {
    if (!ctx) return -EINVAL;
    ctx->tm_clear();
    ctx->tm_on = on != 0;
    return 0;
}

int mi_ctx_timing(MiCtx *ctx, MiFrameTiming *out) {
    if (!ctx || !out) return -EINVAL;
    memset(out, 0, sizeof(*out));
    double st[4] = {0, 0, 0, 0};
    for (size_t i = 0; i + 5 <= ctx->tm_ev.size(); i += 5) {
        if (hipEventSynchronize(ctx->tm_ev[i + 4]) != hipSuccess) {
            ctx->tm_clear();
            return -EIO;
        }
        for (int k = 0; k < 4; k++) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, ctx->tm_ev[i + k], ctx->tm_ev[i + k + 1]) == hipSuccess) st[k] += ms;
        }
    }
    out->frames = ctx->tm_frames;
    out->host_ms = ctx->tm_host_ms;
    out->upload_ms = st[0];
    out->inter_ms = st[1];
    out->intra_ms = st[2];
    out->filter_ms = st[3];
    out->upload_bytes = ctx->tm_bytes;
    out->stage_ms = ctx->tm_stage_ms;
    out->strips_ms = ctx->tm_strips_ms;
    const bool on = ctx->tm_on;
    ctx->tm_clear();
    ctx->tm_on = on;
    return 0;
}

}  // extern "C"

namespace {

// The host side of one frame's execution (no device calls): the intra blocks in the
// persistent queue's order (dependency levels within XCD strips) with their dependency lists
// in queue positions, the inter units bucketed by shape class, the inter residuals grouped by
// (tx size, picture band). scaled[k]: reference k is scaled (OBMC laps then take mi_mc_scaled).
struct FramePlan {
    mi_plan::IntraQueue iq;          // the intra queue, when the front-end did not provide one
    std::vector<MiMcBlock> mc_b, lap_b[2], lap_s[2];
    uint32_t mc_cs[2 * MI_MC_NCLASS + 1], lap_cs[2][2 * MI_MC_NCLASS + 1];
    std::vector<MiTxBlock> itx_b;
    uint32_t itx_bs[MI_N_RECT_TX_SIZES][MI_ITX_BANDS + 1];
    uint32_t itx_dc[MI_N_RECT_TX_SIZES][MI_ITX_BANDS];   // end of each band's DC-only run
    // CDEF and loop-restoration workgroup orders, costliest first (mi_cdef_tile_order /
    // mi_lr_tile_order)
    std::vector<int32_t> cdef_order, lr_order;
    // the inter units run as one grid (mi_mc_frame_sync): chroma MASK units of SEG blocks
    // flagged MI_MC_AFTER_SEG; false when a mask offset or SEG size does not allow it
    bool mc_sync = false;
    double strips_ms = 0;
};

// Flag the chroma MASK units whose mask a luma SEG unit of the same list writes
// (MI_MC_AFTER_SEG) and say whether the list can run as one grid with the in-launch hand-off
// (mi_mc_frame_sync: SEG and MASK mask offsets multiples of 16, SEG units at least 8x8)
bool mark_mc_sync(std::vector<MiMcBlock> &u) {
    std::vector<uint32_t> seg;
    for (const MiMcBlock &b : u) {
        if (b.ref[1] < 0 || (b.comp != MI_MC_SEG && b.comp != MI_MC_MASK)) continue;
        if (b.mask_off & 15) return false;
        if (b.comp == MI_MC_SEG) {
            if (b.plane || b.w < 8 || b.h < 8) return false;
            seg.push_back(b.mask_off);
        }
    }
    std::sort(seg.begin(), seg.end());
    for (MiMcBlock &b : u) {
        b.param &= (uint8_t)~MI_MC_AFTER_SEG;
        if (b.plane && b.ref[1] >= 0 && b.comp == MI_MC_MASK && std::binary_search(seg.begin(), seg.end(), b.mask_off))
            b.param |= (uint8_t)MI_MC_AFTER_SEG;
    }
    return true;
}

void plan_frame(const MiDecFrame *f, const bool scaled[7], FramePlan &pl) {
    // (a plan is reused frame after frame: every list that is appended to starts empty)
    pl.lap_s[0].clear();
    pl.lap_s[1].clear();
    pl.strips_ms = 0;
    if (!f->q_intra) {
        // MI_IR_TIMELINE=<file> (diagnostics): the launch's per-unit stamps, blocks and dependencies
        static const char *tl_path = getenv("MI_IR_TIMELINE");
        pl.iq.timeline = tl_path != nullptr;
        mi_plan::plan_intra(f, pl.iq, [](int n, int min_n, auto &&fn) { return parallel_ranges(n, min_n, fn); });
        pl.strips_ms = pl.iq.ms;
    }
    std::vector<MiMcBlock> &mc_b = pl.mc_b, (&lap_b)[2] = pl.lap_b, (&lap_s)[2] = pl.lap_s;
    uint32_t *mc_cs = pl.mc_cs;
    uint32_t (&lap_cs)[2][2 * MI_MC_NCLASS + 1] = pl.lap_cs;
    bucket_mc(f->mc, f->n_mc, mc_b, mc_cs);
    pl.mc_sync = mark_mc_sync(mc_b);
    for (int k = 0; k < 2; k++) {
        const MiMcBlock *u = k ? f->obmc_v : f->obmc_h;
        std::vector<MiMcBlock> plain;
        for (int i = 0; i < (k ? f->n_obmc_v : f->n_obmc_h); i++) (scaled[u[i].ref[0]] ? lap_s[k] : plain).push_back(u[i]);
        bucket_mc(plain.data(), (int)plain.size(), lap_b[k], lap_cs[k]);
    }
    // the post-filters' workgroups, longest first, so that a launch does not end on a tail of
    // long ones (LR 35.8 -> 31.1 us on the 4K10 bench frame)
    pl.cdef_order.clear();
    pl.lr_order.clear();
    if (f->cdef_on) {
        MiCdef cd;
        memset(&cd, 0, sizeof(cd));
        cd.sb128w = f->sb128w;
        memcpy(cd.y_strength, f->cdef_y, 8);
        memcpy(cd.uv_strength, f->cdef_uv, 8);
        pl.cdef_order.resize((size_t)((f->w + 63) / 64 + 1) * ((f->h + 63) / 64 + 1));
        const int n = mi_cdef_tile_order(f->lf_masks, f->w, f->h, f->layout, &cd, pl.cdef_order.data(),
                                         (int)pl.cdef_order.size());
        pl.cdef_order.resize(n > 0 ? n : 0);
    }
    if (f->restore_planes) {
        MiLr lr;
        memset(&lr, 0, sizeof(lr));
        lr.sb128w = f->lr_sb128w;
        lr.restore_planes = f->restore_planes;
        lr.unit_size_log2[0] = f->lr_unit_size[0];
        lr.unit_size_log2[1] = f->lr_unit_size[1];
        pl.lr_order.resize((size_t)3 * ((f->h + 63) / 64 + 1) * ((f->up_w + 31) / 32 + 1));
        const int n = mi_lr_tile_order(f->lr_mask, f->up_w, f->h, f->layout, &lr, pl.lr_order.data(),
                                       (int)pl.lr_order.size());
        pl.lr_order.resize(n > 0 ? n : 0);
    }
    // residuals grouped by (tx size, picture band) for mi_itx_frame_runs, each group's DC-only
    // blocks (DCT_DCT, eob < 1) first: a counting sort keeping decode order inside a group
    std::vector<MiTxBlock> &itx_b = pl.itx_b;
    itx_b.resize(f->n_inter_tx);
    uint32_t (&itx_bs)[MI_N_RECT_TX_SIZES][MI_ITX_BANDS + 1] = pl.itx_bs;
    uint32_t (&itx_dc)[MI_N_RECT_TX_SIZES][MI_ITX_BANDS] = pl.itx_dc;
    memset(itx_bs, 0, sizeof(itx_bs));
    {
        constexpr int NF = MI_ITX_BANDS;                           // bands per plane
        constexpr int NK = MI_N_RECT_TX_SIZES * NF * 2;
        const int ah = (f->h + 127) & ~127, ssv = f->layout == 1;
        auto key = [&](const MiTxBlock &b) {
            const int ph = b.plane ? ah >> ssv : ah;
            const int q = (int)((int64_t)b.y * NF / ph);
            const int dc = b.txtp == 0 && b.eob < 1;
            return ((int)b.tx * NF + (q < NF - 1 ? q : NF - 1)) * 2 + (dc ? 0 : 1);
        };
        std::vector<uint32_t> start(NK + 1, 0);
        for (int i = 0; i < f->n_inter_tx; i++) start[key(f->inter_tx[i]) + 1]++;
        for (int k = 0; k < NK; k++) start[k + 1] += start[k];
        for (int t = 0; t < MI_N_RECT_TX_SIZES; t++) {
            for (int q = 0; q <= MI_ITX_BANDS; q++) itx_bs[t][q] = start[(t * NF + q) * 2];
            for (int q = 0; q < MI_ITX_BANDS; q++) itx_dc[t][q] = start[(t * NF + q) * 2 + 1];
        }
        for (int i = 0; i < f->n_inter_tx; i++) itx_b[start[key(f->inter_tx[i])]++] = f->inter_tx[i];
    }
}

int frame_run(MiCtx *ctx, const MiDecFrame *f, const MiFramePictures *pics, int *final, void *stream,
              StageEvents &tev, int64_t *bytes) {
    static const bool fx_prof = getenv("MI_FX_PROFILE") != nullptr;
    const auto t_val = std::chrono::steady_clock::now();
    int r = validate(f, pics);
    if (r) return ctx->last_error = r;
    if (fx_prof)
        fprintf(stderr, "frame_run validate %.3f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_val).count());
    hipStream_t s = (hipStream_t)stream;
    const size_t cb = f->bpc == 8 ? 2 : 4, pb = f->bpc == 8 ? 1 : 2;
    const int n = f->n_intra;
    using clk = std::chrono::steady_clock;
    // inter frames: the references (OBMC laps are split by whether their reference is scaled)
    bool scaled[7] = {};
    if (inter_present(f) || f->n_inter_tx) {
        if ((r = validate_refs(f, pics, scaled)) || (r = validate_inter(f, pics, scaled))) return ctx->last_error = r;
    }
    static thread_local FramePlan pl_tl;   // vectors keep their capacity across frames
    FramePlan &pl = pl_tl;
    plan_frame(f, scaled, pl);
    if (ctx->tm_on) ctx->tm_strips_ms += pl.strips_ms;
    // the intra queue: the front-end's (MiDecFrame.q_*, planned in its frame job) or this plan's
    const bool inter = mi_plan::inter_present(f) || f->n_inter_tx;
    const bool have_q = f->q_intra != nullptr;
    const bool granules = have_q ? f->q_granules != 0 : pl.iq.granules;
    const MiIntraBlock *q_blocks = have_q ? f->q_intra : pl.iq.blocks.data();
    const MiTxBlock *q_tx = have_q ? f->q_intra_tx : pl.iq.tx.data();
    const int32_t *q_ds = have_q ? f->q_dep_start : pl.iq.dep_start.data();
    const int32_t *q_deps = have_q ? f->q_deps : pl.iq.deps.data();
    const size_t n_qdeps = have_q ? (size_t)std::max(1, f->q_n_deps) : pl.iq.deps.size();
    const int32_t *q_ss = have_q ? f->q_strip_start : pl.iq.strip_start.data();
    const int n_qss = have_q ? (f->q_nstrips > 1 ? f->q_nstrips + 1 : 0) : (int)pl.iq.strip_start.size();
    std::vector<int32_t> &tl_ds = pl.iq.tl_ds, &tl_deps = pl.iq.tl_deps, &tl_strip = pl.iq.tl_strip;
    std::vector<MiMcBlock> &mc_b = pl.mc_b, (&lap_b)[2] = pl.lap_b, (&lap_s)[2] = pl.lap_s;
    uint32_t *mc_cs = pl.mc_cs;
    uint32_t (&lap_cs)[2][2 * MI_MC_NCLASS + 1] = pl.lap_cs;
    std::vector<MiTxBlock> &itx_b = pl.itx_b;
    uint32_t (&itx_bs)[MI_N_RECT_TX_SIZES][MI_ITX_BANDS + 1] = pl.itx_bs;
    static const char *tl_path = getenv("MI_IR_TIMELINE");
    const int sb128h = (f->h + 127) >> 7;
    std::vector<Section> secs = {
        { q_blocks, (size_t)n * sizeof(MiIntraBlock), 0 },
        { q_tx, (size_t)n * sizeof(MiTxBlock), 0 },
        { q_ds, (size_t)(n + 1) * 4, 0 },
        { q_deps, n_qdeps * 4, 0 },
        { f->coef, f->ncoef * cb, 0 },
        { f->idx, f->nidx, 0 },
        { f->pal, f->npal * pb, 0 },
        { f->lf_level, f->filter_y ? (size_t)f->b4_stride * sb128h * 32 * 4 : 0, 0 },
        { f->lf_masks, (f->filter_y || f->cdef_on) ? (size_t)f->sb128w * sb128h * sizeof(MiAv1Filter) : 0, 0 },
        { f->lr_mask, f->restore_planes ? (size_t)f->lr_sb128w * sb128h * sizeof(MiAv1Restoration) : 0, 0 },
        { mc_b.data(), mc_b.size() * sizeof(MiMcBlock), 0 },                       // 10
        { lap_b[0].data(), lap_b[0].size() * sizeof(MiMcBlock), 0 },               // 11
        { lap_s[0].data(), lap_s[0].size() * sizeof(MiMcBlock), 0 },               // 12
        { lap_b[1].data(), lap_b[1].size() * sizeof(MiMcBlock), 0 },               // 13
        { lap_s[1].data(), lap_s[1].size() * sizeof(MiMcBlock), 0 },               // 14
        { f->warp, (size_t)f->n_warp * sizeof(MiWarpBlock), 0 },                  // 15
        { f->scaled, (size_t)f->n_scaled * sizeof(MiMcBlock), 0 },                // 16
        { f->combine_y, (size_t)f->n_combine_y * sizeof(MiMcCombine), 0 },        // 17
        { f->combine_uv, (size_t)f->n_combine_uv * sizeof(MiMcCombine), 0 },      // 18
        { f->masks, f->nmasks, 0 },                                                 // 19
        { itx_b.data(), itx_b.size() * sizeof(MiTxBlock), 0 },                     // 20
        { nullptr, f->ntmp * 2, 0 },                                                // 21: tmp arena
        { pl.cdef_order.data(), pl.cdef_order.size() * 4, 0 },                     // 22
        { pl.lr_order.data(), pl.lr_order.size() * 4, 0 },                         // 23
    };
    const auto t_st = clk::now();
    if ((r = stage_upload(ctx, secs, s, tev.ev[0], bytes))) return ctx->last_error = r;
    if (ctx->tm_on) ctx->tm_stage_ms += std::chrono::duration<double, std::milli>(clk::now() - t_st).count();
    if (fx_prof) fprintf(stderr, "frame_run stage %.3f ms\n", std::chrono::duration<double, std::milli>(clk::now() - t_st).count());
    tev.mark(1, s);
    uint8_t *dev = ctx->fx_dev;
    auto D = [&](int i) -> void * { return secs[i].bytes ? dev + secs[i].off : nullptr; };

    // The coefficient arena D(4) is this frame's staged copy of the front-end's arena (which
    // the front-end zeroes on the host, as itxfm_add's contract asks of the caller's buffer):
    // no block reads it twice, so the device kernels leave it as it is (MI_ITX_KEEP_COEFS)
    // instead of spending a write pass on zeroing a copy nobody reads again.
    // 0. inter prediction (recon_b_inter's mc / warp_affine / compound / obmc calls over the
    // whole frame: they read reference pictures only), then the inter residuals
    if (inter) {
        MiPicture cur = pics->recon;
        cur.w = f->w;
        MiPicture same[7], any[7];
        for (int k = 0; k < 7; k++) {
            // references the units never read (absent, or scaled for the same-size paths) are
            // stood in for by the current picture: the entry points check every slot's geometry
            const bool have = pics->refs[k].data[0] != nullptr;
            same[k] = have && !scaled[k] ? pics->refs[k] : cur;
            any[k] = have ? pics->refs[k] : cur;
        }
        uint8_t *masks = (uint8_t *)D(19);
        int16_t *tmp = (int16_t *)D(21);
        // luma and chroma units in one grid when the chroma units that read a SEG mask can
        // wait for it inside the launch (4K10 bench frame: 56.9 against 65.3 us)
        if (f->n_mc && (r = pl.mc_sync ? mi_mc_frame_sync(ctx, &cur, same, 7, (const MiMcBlock *)D(10), mc_cs, masks,
                                                          f->nmasks, tmp, stream)
                                       : mi_mc_frame(ctx, &cur, same, 7, (const MiMcBlock *)D(10), mc_cs, masks, tmp, stream)))
            return r;
        if (f->n_warp && (r = mi_mc_warp(ctx, &cur, same, 7, (const MiWarpBlock *)D(15), f->n_warp, tmp, stream)))
            return r;
        if (f->n_scaled && (r = mi_mc_scaled(ctx, &cur, any, 7, (const MiMcBlock *)D(16), f->n_scaled, tmp, stream)))
            return r;
        // compounds with a warped / scaled side: luma, then chroma (a chroma MASK unit reads the
        // mask its luma SEG unit wrote)
        if (f->n_combine_y &&
            (r = mi_mc_combine(ctx, &cur, (const MiMcCombine *)D(17), f->n_combine_y, tmp, masks, stream)))
            return r;
        if (f->n_combine_uv &&
            (r = mi_mc_combine(ctx, &cur, (const MiMcCombine *)D(18), f->n_combine_uv, tmp, masks, stream)))
            return r;
        // obmc(): every above lap, then every left lap (recon.rs:2205-2309)
        for (int k = 0; k < 2; k++) {
            if (!lap_b[k].empty() &&
                (r = mi_mc_frame(ctx, &cur, same, 7, (const MiMcBlock *)D(11 + 2 * k), lap_cs[k], masks, tmp, stream)))
                return r;
            if (!lap_s[k].empty() && (r = mi_mc_scaled(ctx, &cur, any, 7, (const MiMcBlock *)D(12 + 2 * k),
                                                       (int)lap_s[k].size(), tmp, stream)))
                return r;
        }
        // DC-only residuals deferred into the deblocking pass (MI_ITX_DC_DEFER) when nothing
        // reads the reconstruction itself: no intra block predicts from it, and deblocking runs
        // out of place (its output is what CDEF, LR and the reference picture read)
        const bool dc_defer = n == 0 && f->filter_y && pics->recon.data[0] != pics->deblocked.data[0];
        if (f->n_inter_tx &&
            (r = mi_itx_frame_runs(ctx, &cur, (const MiTxBlock *)D(20), itx_bs, pl.itx_dc, D(4),
                                   MI_ITX_KEEP_COEFS | (dc_defer ? MI_ITX_DC_DEFER : 0u), stream)))
            return r;
    }

    tev.mark(2, s);
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
        if ((r = mi_internal::intra_recon(ctx, &fr, 1, n_qss ? q_ss : nullptr, n_qss ? n_qss - 1 : 0,
                                          MI_ITX_KEEP_COEFS, stream, granules)))
            return r;
        if (tl_path && !have_q && n > 1000) {
            std::vector<unsigned long long> t((size_t)n * 16);
            if (hipStreamSynchronize(s) == hipSuccess &&
                hipMemcpy(t.data(), ctx->ir_tl, t.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                if (FILE *fp = fopen(tl_path, "ab")) {
                    const int32_t hdr[4] = { n, (int32_t)tl_deps.size(), (int32_t)tl_strip.size(), granules };
                    fwrite(hdr, 4, 4, fp);
                    fwrite(t.data(), 8, t.size(), fp);
                    fwrite(q_blocks, sizeof(MiIntraBlock), n, fp);
                    fwrite(tl_ds.data(), 4, tl_ds.size(), fp);
                    fwrite(tl_deps.data(), 4, tl_deps.size(), fp);
                    fwrite(tl_strip.data(), 4, tl_strip.size(), fp);
                    fclose(fp);
                }
            }
        }
    }
    tev.mark(3, s);
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
        // (adds the DC runs an inter frame's residual call deferred, if any)
        if ((r = mi_deblock_frame_dc(ctx, cur, &cp[1], &lf, stream))) return r;
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
        cd.order = (const int32_t *)D(22);
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
        lr.order = (const int32_t *)D(23);
        int out = 3;
        if (f->up_w != f->w)
            for (int k = 0; k < 4; k++)
                if (k != idx && k != dbl_idx) { out = k; break; }
        if ((r = mi_lr_frame(ctx, cur, deblocked, slot[out], &lr, stream))) return r;
        idx = out;
    }
    tev.mark(4, s);
    *final = idx;
    return 0;
}

}  // namespace

extern "C" {

int mi_frame_validate(const MiDecFrame *f, const MiFramePictures *pics, const char **why) {
    if (!f || !pics) return -EINVAL;
    g_why = nullptr;
    int r = validate(f, pics);
    bool scaled[7] = {};
    if (!r && (inter_present(f) || f->n_inter_tx)) {
        r = validate_refs(f, pics, scaled);
        if (!r) r = validate_inter(f, pics, scaled);
    }
    if (why) *why = r ? (g_why ? g_why : "?") : nullptr;
    return r;
}

double mi_frame_plan_ms(const MiDecFrame *f, int reps) {
    if (!f || reps < 1) return -1.0;
    // the work list's own checks (mi_frame_run's, without the pictures): plan_frame indexes the
    // owner map, levels and CSR arrays by the list's coordinates and dependency indices
    if (validate(f, nullptr)) return -1.0;
    bool scaled[7] = {};
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    static thread_local FramePlan pl_tl;   // as mi_frame_run keeps it: reused frame after frame
    FramePlan &pl = pl_tl;
    for (int i = 0; i < reps; i++) plan_frame(f, scaled, pl);
    return std::chrono::duration<double, std::milli>(clk::now() - t0).count() / reps;
}

int mi_frame_end(MiCtx *ctx, void *stream) {
    if (!ctx) return -EINVAL;
    const int r = mi_ctx_device_status(ctx, stream);
    // a kernel rejected descriptors: -EINVAL; a stalled or untaken block: -EIO
    return r ? (ctx->last_error = r == -EINVAL ? -EINVAL : -EIO) : 0;
}

}  // extern "C"
