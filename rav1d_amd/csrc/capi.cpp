// capi.cpp — the C-ABI of include/mi_av1dsp.h: contexts, the batched per-frame entry points
// and the table-compatible per-call entry points.
//
// The per-call entry points keep the reference's contract (caller owns buffers, callee zeroes
// the consumed coefficients, src/itx.rs:152-158) and accept host or device pointers; they run
// a one-block launch synchronously on a private stream of device 0.
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <errno.h>
#include <mutex>
#include <string.h>
#include <string>
#include <vector>
#include "common.h"
#include "ctx.h"


namespace {

int fail(MiCtx *c, int e) {
    if (c) c->last_error = e;
    return e;
}

bool is_device_ptr(const void *p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

// Private state for the synchronous per-call entry points.
struct CallState {
    std::mutex mu;
    bool ready = false;
    int err = 0;
    hipStream_t stream = nullptr;
    uint8_t *scratch = nullptr;     // pixels / coefficients / descriptors
    size_t scratch_bytes = 0;
    int init() {
        if (ready) return err;
        ready = true;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return err = -ENODEV;
        if (hipSetDevice(0) != hipSuccess) return err = -ENODEV;
        if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return err = -EIO;
        scratch_bytes = 1 << 20;
        if (hipMalloc(&scratch, scratch_bytes) != hipSuccess) return err = -ENOMEM;
        return err = 0;
    }
    int reserve(size_t n) {   // grow the scratch (only ever grows; callers hold mu)
        if (n <= scratch_bytes) return 0;
        if (hipStreamSynchronize(stream) != hipSuccess) return -EIO;
        (void)hipFree(scratch);
        scratch = nullptr;
        scratch_bytes = 0;
        if (hipMalloc(&scratch, n) != hipSuccess) {
            if (hipMalloc(&scratch, 1 << 20) == hipSuccess) scratch_bytes = 1 << 20;
            return -ENOMEM;
        }
        scratch_bytes = n;
        return 0;
    }
};
CallState g_call;

// The context's device words ([0..63] queue heads, [64] dependency-wait give-up / untaken
// blocks, [65] rejected descriptors, [72..79] XCD worker ranks), allocated zeroed on first use.
// Zeroed on the context's own stream: a null-stream hipMemset is not ordered with a
// non-blocking stream and may land after (or during) the first kernel that uses the words --
// with two contexts whose streams overlap, it reset the queue heads of a running persistent
// intra launch, which then re-ran blocks whose coefficients it had already consumed.
int ctx_words(MiCtx *c, hipStream_t s) {
    if (c->ir_words) return 0;
    if (hipMalloc(&c->ir_words, 128 * sizeof(int)) != hipSuccess) return -ENOMEM;
    if (hipMemsetAsync(c->ir_words, 0, 128 * sizeof(int), s) != hipSuccess) return -EIO;
    return 0;
}

bool same_geometry(const MiPicture *a, const MiPicture *b) {
    return a->bpc == b->bpc && a->w == b->w && a->h == b->h && a->layout == b->layout &&
           a->stride[0] == b->stride[0] && a->stride[1] == b->stride[1];
}

} // namespace

extern "C" {

const char *mi_version(void) { return "rav1d_amd mi_av1dsp 0.1 (gfx950)"; }

int mi_ctx_create(int device, MiCtx **out) {
    if (!out) return -EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return -ENODEV;
    MiCtx *c = new (std::nothrow) MiCtx;
    if (!c) return -ENOMEM;
    c->device = device;
    *out = c;
    return 0;
}

void mi_ctx_destroy(MiCtx *ctx) { delete ctx; }

int mi_ctx_last_error(const MiCtx *ctx) { return ctx ? ctx->last_error : -EINVAL; }

static int itx_frame(MiCtx *ctx, const MiPicture *pic, const MiTxBlock *blocks,
                     const uint32_t *size_start, const uint32_t *band_start, void *coef, unsigned flags,
                     void *stream, const uint32_t *dc_end = nullptr);

int mi_itx_frame(MiCtx *ctx, const MiPicture *pic, const MiTxBlock *blocks,
                 const uint32_t size_start[MI_N_RECT_TX_SIZES + 1], void *coef, unsigned flags,
                 void *stream) {
    return itx_frame(ctx, pic, blocks, size_start, nullptr, coef, flags, stream);
}

int mi_itx_frame_banded(MiCtx *ctx, const MiPicture *pic, const MiTxBlock *blocks,
                        const uint32_t band_start[MI_N_RECT_TX_SIZES][MI_ITX_BANDS + 1], void *coef,
                        unsigned flags, void *stream) {
    if (!band_start) return fail(ctx, -EINVAL);
    // bands of one size are consecutive ranges and the sizes follow each other
    uint32_t ss[MI_N_RECT_TX_SIZES + 1];
    for (int t = 0; t < MI_N_RECT_TX_SIZES; t++) {
        ss[t] = band_start[t][0];
        if (t && band_start[t][0] != band_start[t - 1][MI_ITX_BANDS]) return fail(ctx, -EINVAL);
        for (int q = 0; q < MI_ITX_BANDS; q++)
            if (band_start[t][q + 1] < band_start[t][q]) return fail(ctx, -EINVAL);
    }
    ss[MI_N_RECT_TX_SIZES] = band_start[MI_N_RECT_TX_SIZES - 1][MI_ITX_BANDS];
    return itx_frame(ctx, pic, blocks, ss, &band_start[0][0], coef, flags, stream);
}

int mi_itx_frame_runs(MiCtx *ctx, const MiPicture *pic, const MiTxBlock *blocks,
                      const uint32_t band_start[MI_N_RECT_TX_SIZES][MI_ITX_BANDS + 1],
                      const uint32_t dc_end[MI_N_RECT_TX_SIZES][MI_ITX_BANDS], void *coef, unsigned flags,
                      void *stream) {
    if (!band_start || !dc_end) return fail(ctx, -EINVAL);
    uint32_t ss[MI_N_RECT_TX_SIZES + 1];
    for (int t = 0; t < MI_N_RECT_TX_SIZES; t++) {
        ss[t] = band_start[t][0];
        if (t && band_start[t][0] != band_start[t - 1][MI_ITX_BANDS]) return fail(ctx, -EINVAL);
        for (int q = 0; q < MI_ITX_BANDS; q++)
            if (band_start[t][q + 1] < band_start[t][q] || dc_end[t][q] < band_start[t][q] ||
                dc_end[t][q] > band_start[t][q + 1])
                return fail(ctx, -EINVAL);
    }
    ss[MI_N_RECT_TX_SIZES] = band_start[MI_N_RECT_TX_SIZES - 1][MI_ITX_BANDS];
    return itx_frame(ctx, pic, blocks, ss, &band_start[0][0], coef, flags, stream, &dc_end[0][0]);
}

static int itx_frame(MiCtx *ctx, const MiPicture *pic, const MiTxBlock *blocks,
                     const uint32_t *size_start, const uint32_t *band_start, void *coef, unsigned flags,
                     void *stream, const uint32_t *dc_end) {
    if (!ctx || !pic || !size_start) return fail(ctx, -EINVAL);
    if (pic->bpc != 8 && pic->bpc != 10 && pic->bpc != 12) return fail(ctx, -EINVAL);
    mi::ItxArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) {
        a.plane[p] = (uint8_t *)pic->data[p];
        a.stride[p] = pic->stride[p ? 1 : 0];
    }
    a.blocks = blocks;
    a.coef = (uint8_t *)coef;
    a.bdmax = (1 << pic->bpc) - 1;
    a.zero_coefs = (flags & MI_ITX_KEEP_COEFS) ? 0 : 1;
    if (flags & ~(MI_ITX_KEEP_COEFS | MI_ITX_DC_DEFER)) return fail(ctx, -EINVAL);
    if ((flags & MI_ITX_DC_DEFER) && !dc_end) return fail(ctx, -EINVAL);
    {
        const int sh = pic->layout == 1 || pic->layout == 2, sv = pic->layout == 1;
        const int aw = (pic->w + 127) & ~127, ah = (pic->h + 127) & ~127;
        for (int p = 0; p < (pic->layout ? 3 : 1); p++) {
            a.pw[p] = p ? aw >> sh : aw;
            a.ph[p] = p ? ah >> sv : ah;
        }
    }
    if (int e = ctx_words(ctx, (hipStream_t)stream)) return fail(ctx, e);
    a.err = ctx->ir_words + 65;
    for (int k = 0; k < MI_N_RECT_TX_SIZES; k++)
        if (size_start[k + 1] < size_start[k]) return fail(ctx, -EINVAL);
    const int wg = mi::itx_fill_schedule(a, size_start, band_start, dc_end);
    if (flags & MI_ITX_DC_DEFER) {
        // the DC runs go to the context's DC map for the next mi_deblock_frame_dc; under stream
        // capture they are added to the pixels as without the flag (a tag fixed in a graph would
        // let a replay match the map entries of the previous replay)
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing((hipStream_t)stream, &cap) != hipSuccess) return fail(ctx, -EIO);
        ctx->dc_pending = 0;
        if (cap == hipStreamCaptureStatusNone) {
            const mi::DcMapGeom g = mi::dc_map_geom(pic->w, pic->h, pic->layout);
            if (g.entries > ctx->dc_map_n) {
                if (ctx->dc_map) (void)hipFree(ctx->dc_map);
                ctx->dc_map = nullptr;
                ctx->dc_map_n = 0;
                if (hipMalloc(&ctx->dc_map, g.entries * 4) != hipSuccess) return fail(ctx, -ENOMEM);
                if (hipMemsetAsync(ctx->dc_map, 0, g.entries * 4, (hipStream_t)stream) != hipSuccess) return fail(ctx, -EIO);
                ctx->dc_map_n = g.entries;
                ctx->dc_tag = 0;
            }
            if (++ctx->dc_tag > 0xffffu) {   // the 16-bit tag wraps: no stale entry may match
                if (hipMemsetAsync(ctx->dc_map, 0, ctx->dc_map_n * 4, (hipStream_t)stream) != hipSuccess) return fail(ctx, -EIO);
                ctx->dc_tag = 1;
            }
            a.dc_map = ctx->dc_map;
            for (int p = 0; p < 3; p++) {
                a.dc_off[p] = g.off[p];
                a.dc_stride[p] = g.stride[p];
            }
            a.dc_tag = ctx->dc_tag;
            ctx->dc_pending = ctx->dc_tag;
            ctx->dc_w = pic->w;
            ctx->dc_h = pic->h;
            ctx->dc_layout = pic->layout;
        }
    }
    if (wg == 0) return 0;
    if (!blocks || !coef) return fail(ctx, -EINVAL);
    // One launch (itx.hip): the large sizes' workgroups first, the small ones fill in around
    // them. A side stream for the large sizes (event fork/join) measured slower (4K10 itx
    // 56 -> 74 us) than the cross-queue dependency saves.
    hipStream_t s = (hipStream_t)stream;
    const int r = mi::launch_itx_frame(a, wg, pic->bpc, s);
    return r ? fail(ctx, -EIO) : 0;
}

}  // extern "C"

namespace {
// McArgs from the current picture and the references (planes, strides, clamp bounds, bit
// depth). same_size: the references must share cur's geometry (non-scaled MC, warp).
int fill_mc_args(mi::McArgs &a, const MiPicture *cur, const MiPicture *refs, int nrefs, bool same_size) {
    memset(&a, 0, sizeof(a));
    if (cur->bpc != 8 && cur->bpc != 10 && cur->bpc != 12) return -EINVAL;
    if (nrefs < 0 || nrefs > 7 || (nrefs && !refs)) return -EINVAL;
    const int ss_hor = cur->layout == 1 || cur->layout == 2, ss_ver = cur->layout == 1;
    for (int p = 0; p < 3; p++) a.dst[p] = (uint8_t *)cur->data[p];
    a.dst_stride[0] = cur->stride[0];
    a.dst_stride[1] = cur->stride[1];
    for (int r = 0; r < nrefs; r++) {
        if (same_size ? !same_geometry(cur, &refs[r])
                      : refs[r].bpc != cur->bpc || refs[r].layout != cur->layout || refs[r].w <= 0 || refs[r].h <= 0)
            return -EINVAL;
        for (int p = 0; p < 3; p++) {
            const int sh = p ? ss_hor : 0, sv = p ? ss_ver : 0;
            a.ref[r][p] = (const uint8_t *)refs[r].data[p];
            a.ref_w[r][p] = (refs[r].w + sh) >> sh;
            a.ref_h[r][p] = (refs[r].h + sv) >> sv;
        }
        a.ref_stride[r][0] = refs[r].stride[0];
        a.ref_stride[r][1] = refs[r].stride[1];
        // mc_kernel forms reference row offsets with 24-bit multiplies
        for (int k = 0; k < 2; k++)
            if (refs[r].stride[k] <= 0 || refs[r].stride[k] >= (1 << 24)) return -EINVAL;
    }
    a.nrefs = nrefs;
    a.bpc = cur->bpc;
    a.ib = cur->bpc == 8 ? 4 : 14 - cur->bpc;
    a.bias = cur->bpc == 8 ? 0 : 8192;
    a.bdmax = (1 << cur->bpc) - 1;
    a.layout = cur->layout;
    a.seg_ss_hor = cur->layout ? ss_hor : 0;   // w_mask[chr_layout_idx] (recon_tmpl.c:1868)
    a.seg_ss_ver = cur->layout ? ss_ver : 0;
    return 0;
}
}  // namespace

extern "C" {

int mi_mc_frame(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
                const MiMcBlock *blocks, const uint32_t class_start[2 * MI_MC_NCLASS + 1], uint8_t *masks,
                int16_t *tmp, void *stream) {
    return mi_mc_frame_ex(ctx, cur, refs, nrefs, blocks, class_start, masks, tmp, 0, stream);
}

int mi_mc_frame_ex(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
                   const MiMcBlock *blocks, const uint32_t class_start[2 * MI_MC_NCLASS + 1], uint8_t *masks,
                   int16_t *tmp, unsigned flags, void *stream) {
    if (!ctx || !cur || !class_start || (flags & ~MI_MC_ONE_GRID)) return fail(ctx, -EINVAL);
    for (int k = 0; k < 2 * MI_MC_NCLASS; k++)
        if (class_start[k] > class_start[k + 1]) return fail(ctx, -EINVAL);
    mi::McArgs a;
    // scaled references take mi_mc_scaled (the reference's mc_scaled path)
    if (int e = fill_mc_args(a, cur, refs, nrefs, true)) return fail(ctx, e);
    if (class_start[2 * MI_MC_NCLASS] == class_start[0]) return 0;
    if (!blocks || !nrefs) return fail(ctx, -EINVAL);
    a.blocks = blocks;
    a.masks = masks;
    a.tmp = tmp;
    memcpy(a.class_start, class_start, sizeof(a.class_start));
    const int w0 = mi::mc_plan(a, 0), w1 = mi::mc_plan(a, 1);
    if (w0 < 0 || w1 < 0) return fail(ctx, -EINVAL);
    hipStream_t s = (hipStream_t)stream;
    // luma first: chroma units of SEG blocks read the mask their luma unit writes (one grid
    // only when the caller says no chroma unit of this call does)
    int r;
    if ((flags & MI_MC_ONE_GRID) && w0 && w1) {
        r = mi::launch_mc(a, 2, w0 + w1, s);
    } else {
        r = mi::launch_mc(a, 0, w0, s);
        if (!r) r = mi::launch_mc(a, 1, w1, s);
    }
    return r ? fail(ctx, -EIO) : 0;
}

// The device error word of the MC hand-off: bit 1 a unit's mask offset lies past the flag
// buffer (mask_bytes too small for it: -EINVAL), bit 0 a wait gave up (-ETIMEDOUT). Both
// status entry points report the same code.
static int mc_err_code(int e) { return (e & 2) ? -EINVAL : -ETIMEDOUT; }

int mi_mc_frame_sync(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
                     const MiMcBlock *blocks, const uint32_t class_start[2 * MI_MC_NCLASS + 1], uint8_t *masks,
                     size_t mask_bytes, int16_t *tmp, void *stream) {
    if (!ctx || !cur || !class_start) return fail(ctx, -EINVAL);
    for (int k = 0; k < 2 * MI_MC_NCLASS; k++)
        if (class_start[k] > class_start[k + 1]) return fail(ctx, -EINVAL);
    mi::McArgs a;
    if (int e = fill_mc_args(a, cur, refs, nrefs, true)) return fail(ctx, e);
    if (class_start[2 * MI_MC_NCLASS] == class_start[0]) return 0;
    if (!blocks || !nrefs || (mask_bytes && !masks)) return fail(ctx, -EINVAL);
    a.blocks = blocks;
    a.masks = masks;
    a.tmp = tmp;
    memcpy(a.class_start, class_start, sizeof(a.class_start));
    const int w0 = mi::mc_plan(a, 0), w1 = mi::mc_plan(a, 1);
    if (w0 < 0 || w1 < 0) return fail(ctx, -EINVAL);
    hipStream_t s = (hipStream_t)stream;
    // Under stream capture the epoch below would be frozen into the graph: a replay would find
    // the flags of its previous replay already at "its" epoch and read masks that are still
    // being rewritten. Captured calls therefore take the two launches of mi_mc_frame (luma,
    // then chroma; no flags), which any number of replays orders correctly.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess) return fail(ctx, -EIO);
    if (cap != hipStreamCaptureStatusNone) {
        int r = w0 ? mi::launch_mc(a, 0, w0, s) : 0;
        if (!r && w1) r = mi::launch_mc(a, 1, w1, s);
        return r ? fail(ctx, -EIO) : 0;
    }
    // the tile flags: 32 per 16 mask bytes (a SEG unit has at most 32 tiles), zeroed when
    // allocated and never reset (each call has its own epoch)
    const size_t nf = (mask_bytes / 16 + 1) * 32;
    if (nf > 0xffffffffu) return fail(ctx, -EINVAL);
    if (nf > ctx->mc_flags_n) {
        if (ctx->mc_flags) (void)hipFree(ctx->mc_flags);
        ctx->mc_flags = nullptr;
        ctx->mc_flags_n = 0;
        if (hipMalloc(&ctx->mc_flags, nf * sizeof(uint32_t)) != hipSuccess) return fail(ctx, -ENOMEM);
        if (hipMemsetAsync(ctx->mc_flags, 0, nf * sizeof(uint32_t), s) != hipSuccess) return fail(ctx, -EIO);
        ctx->mc_flags_n = nf;
    }
    if (!ctx->mc_err) {
        if (hipMalloc(&ctx->mc_err, sizeof(int)) != hipSuccess) return fail(ctx, -ENOMEM);
        if (hipMemsetAsync(ctx->mc_err, 0, sizeof(int), s) != hipSuccess) return fail(ctx, -EIO);
    }
    if (++ctx->mc_epoch == 0) ctx->mc_epoch = 1;
    a.seg_flags = ctx->mc_flags;
    a.seg_epoch = ctx->mc_epoch;
    a.seg_nflags = (uint32_t)nf;
    a.err = ctx->mc_err;
    // one grid, the luma group's waves first (see mi_av1dsp.h)
    const int r = w0 && w1 ? mi::launch_mc(a, 2, w0 + w1, s) : mi::launch_mc(a, w0 ? 0 : 1, w0 ? w0 : w1, s);
    return r ? fail(ctx, -EIO) : 0;
}

int mi_mc_sync_status(MiCtx *ctx, void *stream) {
    if (!ctx) return -EINVAL;
    if (!ctx->mc_err) return 0;
    int e = 0;
    if (hipMemcpyAsync(&e, ctx->mc_err, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
        return fail(ctx, -EIO);
    if (e && hipMemsetAsync(ctx->mc_err, 0, sizeof(int), (hipStream_t)stream) != hipSuccess) return fail(ctx, -EIO);
    return e ? fail(ctx, mc_err_code(e)) : 0;
}

int mi_mc_scaled(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
                 const MiMcBlock *blocks, int n, int16_t *tmp, void *stream) {
    if (!ctx || !cur || n < 0) return fail(ctx, -EINVAL);
    mi::McArgs a;
    if (int e = fill_mc_args(a, cur, refs, nrefs, false)) return fail(ctx, e);
    if (!n) return 0;
    if (!blocks || !nrefs) return fail(ctx, -EINVAL);
    a.tmp = tmp;
    return mi::launch_mc_scaled(a, blocks, n, cur->w, cur->h, (hipStream_t)stream) ? fail(ctx, -EIO) : 0;
}

int mi_mc_warp(MiCtx *ctx, const MiPicture *cur, const MiPicture *refs, int nrefs,
               const MiWarpBlock *blocks, int n, int16_t *tmp, void *stream) {
    if (!ctx || !cur || n < 0) return fail(ctx, -EINVAL);
    mi::McArgs a;
    if (int e = fill_mc_args(a, cur, refs, nrefs, true)) return fail(ctx, e);
    if (!n) return 0;
    if (!blocks || !nrefs) return fail(ctx, -EINVAL);
    a.tmp = tmp;
    return mi::launch_mc_warp(a, blocks, n, (hipStream_t)stream) ? fail(ctx, -EIO) : 0;
}

int mi_mc_combine(MiCtx *ctx, const MiPicture *cur, const MiMcCombine *units, int n,
                  const int16_t *tmp, uint8_t *masks, void *stream) {
    if (!ctx || !cur || n < 0) return fail(ctx, -EINVAL);
    mi::McArgs a;
    if (int e = fill_mc_args(a, cur, nullptr, 0, true)) return fail(ctx, e);
    if (!n) return 0;
    if (!units || !tmp) return fail(ctx, -EINVAL);
    a.tmp = const_cast<int16_t *>(tmp);
    a.masks = masks;
    return mi::launch_mc_combine(a, units, n, (hipStream_t)stream) ? fail(ctx, -EIO) : 0;
}

int mi_superres_frame(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, void *stream) {
    if (!ctx || !src || !dst) return fail(ctx, -EINVAL);
    if (src->bpc != dst->bpc || src->layout != dst->layout || src->h != dst->h || src->w <= 0 ||
        dst->w < src->w || dst->w > 2 * src->w + 16 || (src->bpc != 8 && src->bpc != 10 && src->bpc != 12))
        return fail(ctx, -EINVAL);
    // scale_fac / get_upscale_x0 (decode.rs:4644-4648, 4776-4778, 4872-4878)
    auto scale_fac = [](int ref_sz, int this_sz) { return ((ref_sz << 14) + (this_sz >> 1)) / this_sz; };
    auto upscale_x0 = [](int in_w, int out_w, int step) {
        const int err = out_w * step - (in_w << 14);
        const int x0 = (-((out_w - in_w) << 13) + (out_w >> 1)) / out_w + 128 - err / 2;
        return x0 & 0x3fff;
    };
    mi::SuperresArgs a;
    memset(&a, 0, sizeof(a));
    const int ss_hor = src->layout == 1 || src->layout == 2, ss_ver = src->layout == 1;
    const int in_cw = (src->w + ss_hor) >> ss_hor, out_cw = (dst->w + ss_hor) >> ss_hor;
    a.step[0] = scale_fac(src->w, dst->w);
    a.step[1] = scale_fac(in_cw, out_cw);
    a.start[0] = upscale_x0(src->w, dst->w, a.step[0]);
    a.start[1] = upscale_x0(in_cw, out_cw, a.step[1]);
    const int bw4 = ((src->w + 7) >> 3) << 1;   // f->bw
    a.nplanes = src->layout ? 3 : 1;
    for (int p = 0; p < a.nplanes; p++) {
        const int sh = p ? ss_hor : 0, sv = p ? ss_ver : 0;
        a.src[p] = (const uint8_t *)src->data[p];
        a.dst[p] = (uint8_t *)dst->data[p];
        a.src_w[p] = (4 * bw4 + sh) >> sh;
        a.dst_w[p] = (dst->w + sh) >> sh;
        a.h[p] = (src->h + sv) >> sv;
        a.chunks = std::max(a.chunks, (a.dst_w[p] + 255) / 256);
    }
    a.src_stride[0] = src->stride[0];
    a.src_stride[1] = src->stride[1];
    a.dst_stride[0] = dst->stride[0];
    a.dst_stride[1] = dst->stride[1];
    a.bpc = src->bpc;
    return mi::launch_superres(a, (hipStream_t)stream) ? fail(ctx, -EIO) : 0;
}

int mi_ipred_blocks(MiCtx *ctx, const MiPicture *pic, const MiIpredBlock *blocks, int n,
                    const void *edges, const int16_t *ac, const uint8_t *idx, void *stream) {
    if (!ctx || !pic || n < 0) return fail(ctx, -EINVAL);
    if (pic->bpc != 8 && pic->bpc != 10 && pic->bpc != 12) return fail(ctx, -EINVAL);
    if (!n) return 0;
    if (!blocks || !edges) return fail(ctx, -EINVAL);
    mi::IpredArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) a.dst[p] = (uint8_t *)pic->data[p];
    a.stride[0] = pic->stride[0];
    a.stride[1] = pic->stride[1];
    a.blocks = blocks;
    a.edges = (const uint8_t *)edges;
    a.ac = ac;
    a.idx = idx;
    a.bpc = pic->bpc;
    a.bdmax = (1 << pic->bpc) - 1;
    return mi::launch_ipred(a, n, (hipStream_t)stream) ? fail(ctx, -EIO) : 0;
}

int mi_intra_blocks(MiCtx *ctx, const MiPicture *pic, const MiIntraBlock *blocks, int n,
                    const int16_t *ac, const uint8_t *idx, const void *pal, void *stream) {
    if (!ctx || !pic || n < 0) return fail(ctx, -EINVAL);
    if (pic->bpc != 8 && pic->bpc != 10 && pic->bpc != 12) return fail(ctx, -EINVAL);
    if (!n) return 0;
    if (!blocks) return fail(ctx, -EINVAL);
    mi::IpredArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) a.dst[p] = (uint8_t *)pic->data[p];
    a.stride[0] = pic->stride[0];
    a.stride[1] = pic->stride[1];
    a.iblocks = blocks;
    a.ac = ac;
    a.idx = idx;
    a.pal = (const uint8_t *)pal;
    a.bpc = pic->bpc;
    a.bdmax = (1 << pic->bpc) - 1;
    return mi::launch_intra(a, n, (hipStream_t)stream) ? fail(ctx, -EIO) : 0;
}

int mi_intra_recon(MiCtx *ctx, const MiIntraFrame *frames, int nframes, unsigned flags, void *stream) {
    return mi_internal::intra_recon(ctx, frames, nframes, nullptr, 1, flags, stream, (flags & MI_IR_EDGE_GRANULES) != 0);
}

int mi_ctx_device_status(MiCtx *ctx, void *stream) {
    if (!ctx) return -EINVAL;
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return fail(ctx, -EIO);
    if (ctx->mc_err) {   // a one-grid MC hand-off wait gave up (mi_mc_frame_sync)
        int e = 0;
        if (hipMemcpy(&e, ctx->mc_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return fail(ctx, -EIO);
        if (e) {
            if (hipMemset(ctx->mc_err, 0, sizeof(int)) != hipSuccess) return fail(ctx, -EIO);
            return fail(ctx, mc_err_code(e));
        }
    }
    if (!ctx->ir_words) return 0;
    int w[66];
    if (hipMemcpy(w, ctx->ir_words, sizeof(w), hipMemcpyDeviceToHost) != hipSuccess) return fail(ctx, -EIO);
    if (w[65]) {   // a kernel rejected (skipped) descriptors
        if (hipMemsetAsync(ctx->ir_words + 65, 0, sizeof(int), (hipStream_t)stream) != hipSuccess ||
            hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
            return fail(ctx, -EIO);
        return fail(ctx, -EINVAL);
    }
    if (getenv("MI_DEBUG"))
        fprintf(stderr, "mi_ctx_device_status: heads %d %d %d %d %d %d %d %d err %d\n", w[0], w[1], w[2], w[3], w[4],
                w[5], w[6], w[7], w[64]);
    // [64]: bit 0 a dependency wait gave up, bit 2 a launch left blocks untaken (a frame
    // whose XCD received no workgroup): set on the device by every launch, sticky until read
    if (w[64]) {
        if (hipMemsetAsync(ctx->ir_words + 64, 0, sizeof(int), (hipStream_t)stream) != hipSuccess ||
            hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
            return fail(ctx, -EIO);
        return fail(ctx, (w[64] & 1) ? -ETIMEDOUT : -EIO);
    }
    return 0;
}

int mi_deblock_frame(MiCtx *ctx, const MiPicture *pic, const MiLoopFilter *lf, void *stream) {
    if (!ctx || !pic || !lf) return fail(ctx, -EINVAL);
    if (pic->bpc != 8 && pic->bpc != 10 && pic->bpc != 12) return fail(ctx, -EINVAL);
    if (!lf->filter_y) return 0;   // deblocking off for the frame (recon.rs:4047-4060)
    if (!lf->level || !lf->masks || lf->sb128w <= 0) return fail(ctx, -EINVAL);
    mi::LfArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) {
        a.plane[p] = (uint8_t *)pic->data[p];
        a.stride[p] = pic->stride[p ? 1 : 0];
    }
    a.level = (const uint32_t *)lf->level;
    a.b4_stride = lf->b4_stride;
    a.masks = lf->masks;
    a.w4 = (pic->w + 3) >> 2;
    a.h4 = (pic->h + 3) >> 2;
    a.sb128w = lf->sb128w;
    a.sb128h = (pic->h + 127) >> 7;
    if (a.sb128w != (pic->w + 127) >> 7 || a.b4_stride < (int64_t)a.sb128w * 32) return fail(ctx, -EINVAL);
    a.ss_hor = pic->layout == 1 || pic->layout == 2;
    a.ss_ver = pic->layout == 1;
    a.bdmax = (1 << pic->bpc) - 1;
    a.bdm8 = pic->bpc - 8;
    a.filter_uv = pic->layout != 0 && lf->filter_uv;
    memcpy(a.lim_e, lf->lim_e, 64);
    memcpy(a.lim_i, lf->lim_i, 64);
    const int nplanes = a.filter_uv ? 3 : 1;
    mi::LfArgs cols = a, rows = a;
    int nc = 0, nr = 0;
    for (int p = 0; p < 3; p++) {
        const int sh = p ? a.ss_hor : 0, sv = p ? a.ss_ver : 0;
        cols.blk_start[p] = nc;
        rows.blk_start[p] = nr;
        if (p >= nplanes) continue;
        cols.units_x[p] = (a.w4 + sh) >> sh;
        cols.rows[p] = (a.sb128h * 128) >> sv;
        nc += ((cols.units_x[p] + 63) / 64) * ((cols.rows[p] + 3) / 4);
        rows.units_x[p] = (a.sb128w * 128) >> sh;
        rows.rows[p] = p ? a.sb128h * (32 >> sv) : a.h4;
        nr += ((rows.units_x[p] + 63) / 64) * ((rows.rows[p] + 3) / 4);
    }
    cols.blk_start[3] = nc;
    rows.blk_start[3] = nr;
    const int r = mi::launch_deblock(cols, rows, pic->bpc, (hipStream_t)stream);
    return r ? fail(ctx, -EIO) : 0;
}

static int deblock_tiles(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, const MiLoopFilter *lf,
                         void *stream, uint32_t dc_tag);

int mi_deblock_frame_to(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, const MiLoopFilter *lf,
                        void *stream) {
    return deblock_tiles(ctx, src, dst, lf, stream, 0);
}

int mi_deblock_frame_dc(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, const MiLoopFilter *lf,
                        void *stream) {
    if (!ctx) return -EINVAL;
    const uint32_t tag = ctx->dc_pending;
    ctx->dc_pending = 0;
    if (tag && (!src || src->w != ctx->dc_w || src->h != ctx->dc_h || src->layout != ctx->dc_layout))
        return fail(ctx, -EINVAL);
    return deblock_tiles(ctx, src, dst, lf, stream, tag);
}

static int deblock_tiles(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, const MiLoopFilter *lf,
                         void *stream, uint32_t dc_tag) {
    if (!ctx || !src || !dst || !lf) return fail(ctx, -EINVAL);
    if (src->bpc != 8 && src->bpc != 10 && src->bpc != 12) return fail(ctx, -EINVAL);
    if (!same_geometry(src, dst)) return fail(ctx, -EINVAL);
    if (src->data[0] == dst->data[0]) {
        if (dc_tag) return fail(ctx, -EINVAL);   // deferred DC needs the out-of-place tiles
        return mi_deblock_frame(ctx, dst, lf, stream);
    }
    const int sh = src->layout == 1 || src->layout == 2, sv = src->layout == 1;
    const int nplanes = src->layout == 0 ? 1 : 3;
    const size_t px = src->bpc == 8 ? 1 : 2;
    const int sb128w = (src->w + 127) >> 7, sb128h = (src->h + 127) >> 7;
    for (int p = 0; p < nplanes; p++)
        if (src->stride[p ? 1 : 0] % 16 || (uintptr_t)src->data[p] % 16 || (uintptr_t)dst->data[p] % 16 ||
            src->stride[p ? 1 : 0] < (ptrdiff_t)(((sb128w * 128) >> (p ? sh : 0)) * px))
            return fail(ctx, -EINVAL);
    const bool edges = lf->filter_y != 0;
    if (!edges && !dc_tag) {   // deblocking off for the frame: the output is the input
        for (int p = 0; p < nplanes; p++) {
            const size_t rows = (size_t)(sb128h * 128) >> (p ? sv : 0);
            const ptrdiff_t s = src->stride[p ? 1 : 0];
            if (hipMemcpyAsync(dst->data[p], src->data[p], rows * s, hipMemcpyDeviceToDevice,
                               (hipStream_t)stream) != hipSuccess)
                return fail(ctx, -EIO);
        }
        return 0;
    }
    if (edges && (!lf->level || !lf->masks || lf->sb128w != sb128w || lf->b4_stride < (int64_t)sb128w * 32))
        return fail(ctx, -EINVAL);
    mi::LfTileArgs a;
    memset(&a, 0, sizeof(a));
    a.level = (const uint32_t *)lf->level;
    a.b4_stride = lf->b4_stride;
    a.masks = lf->masks;
    a.sb128w = sb128w;
    a.w4 = (src->w + 3) >> 2;
    a.h4 = (src->h + 3) >> 2;
    a.ss_hor = sh;
    a.ss_ver = sv;
    a.bdmax = (1 << src->bpc) - 1;
    a.bdm8 = src->bpc - 8;
    const int filter_uv = edges && src->layout != 0 && lf->filter_uv;
    memcpy(a.lim_e, lf->lim_e, 64);
    memcpy(a.lim_i, lf->lim_i, 64);
    int n = 0;
    for (int p = 0; p < 3; p++) {
        a.tile_start[p] = n;
        if (p >= nplanes) continue;
        const int h = p ? sh : 0, v = p ? sv : 0;
        a.src[p] = (const uint8_t *)src->data[p];
        a.dst[p] = (uint8_t *)dst->data[p];
        a.stride[p] = src->stride[p ? 1 : 0];
        a.pw[p] = (sb128w * 128) >> h;
        a.ph[p] = (sb128h * 128) >> v;
        // filter_uv off: chroma tiles are copies (no edge codes); deblocking off (deferred DC
        // only): every tile is a copy plus its units' DC
        const bool off = !edges || (p && !filter_uv);
        a.cols_ux[p] = off ? 0 : (a.w4 + h) >> h;
        a.cols_rows[p] = off ? 0 : a.ph[p];
        a.rows_px[p] = off ? 0 : a.pw[p];
        a.rows_uy[p] = off ? 0 : p ? sb128h * (32 >> v) : a.h4;
        a.tiles_x[p] = (a.pw[p] + mi::kLfTW - 1) / mi::kLfTW;
        n += a.tiles_x[p] * ((a.ph[p] + mi::kLfTH - 1) / mi::kLfTH);
    }
    a.tile_start[3] = n;
    if (dc_tag) {
        const mi::DcMapGeom g = mi::dc_map_geom(src->w, src->h, src->layout);
        a.dc_map = ctx->dc_map;
        for (int p = 0; p < 3; p++) {
            a.dc_off[p] = g.off[p];
            a.dc_stride[p] = g.stride[p];
        }
        a.dc_tag = dc_tag;
    }
    return mi::launch_deblock_tiles(a, src->bpc, (hipStream_t)stream) ? fail(ctx, -EIO) : 0;
}

int mi_cdef_frame(MiCtx *ctx, const MiPicture *src, const MiPicture *dst, const MiCdef *cd,
                  void *stream) {
    if (!ctx || !src || !dst || !cd || !cd->masks) return fail(ctx, -EINVAL);
    if (src->bpc != dst->bpc || src->w != dst->w || src->h != dst->h || src->layout != dst->layout ||
        src->stride[0] != dst->stride[0] || src->stride[1] != dst->stride[1])
        return fail(ctx, -EINVAL);
    if (src->bpc != 8 && src->bpc != 10 && src->bpc != 12) return fail(ctx, -EINVAL);
    mi::CdefArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) {
        a.src[p] = (const uint8_t *)src->data[p];
        a.dst[p] = (uint8_t *)dst->data[p];
        a.stride[p] = src->stride[p ? 1 : 0];
    }
    a.masks = cd->masks;
    a.sb128w = cd->sb128w;
    if (a.sb128w != (src->w + 127) >> 7) return fail(ctx, -EINVAL);
    a.bw4 = ((src->w + 7) >> 3) << 1;
    a.bh4 = ((src->h + 7) >> 3) << 1;
    a.layout = src->layout;
    a.ss_hor = src->layout == 1 || src->layout == 2;
    a.ss_ver = src->layout == 1;
    a.bdm8 = src->bpc - 8;
    a.damping = cd->damping + a.bdm8;
    memcpy(a.y_strength, cd->y_strength, 8);
    memcpy(a.uv_strength, cd->uv_strength, 8);
    a.tiles_x = (a.bw4 * 4 + 63) / 64;
    a.order = cd->order;
    const int tiles_y = (a.bh4 * 4 + 63) / 64;
    const int r = mi::launch_cdef(a, a.tiles_x * tiles_y, src->bpc, (hipStream_t)stream);
    return r ? fail(ctx, -EIO) : 0;
}

// Costliest class first (cls[t] in 0 .. nclass-1, higher = costlier); within a class the items
// are dealt to the XCDs in contiguous picture runs: workgroup b runs on XCD b % 8, so XCD x takes
// one run of each class and neighbouring tiles share an L2 (the locality xcd_block gives the
// grid order: CDEF 39.2 us this way, 40.1 in xcd_block's grid order, 42.2 for a plain
// costliest-first order)
static void deal_classes(const std::vector<uint8_t> &cls, int nclass, int32_t *order) {
    const int nt = (int)cls.size();
    int b = 0;
    for (int c = nclass - 1; c >= 0; c--) {
        std::vector<int32_t> items;
        for (int t = 0; t < nt; t++)
            if (cls[t] == c) items.push_back(t);
        const int L = (int)items.size();
        int cnt[8] = {}, pos[8];
        for (int r = 0; r < L; r++) cnt[(b + r) & 7]++;
        for (int x = 0, acc = 0; x < 8; x++) {
            pos[x] = acc;
            acc += cnt[x];
        }
        for (int r = 0; r < L; r++) order[b + r] = items[pos[(b + r) & 7]++];
        b += L;
    }
}

int mi_cdef_tile_order(const MiAv1Filter *masks, int w, int h, int layout, const MiCdef *cd, int32_t *order, int n) {
    if (!masks || !cd || !order || w <= 0 || h <= 0 || layout < 0 || layout > 3) return -EINVAL;
    if (cd->sb128w != (w + 127) >> 7) return -EINVAL;
    const int bw4 = ((w + 7) >> 3) << 1, bh4 = ((h + 7) >> 3) << 1;
    const int tx = (bw4 * 4 + 63) / 64, ty = (bh4 * 4 + 63) / 64, nt = tx * ty;
    if (nt > n) return -EINVAL;
    // cost class per unit (cdef_kernel's own tests): 2 a primary strength (direction search and
    // filter), 1 a secondary one only, 0 nothing to filter (no strength, or every 8x8 skipped);
    // then a stable counting sort, costliest first
    std::vector<uint8_t> cls(nt, 0);
    for (int t = 0; t < nt; t++) {
        const int x = t % tx, y = t / tx;
        const MiAv1Filter &lf = masks[(y >> 1) * cd->sb128w + (x >> 1)];
        const int idx = lf.cdef_idx[(y & 1) * 2 + (x & 1)];
        if (idx < 0) continue;
        const int yl = cd->y_strength[idx], uvl = layout ? cd->uv_strength[idx] : 0;
        if (!yl && !uvl) continue;
        // the unit's 8x8 rows (16 per 128-px superblock row, half of them per 64-px unit) and
        // its half of each row's 32-bit noskip word
        unsigned any = 0;
        for (int r = 8 * (y & 1); r < 8 * (y & 1) + 8; r++)
            any |= ((unsigned)lf.noskip_mask[r][1] << 16 | lf.noskip_mask[r][0]) >> (16 * (x & 1)) & 0xffffu;
        if (!any) continue;
        cls[t] = (yl >> 2) || (uvl >> 2) ? 2 : 1;
    }
    deal_classes(cls, 3, order);
    return nt;
}

// The (plane, stripe, tile) grid of mi_lr_frame for a w x h picture (pw, ph, tw, tiles_x,
// blk_start of `a`); -EINVAL for unit sizes outside the bitstream's
static int lr_layout(int w, int h, int layout, const MiLr *lr, mi::LrArgs &a) {
    const int ss_hor = layout == 1 || layout == 2, ss_ver = layout == 1;
    for (int c = 0; c < 2; c++) {
        const int l2 = lr->unit_size_log2[c];
        if ((lr->restore_planes & (c ? 6 : 1)) && (l2 < 5 || l2 > 8)) return -EINVAL;
    }
    a.restore = lr->restore_planes;
    a.ss_hor = ss_hor;
    a.ss_ver = ss_ver;
    a.unit_log2[0] = lr->unit_size_log2[0];
    a.unit_log2[1] = lr->unit_size_log2[1];
    a.sb128w = lr->sb128w;
    const int nplanes = layout ? 3 : 1;
    int nb = 0;
    for (int p = 0; p < 3; p++) {
        a.blk_start[p] = nb;
        if (p >= nplanes) continue;
        const int sh = p ? ss_hor : 0, sv = p ? ss_ver : 0;
        a.pw[p] = (w + sh) >> sh;
        a.ph[p] = (h + sv) >> sv;
        const int us = 1 << lr->unit_size_log2[p ? 1 : 0];
        a.tw[p] = ((a.restore >> p) & 1) && us < 64 ? 32 : 64;
        a.tiles_x[p] = (a.pw[p] + a.tw[p] - 1) / a.tw[p];
        // stripes: 64 luma rows, the first 56 (lr_apply.rs:54)
        int stripes = 0;
        while ((stripes ? (64 * stripes - 8) >> sv : 0) < a.ph[p]) stripes++;
        nb += stripes * a.tiles_x[p];
    }
    a.blk_start[3] = nb;
    return 0;
}

int mi_lr_frame(MiCtx *ctx, const MiPicture *cdef, const MiPicture *deblocked, const MiPicture *dst,
                const MiLr *lr, void *stream) {
    if (!ctx || !cdef || !deblocked || !dst || !lr) return fail(ctx, -EINVAL);
    if (!same_geometry(cdef, deblocked) || !same_geometry(cdef, dst)) return fail(ctx, -EINVAL);
    if (cdef->bpc != 8 && cdef->bpc != 10 && cdef->bpc != 12) return fail(ctx, -EINVAL);
    if (lr->restore_planes && (!lr->lr_mask || lr->sb128w != (cdef->w + 127) >> 7)) return fail(ctx, -EINVAL);
    mi::LrArgs a;
    memset(&a, 0, sizeof(a));
    if (lr_layout(cdef->w, cdef->h, cdef->layout, lr, a)) return fail(ctx, -EINVAL);
    a.lr_mask = lr->lr_mask;
    a.bd = cdef->bpc;
    a.order = lr->order;
    for (int p = 0; p < (cdef->layout ? 3 : 1); p++) {
        a.src[p] = (const uint8_t *)cdef->data[p];
        a.lpf[p] = (const uint8_t *)deblocked->data[p];
        a.dst[p] = (uint8_t *)dst->data[p];
        a.stride[p] = cdef->stride[p ? 1 : 0];
        // lr.hip forms row offsets with one 24-bit multiply
        if (a.stride[p] <= 0 || a.stride[p] >= (1 << 24) || (int64_t)a.ph[p] * a.stride[p] >= (1LL << 32))
            return fail(ctx, -EINVAL);
    }
    const int r = mi::launch_lr(a, cdef->bpc, (hipStream_t)stream);
    return r ? fail(ctx, -EIO) : 0;
}

int mi_lr_tile_order(const MiAv1Restoration *mask, int w, int h, int layout, const MiLr *lr, int32_t *order,
                     int n) {
    if (!lr || !order || w <= 0 || h <= 0 || layout < 0 || layout > 3) return -EINVAL;
    if (lr->restore_planes && !mask) return -EINVAL;
    mi::LrArgs a;
    memset(&a, 0, sizeof(a));
    if (lr_layout(w, h, layout, lr, a) || a.blk_start[3] > n) return -EINVAL;
    // cost class per tile (lr_kernel's unit lookup): 3 self-guided with both radii, 2 with one
    // (sgr_params 10-15), 1 Wiener, 0 copy; then a stable counting sort, costliest first
    std::vector<uint8_t> cls(a.blk_start[3], 0);
    for (int p = 0; p < 3; p++) {
        if (!((a.restore >> p) & 1)) continue;
        const int ssh = p ? a.ss_hor : 0, ssv = p ? a.ss_ver : 0, pw = a.pw[p], ph = a.ph[p];
        const int us = 1 << a.unit_log2[p ? 1 : 0], nu = std::max(1, (pw + (us >> 1)) / us);
        for (int b = a.blk_start[p]; b < a.blk_start[p + 1]; b++) {
            const int lb = b - a.blk_start[p], k = lb / a.tiles_x[p], ti = lb - k * a.tiles_x[p];
            const int xu = std::min(ti * a.tw[p] / us, nu - 1) * us;
            int ay = ((64 * k) >> ssv) & ~(us - 1);
            if (ay && ay + (us >> 1) > ph) ay -= us;
            ay <<= ssv;
            const int t = mask[(ay >> 7) * a.sb128w + (xu >> (7 - ssh))].lr[p][(((ay >> 6) & 1) << 1) + ((xu >> (6 - ssh)) & 1)].type;
            cls[b] = t == 0 ? 0 : t == 2 ? 1 : t >= 3 && t - 3 < 10 ? 3 : t >= 3 ? 2 : 0;
        }
    }
    // (each class dealt to the XCDs in contiguous picture runs, as CDEF's order is, halves LR's
    // HBM reads, 68.0 -> 35.9 MB, but runs 35.0-35.8 us against 31.5-32.1: DESIGN.md, round 6)
    int start[5] = {};
    for (uint8_t c : cls) start[3 - c + 1]++;
    for (int c = 0; c < 4; c++) start[c + 1] += start[c];
    for (int b = 0; b < a.blk_start[3]; b++) order[start[3 - cls[b]]++] = b;
    return a.blk_start[3];
}

static int fg_tables() {
    static std::once_flag once;
    static int tables_rc = 0;
    std::call_once(once, [] { tables_rc = mi::init_fg_tables(); });
    return tables_rc ? -EIO : 0;
}
static bool fg_data_ok(const MiFilmGrainData *data) {
    return !(data->num_y_points < 0 || data->num_y_points > 14 || data->ar_coeff_lag < 0 || data->ar_coeff_lag > 3 ||
             data->num_uv_points[0] < 0 || data->num_uv_points[0] > 10 || data->num_uv_points[1] < 0 ||
             data->num_uv_points[1] > 10 || data->ar_coeff_shift < 6 || data->ar_coeff_shift > 9);
}

static int fg_setup(MiCtx *ctx, const MiPicture *in, const MiPicture *out, const MiFilmGrainData *data,
                    int is_id, mi::FgArgs &a) {
    if (int e = fg_tables()) return e;
    if (in->bpc != 8 && in->bpc != 10 && in->bpc != 12) return -EINVAL;
    if (!fg_data_ok(data)) return -EINVAL;
    memset(&a, 0, sizeof(a));
    a.data = *data;
    a.bpc = in->bpc;
    a.layout = in->layout;
    a.ss_x = in->layout == 1 || in->layout == 2;
    a.ss_y = in->layout == 1;
    a.w = in->w;
    a.h = in->h;
    a.is_id = is_id;
    a.nrows = (in->h + 31) >> 5;
    a.nblocks = (in->w + 31) >> 5;
    if (!ctx->fg_lut && hipMalloc(&ctx->fg_lut, 3 * 73 * 88 * sizeof(int16_t)) != hipSuccess) return -ENOMEM;
    if (!ctx->fg_scaling && hipMalloc(&ctx->fg_scaling, 3 * 4096) != hipSuccess) return -ENOMEM;
    const size_t ob = (size_t)a.nrows * a.nblocks;
    if (ob > ctx->fg_offsets_bytes) {
        if (ctx->fg_offsets) (void)hipFree(ctx->fg_offsets);
        ctx->fg_offsets = nullptr;
        if (hipMalloc(&ctx->fg_offsets, ob) != hipSuccess) return -ENOMEM;
        ctx->fg_offsets_bytes = ob;
    }
    a.lut = ctx->fg_lut;
    a.scaling = ctx->fg_scaling;
    a.offsets = ctx->fg_offsets;
    if (out) {
        if (!same_geometry(in, out)) return -EINVAL;
        const int nplanes = in->layout ? 3 : 1;
        int nb = 0;
        for (int p = 0; p < 3; p++) {
            a.blk_start[p] = nb;
            if (p >= nplanes) continue;
            a.src[p] = (const uint8_t *)in->data[p];
            a.dst[p] = (uint8_t *)out->data[p];
            a.stride[p] = in->stride[p ? 1 : 0];
            const int sh = p ? a.ss_x : 0, sv = p ? a.ss_y : 0;
            a.pw[p] = (in->w + sh) >> sh;
            a.ph[p] = (in->h + sv) >> sv;
            a.chunks[p] = (a.pw[p] + 511) / 512;   // 64-lane waves per row, 8 contiguous px per lane
            a.grain[p] = p == 0 ? data->num_y_points != 0
                                : (data->chroma_scaling_from_luma || data->num_uv_points[p - 1]);
            nb += (int)(((int64_t)a.chunks[p] * a.ph[p] + 4 * mi::kFgItems - 1) / (4 * mi::kFgItems));
        }
        a.blk_start[3] = nb;
    }
    return 0;
}

int mi_film_grain_prep(MiCtx *ctx, const MiPicture *in, const MiFilmGrainData *data, void *stream) {
    if (!ctx || !in || !data) return fail(ctx, -EINVAL);
    mi::FgArgs a;
    if (int e = fg_setup(ctx, in, nullptr, data, 0, a)) return fail(ctx, e);
    return mi::launch_fg(a, (hipStream_t)stream, true, false) ? fail(ctx, -EIO) : 0;
}

int mi_film_grain_apply(MiCtx *ctx, const MiPicture *in, const MiPicture *out, const MiFilmGrainData *data,
                        int mtrx_identity, void *stream) {
    if (!ctx || !in || !out || !data) return fail(ctx, -EINVAL);
    mi::FgArgs a;
    if (int e = fg_setup(ctx, in, out, data, mtrx_identity, a)) return fail(ctx, e);
    return mi::launch_fg(a, (hipStream_t)stream, false, true) ? fail(ctx, -EIO) : 0;
}

int mi_film_grain_frame(MiCtx *ctx, const MiPicture *in, const MiPicture *out, const MiFilmGrainData *data,
                        int mtrx_identity, void *stream) {
    if (!ctx || !in || !out || !data) return fail(ctx, -EINVAL);
    mi::FgArgs a;
    if (int e = fg_setup(ctx, in, out, data, mtrx_identity, a)) return fail(ctx, e);
    return mi::launch_fg(a, (hipStream_t)stream, true, true) ? fail(ctx, -EIO) : 0;
}

// ---- table-compatible per-call entry points ------------------------------------------

int mi_dsp_itxfm_add(int tx, int txtp, void *dst, ptrdiff_t stride, void *coeff, int eob,
                     int bitdepth_max) {
    if (tx < 0 || tx >= MI_N_RECT_TX_SIZES || !mi::itx_type_valid(tx, txtp) || !dst || !coeff ||
        eob < 0)
        return -EINVAL;
    const int bpc = bitdepth_max == 255 ? 8 : bitdepth_max == 1023 ? 10 : bitdepth_max == 4095 ? 12 : 0;
    if (!bpc) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    if (hipSetDevice(0) != hipSuccess) return -ENODEV;

    const mi::TxDim d = mi::tx_dim(tx);
    const int px = bpc == 8 ? 1 : 2, cb = bpc == 8 ? 2 : 4;
    const size_t ncoef = (size_t)mi::imin_c(d.w, 32) * mi::imin_c(d.h, 32);
    const size_t row_bytes = (size_t)d.w * px;
    hipStream_t s = g_call.stream;

    // device layout in scratch: [pixels h*row_bytes][coef][descriptor]
    uint8_t *dpix = g_call.scratch;
    uint8_t *dcoef = dpix + 64 * 128;
    MiTxBlock *dblk = (MiTxBlock *)(dcoef + 32 * 32 * 4);

    const bool dst_dev = is_device_ptr(dst), cf_dev = is_device_ptr(coeff);
    std::vector<uint8_t> hpix;
    if (dst_dev) {
        for (int y = 0; y < d.h; y++)
            if (hipMemcpyAsync(dpix + y * row_bytes, (uint8_t *)dst + y * stride, row_bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
                return -EIO;
    } else {
        hpix.resize(row_bytes * d.h);
        for (int y = 0; y < d.h; y++) memcpy(&hpix[y * row_bytes], (uint8_t *)dst + y * stride, row_bytes);
        if (hipMemcpyAsync(dpix, hpix.data(), hpix.size(), hipMemcpyHostToDevice, s) != hipSuccess) return -EIO;
    }
    if (hipMemcpyAsync(dcoef, coeff, ncoef * cb, cf_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s) != hipSuccess)
        return -EIO;
    MiTxBlock hb{};
    hb.tx = (uint8_t)tx;
    hb.txtp = (uint8_t)txtp;
    hb.eob = eob;
    if (hipMemcpyAsync(dblk, &hb, sizeof(hb), hipMemcpyHostToDevice, s) != hipSuccess) return -EIO;

    mi::ItxArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) { a.plane[p] = dpix; a.stride[p] = (int64_t)row_bytes; }
    a.blocks = dblk;
    a.coef = dcoef;
    a.bdmax = bitdepth_max;
    a.zero_coefs = 1;
    a.pw[0] = d.w;
    a.ph[0] = d.h;
    a.err = (int *)(dblk + 1);   // scratch word: the host checked tx / txtp above
    uint32_t ss1[MI_N_RECT_TX_SIZES + 1];
    for (int k = 0; k <= MI_N_RECT_TX_SIZES; k++) ss1[k] = k > tx ? 1 : 0;
    const int nwg = mi::itx_fill_schedule(a, ss1);
    if (mi::launch_itx_frame(a, nwg, bpc, s)) return -EIO;

    if (dst_dev) {
        for (int y = 0; y < d.h; y++)
            if (hipMemcpyAsync((uint8_t *)dst + y * stride, dpix + y * row_bytes, row_bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
                return -EIO;
    } else {
        if (hipMemcpyAsync(hpix.data(), dpix, hpix.size(), hipMemcpyDeviceToHost, s) != hipSuccess) return -EIO;
    }
    if (hipMemcpyAsync(coeff, dcoef, ncoef * cb, cf_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s) != hipSuccess)
        return -EIO;
    if (hipStreamSynchronize(s) != hipSuccess) return -EIO;
    if (!dst_dev)
        for (int y = 0; y < d.h; y++) memcpy((uint8_t *)dst + y * stride, &hpix[y * row_bytes], row_bytes);
    return 0;
}

int mi_dsp_intra_pred(int mode, void *dst, ptrdiff_t stride, const void *topleft, int w, int h,
                      int angle, int max_width, int max_height, int bitdepth_max) {
    if (mode < 0 || mode > 13 || !dst || !topleft || w < 4 || h < 4 || w > 64 || h > 64 ||
        (w & (w - 1)) || (h & (h - 1)) || (mode == 13 && (w > 32 || h > 32)))
        return -EINVAL;
    const int bpc = bitdepth_max == 255 ? 8 : bitdepth_max == 1023 ? 10 : bitdepth_max == 4095 ? 12 : 0;
    if (!bpc) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    if (hipSetDevice(0) != hipSuccess) return -ENODEV;
    const int px = bpc == 8 ? 1 : 2;
    const size_t row_bytes = (size_t)w * px;
    hipStream_t s = g_call.stream;
    // device scratch: [pixels 64 rows x 128 B][edge 257 samples][descriptor]
    uint8_t *dpix = g_call.scratch;
    uint8_t *dedge = dpix + 64 * 128;
    MiIpredBlock *dblk = (MiIpredBlock *)(dedge + 1024);
    const int ext = w + h;                      // samples read on each side of topleft
    const uint8_t *esrc = (const uint8_t *)topleft - (ptrdiff_t)ext * px;
    const hipMemcpyKind ek = is_device_ptr(topleft) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (hipMemcpyAsync(dedge, esrc, (size_t)(2 * ext + 1) * px, ek, s) != hipSuccess) return -EIO;
    MiIpredBlock hb{};
    hb.edge_off = (uint32_t)ext;
    hb.w = (uint8_t)w;
    hb.h = (uint8_t)h;
    hb.mode = (uint8_t)mode;
    hb.angle = (uint16_t)angle;
    hb.max_w = (uint16_t)max_width;
    hb.max_h = (uint16_t)max_height;
    if (hipMemcpyAsync(dblk, &hb, sizeof(hb), hipMemcpyHostToDevice, s) != hipSuccess) return -EIO;
    mi::IpredArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) a.dst[p] = dpix;
    a.stride[0] = a.stride[1] = (int64_t)row_bytes;
    a.blocks = dblk;
    a.edges = dedge;
    a.bpc = bpc;
    a.bdmax = bitdepth_max;
    if (mi::launch_ipred(a, 1, s)) return -EIO;
    const bool dst_dev = is_device_ptr(dst);
    std::vector<uint8_t> hpix(dst_dev ? 0 : row_bytes * h);
    for (int y = 0; y < h; y++) {
        const hipError_t e = dst_dev
            ? hipMemcpyAsync((uint8_t *)dst + y * stride, dpix + y * row_bytes, row_bytes, hipMemcpyDeviceToDevice, s)
            : hipMemcpyAsync(&hpix[y * row_bytes], dpix + y * row_bytes, row_bytes, hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return -EIO;
    }
    if (hipStreamSynchronize(s) != hipSuccess) return -EIO;
    if (!dst_dev)
        for (int y = 0; y < h; y++) memcpy((uint8_t *)dst + y * stride, &hpix[y * row_bytes], row_bytes);
    return 0;
}

// ---- helpers of the remaining per-call entries: caller pixel windows <-> device scratch ----
namespace {
int bpc_of(int bitdepth_max) {
    return bitdepth_max == 255 ? 8 : bitdepth_max == 1023 ? 10 : bitdepth_max == 4095 ? 12 : 0;
}
// rows [r0, r1) x bytes [b0, b1) around `base` (host or device, any stride sign) <-> a packed
// device window of pitch (b1 - b0)
int win_in(uint8_t *dev, const void *base, ptrdiff_t stride, int r0, int r1, ptrdiff_t b0, ptrdiff_t b1, hipStream_t s) {
    for (int r = r0; r < r1; r++)
        if (hipMemcpyAsync(dev + (size_t)(r - r0) * (b1 - b0), (const uint8_t *)base + r * stride + b0, b1 - b0,
                           hipMemcpyDefault, s) != hipSuccess)
            return -EIO;
    return 0;
}
int win_out(void *base, ptrdiff_t stride, const uint8_t *dev, int r0, int r1, ptrdiff_t b0, ptrdiff_t b1, hipStream_t s) {
    for (int r = r0; r < r1; r++)
        if (hipMemcpyAsync((uint8_t *)base + r * stride + b0, dev + (size_t)(r - r0) * (b1 - b0), b1 - b0,
                           hipMemcpyDefault, s) != hipSuccess)
            return -EIO;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO;
}
int copy_in(void *dev, const void *src, size_t n, hipStream_t s) {
    return hipMemcpyAsync(dev, src, n, hipMemcpyDefault, s) == hipSuccess ? 0 : -EIO;
}
}  // namespace

extern "C" {

int mi_dsp_cfl_pred(int mode, void *dst, ptrdiff_t stride, const void *topleft, int w, int h, const int16_t *ac,
                    int alpha, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !dst || !topleft || !ac || (mode != 0 && mode != 3 && mode != 4 && mode != 5) || w < 4 || h < 4 ||
        w > 32 || h > 32 || (w & (w - 1)) || (h & (h - 1)))
        return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    uint8_t *dpix = g_call.scratch, *dedge = dpix + 64 * 128, *dac = dedge + 1024;
    MiIpredBlock *dblk = (MiIpredBlock *)(dac + 64 * 64 * 2);
    int e = copy_in(dedge, (const uint8_t *)topleft - (ptrdiff_t)h * px, (size_t)(w + h + 1) * px, s);
    if (!e) e = copy_in(dac, ac, (size_t)w * h * 2, s);
    MiIpredBlock hb{};
    hb.edge_off = (uint32_t)h;
    hb.w = (uint8_t)w;
    hb.h = (uint8_t)h;
    hb.mode = (uint8_t)(MI_IPRED_CFL + mode);
    hb.alpha = (int8_t)alpha;
    if (!e) e = copy_in(dblk, &hb, sizeof(hb), s);
    if (e) return e;
    mi::IpredArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) a.dst[p] = dpix;
    a.stride[0] = a.stride[1] = (int64_t)w * px;
    a.blocks = dblk;
    a.edges = dedge;
    a.ac = (const int16_t *)dac;
    a.bpc = bpc;
    a.bdmax = bitdepth_max;
    if (mi::launch_ipred(a, 1, s)) return -EIO;
    return win_out(dst, stride, dpix, 0, h, 0, (ptrdiff_t)w * px, s);
}

int mi_dsp_pal_pred(void *dst, ptrdiff_t stride, const void *pal, const uint8_t *idx, int w, int h, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !dst || !pal || !idx || w < 4 || h < 4 || w > 64 || h > 64) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    uint8_t *dpix = g_call.scratch, *dpal = dpix + 64 * 128, *didx = dpal + 64;
    MiIpredBlock *dblk = (MiIpredBlock *)(didx + 64 * 64);
    int e = copy_in(dpal, pal, 8 * (size_t)px, s);
    if (!e) e = copy_in(didx, idx, (size_t)w * h, s);
    MiIpredBlock hb{};
    hb.w = (uint8_t)w;
    hb.h = (uint8_t)h;
    hb.mode = MI_IPRED_PAL;
    if (!e) e = copy_in(dblk, &hb, sizeof(hb), s);
    if (e) return e;
    mi::IpredArgs a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) a.dst[p] = dpix;
    a.stride[0] = a.stride[1] = (int64_t)w * px;
    a.blocks = dblk;
    a.edges = dpal;
    a.idx = didx;
    a.bpc = bpc;
    a.bdmax = bitdepth_max;
    if (mi::launch_ipred(a, 1, s)) return -EIO;
    return win_out(dst, stride, dpix, 0, h, 0, (ptrdiff_t)w * px, s);
}

int mi_dsp_cfl_ac(int layout, int16_t *ac, const void *y, ptrdiff_t stride, int w_pad, int h_pad, int cw, int ch,
                  int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !ac || !y || layout < 1 || layout > 3 || cw < 4 || ch < 4 || cw > 32 || ch > 32 ||
        (cw & (cw - 1)) || (ch & (ch - 1)) || w_pad < 0 || h_pad < 0 || 4 * w_pad >= cw || 4 * h_pad >= ch)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    const int ss_hor = layout != 3, ss_ver = layout == 1;
    const int rows = (ch - 4 * h_pad) << ss_ver, cols = (cw - 4 * w_pad) << ss_hor;
    hipStream_t s = g_call.stream;
    uint8_t *dy = g_call.scratch;
    int16_t *dac = (int16_t *)(dy + 64 * 128);
    if (int e = win_in(dy, y, stride, 0, rows, 0, (ptrdiff_t)cols * px, s)) return e;
    mi::CflAcArgs a;
    a.ac = dac;
    a.y = dy;
    a.stride = (int64_t)cols * px;
    a.w_pad = w_pad;
    a.h_pad = h_pad;
    a.cw = cw;
    a.ch = ch;
    a.ss_hor = ss_hor;
    a.ss_ver = ss_ver;
    if (mi::launch_cfl_ac(a, bpc, s)) return -EIO;
    if (hipMemcpyAsync(ac, dac, (size_t)cw * ch * 2, hipMemcpyDefault, s) != hipSuccess) return -EIO;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO;
}

int mi_dsp_loop_filter_sb(int cls, int dir, void *dst, ptrdiff_t stride, const uint32_t *vmask,
                          const uint8_t (*lvl)[4], ptrdiff_t b4_stride, const void *lut, int wh, int bitdepth_max) {
    (void)wh;
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || cls < 0 || cls > 1 || dir < 0 || dir > 1 || !dst || !vmask || !lvl || !lut) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    mi::LfCallArgs a;
    memset(&a, 0, sizeof(a));
    if (hipMemcpy(a.vmask, vmask, (cls ? 2 : 3) * sizeof(uint32_t), hipMemcpyDefault) != hipSuccess) return -EIO;
    const unsigned vm = a.vmask[0] | a.vmask[1] | a.vmask[2];
    if (!vm) return 0;
    const int nu = 32 - __builtin_clz(vm);                 // units up to the highest set bit
    // level pairs {unit, neighbour}: the caller's map is strided (b4_stride entries per row)
    uint8_t lv[64] = {0};
    const ptrdiff_t ul = dir == 0 ? b4_stride : 1, pl = dir == 0 ? -1 : -b4_stride;
    for (int k = 0; k < nu; k++) {
        if (!(vm & (1u << k))) continue;
        if (hipMemcpy(&lv[2 * k], &lvl[k * ul][0], 1, hipMemcpyDefault) != hipSuccess ||
            hipMemcpy(&lv[2 * k + 1], &lvl[k * ul + pl][0], 1, hipMemcpyDefault) != hipSuccess)
            return -EIO;
    }
    uint8_t lt[128];
    if (hipMemcpy(lt, lut, 128, hipMemcpyDefault) != hipSuccess) return -EIO;   // Av1FilterLUT.e, .i
    memcpy(a.lim_e, lt, 64);
    memcpy(a.lim_i, lt + 64, 64);
    // the pixel window: 8 samples either side of the edge, 4 * nu along it
    const int r0 = dir == 0 ? 0 : -8, r1 = dir == 0 ? 4 * nu : 8;
    const ptrdiff_t b0 = (dir == 0 ? -8 : 0) * px, b1 = (dir == 0 ? 8 : 4 * nu) * px;
    uint8_t *dwin = g_call.scratch, *dlv = dwin + (1 << 19);
    if (int e = win_in(dwin, dst, stride, r0, r1, b0, b1, s)) return e;
    if (int e = copy_in(dlv, lv, sizeof(lv), s)) return e;
    a.dst = dwin + (size_t)(-r0) * (b1 - b0) - b0;
    a.stride = b1 - b0;
    a.lvl = dlv;
    a.cls = cls;
    a.dir = dir;
    a.bdm8 = bpc - 8;
    a.bdmax = bitdepth_max;
    if (mi::launch_lf_sb_call(a, bpc, s)) return -EIO;
    return win_out(dst, stride, dwin, r0, r1, b0, b1, s);
}

int mi_dsp_cdef_filter(int fb, void *dst, ptrdiff_t stride, const void *left, const void *top, const void *bottom,
                       int pri, int sec, int dir, int damping, int edges, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || fb < 0 || fb > 2 || !dst || dir < 0 || dir > 7 || pri < 0 || sec < 0) return -EINVAL;
    const int w = fb == 0 ? 8 : 4, h = fb == 2 ? 4 : 8;
    if (((edges & 1) && !left) || ((edges & 4) && !top) || ((edges & 8) && !bottom)) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    // one packed window, pitch P, column 0 = x - 2: rows 0-1 from top, 2..h+1 the block,
    // h+2..h+3 from bottom; only the columns the edge flags allow are read from the caller
    const ptrdiff_t P = (ptrdiff_t)(w + 4) * px;
    const ptrdiff_t x0 = (edges & 1) ? -2 * px : 0, x1 = (ptrdiff_t)(w + ((edges & 2) ? 2 : 0)) * px;
    uint8_t *win = g_call.scratch, *dleft = win + 4096, *dout = dleft + 4096;
    auto rows = [&](const void *src, int r0, int n, ptrdiff_t c0) -> int {
        for (int r = 0; r < n; r++)
            if (hipMemcpyAsync(win + (size_t)(r0 + r) * P + 2 * px + c0, (const uint8_t *)src + r * stride + c0, x1 - c0,
                               hipMemcpyDefault, s) != hipSuccess)
                return -EIO;
        return 0;
    };
    int e = rows(dst, 2, h, 0);
    if (!e && (edges & 4)) e = rows(top, 0, 2, x0);
    if (!e && (edges & 8)) e = rows(bottom, 2 + h, 2, x0);
    if (!e && (edges & 1)) e = copy_in(dleft, left, (size_t)h * 2 * px, s);
    if (e) return e;
    mi::CdefCallArgs a;
    memset(&a, 0, sizeof(a));
    a.top = win + 2 * px;
    a.dst = win + 2 * P + 2 * px;
    a.bottom = win + (2 + h) * P + 2 * px;
    a.left = dleft;
    a.out = dout;
    a.stride = P;
    a.w = w;
    a.h = h;
    a.pri = pri;
    a.sec = sec;
    a.dir = dir;
    a.damping = damping;
    a.edges = edges;
    a.bdm8 = bpc - 8;
    if (mi::launch_cdef_call(a, bpc, false, s)) return -EIO;
    return win_out(dst, stride, dout, 0, h, 0, (ptrdiff_t)w * px, s);
}

int mi_dsp_cdef_dir(const void *img, ptrdiff_t stride, unsigned *var, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !img || !var) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    uint8_t *win = g_call.scratch, *dout = win + 4096;
    if (int e = win_in(win, img, stride, 0, 8, 0, 8 * px, s)) return e;
    mi::CdefCallArgs a;
    memset(&a, 0, sizeof(a));
    a.dst = win;
    a.out = dout;
    a.stride = 8 * px;
    a.bdm8 = bpc - 8;
    if (mi::launch_cdef_call(a, bpc, true, s)) return -EIO;
    int r[2];
    if (hipMemcpyAsync(r, dout, sizeof(r), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    *var = (unsigned)r[1];
    return r[0];
}

// ---- mc table (src/mc.rs:1174-1338): put / prep, combine, blend, emu_edge ----
namespace {
void mc_call_bd(mi::McCallArgs &a, int bpc, int bdmax) {
    a.bpc = bpc;
    a.ib = bpc == 8 ? 4 : 14 - bpc;
    a.bias = bpc == 8 ? 0 : 8192;
    a.bdmax = bdmax;
}
bool mc_dims_ok(int w, int h) { return w >= 2 && h >= 2 && w <= 128 && h <= 128; }
}  // namespace

int mi_dsp_mc_put(int filter2d, void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int w, int h,
                  int mx, int my, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !dst || !src || filter2d < 0 || filter2d > 9 || !mc_dims_ok(w, h) || mx < 0 || mx > 15 || my < 0 ||
        my > 15)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    // source window: rows -3 .. h+4, columns -3 .. w+4 (8-tap reach; bilinear uses +1)
    const int r0 = filter2d == 9 ? 0 : -3, r1 = h + (filter2d == 9 ? 1 : 5);
    const ptrdiff_t b0 = (filter2d == 9 ? 0 : -3) * px, b1 = (ptrdiff_t)(w + (filter2d == 9 ? 1 : 5)) * px;
    uint8_t *win = g_call.scratch, *dout = win + (1 << 19);
    if (int e = win_in(win, src, src_stride, r0, r1, b0, b1, s)) return e;
    mi::McCallArgs a;
    memset(&a, 0, sizeof(a));
    a.src = win + (size_t)(-r0) * (b1 - b0) - b0;
    a.src_stride = b1 - b0;
    a.dst = dout;
    a.dst_stride = (int64_t)w * px;
    a.w = w; a.h = h; a.mx = mx; a.my = my; a.filter2d = filter2d;
    mc_call_bd(a, bpc, bitdepth_max);
    if (mi::launch_mc_call(a, 0, s)) return -EIO;
    return win_out(dst, dst_stride, dout, 0, h, 0, (ptrdiff_t)w * px, s);
}

int mi_dsp_mc_prep(int filter2d, int16_t *tmp, const void *src, ptrdiff_t src_stride, int w, int h, int mx, int my,
                   int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !tmp || !src || filter2d < 0 || filter2d > 9 || !mc_dims_ok(w, h) || mx < 0 || mx > 15 || my < 0 ||
        my > 15)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    const int r0 = filter2d == 9 ? 0 : -3, r1 = h + (filter2d == 9 ? 1 : 5);
    const ptrdiff_t b0 = (filter2d == 9 ? 0 : -3) * px, b1 = (ptrdiff_t)(w + (filter2d == 9 ? 1 : 5)) * px;
    uint8_t *win = g_call.scratch;
    int16_t *dtmp = (int16_t *)(win + (1 << 19));
    if (int e = win_in(win, src, src_stride, r0, r1, b0, b1, s)) return e;
    mi::McCallArgs a;
    memset(&a, 0, sizeof(a));
    a.src = win + (size_t)(-r0) * (b1 - b0) - b0;
    a.src_stride = b1 - b0;
    a.tmp1 = dtmp;
    a.prep = 1;
    a.w = w; a.h = h; a.mx = mx; a.my = my; a.filter2d = filter2d;
    mc_call_bd(a, bpc, bitdepth_max);
    if (mi::launch_mc_call(a, 0, s)) return -EIO;
    if (hipMemcpyAsync(tmp, dtmp, (size_t)w * h * 2, hipMemcpyDefault, s) != hipSuccess) return -EIO;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO;
}

namespace {
// avg / w_avg / mask / w_mask / blend*: op as mc_call_comb_kernel
int mc_combine(int op, void *dst, ptrdiff_t ds, const int16_t *t1, const int16_t *t2, const void *tmp_px,
               int w, int h, const uint8_t *mask, uint8_t *mask_out, int weight, int sign, int layout, int bdmax) {
    const int bpc = bpc_of(bdmax);
    if (!bpc || !dst || !mc_dims_ok(w, h)) return -EINVAL;
    if ((op <= 3 && (!t1 || !t2)) || ((op == 2 || op == 4) && !mask) || (op == 3 && !mask_out) ||
        (op >= 4 && !tmp_px) || (op == 3 && (layout < 1 || layout > 3)))
        return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    const size_t n = (size_t)w * h;
    uint8_t *dd = g_call.scratch, *d1 = dd + 65536, *d2 = d1 + 65536, *dm = d2 + 65536, *dmo = dm + 16384,
            *dt = dmo + 16384;
    mi::McCallArgs a;
    memset(&a, 0, sizeof(a));
    int e = 0;
    if (op <= 3) {
        e = copy_in(d1, t1, n * 2, s);
        if (!e) e = copy_in(d2, t2, n * 2, s);
    }
    if (!e && (op == 2 || op == 4)) e = copy_in(dm, mask, n, s);
    if (!e && op >= 4) e = copy_in(dt, tmp_px, n * px, s);
    if (!e && op >= 4) e = win_in(dd, dst, ds, 0, h, 0, (ptrdiff_t)w * px, s);   // blends read dst
    if (e) return e;
    a.dst = dd;
    a.dst_stride = (int64_t)w * px;
    a.tmp1 = (int16_t *)d1;
    a.tmp2 = (const int16_t *)d2;
    a.mask = dm;
    a.mask_out = dmo;
    a.src = dt;
    a.w = w; a.h = h; a.op = op; a.weight = weight; a.sign = sign;
    a.ss_hor = layout == 1 || layout == 2;
    a.ss_ver = layout == 1;
    mc_call_bd(a, bpc, bdmax);
    if (mi::launch_mc_call(a, 1, s)) return -EIO;
    if (op == 3 && hipMemcpyAsync(mask_out, dmo, (size_t)(w >> a.ss_hor) * (h >> a.ss_ver), hipMemcpyDefault, s) != hipSuccess)
        return -EIO;
    return win_out(dst, ds, dd, 0, h, 0, (ptrdiff_t)w * px, s);
}
}  // namespace

int mi_dsp_mc_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                  int bitdepth_max) {
    return mc_combine(0, dst, dst_stride, tmp1, tmp2, nullptr, w, h, nullptr, nullptr, 0, 0, 0, bitdepth_max);
}
int mi_dsp_mc_w_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h, int weight,
                    int bitdepth_max) {
    return mc_combine(1, dst, dst_stride, tmp1, tmp2, nullptr, w, h, nullptr, nullptr, weight, 0, 0, bitdepth_max);
}
int mi_dsp_mc_mask(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w, int h,
                   const uint8_t *mask, int bitdepth_max) {
    return mc_combine(2, dst, dst_stride, tmp1, tmp2, nullptr, w, h, mask, nullptr, 0, 0, 0, bitdepth_max);
}
int mi_dsp_mc_w_mask(int layout, void *dst, ptrdiff_t dst_stride, const int16_t *tmp1, const int16_t *tmp2, int w,
                     int h, uint8_t *mask, int sign, int bitdepth_max) {
    return mc_combine(3, dst, dst_stride, tmp1, tmp2, nullptr, w, h, nullptr, mask, 0, sign, layout, bitdepth_max);
}
int mi_dsp_mc_blend(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h, const uint8_t *mask,
                    int bitdepth_max) {
    return mc_combine(4, dst, dst_stride, nullptr, nullptr, tmp, w, h, mask, nullptr, 0, 0, 0, bitdepth_max);
}
int mi_dsp_mc_blend_v(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h, int bitdepth_max) {
    return mc_combine(5, dst, dst_stride, nullptr, nullptr, tmp, w, h, nullptr, nullptr, 0, 0, 0, bitdepth_max);
}
int mi_dsp_mc_blend_h(void *dst, ptrdiff_t dst_stride, const void *tmp, int w, int h, int bitdepth_max) {
    return mc_combine(6, dst, dst_stride, nullptr, nullptr, tmp, w, h, nullptr, nullptr, 0, 0, 0, bitdepth_max);
}

int mi_dsp_mc_emu_edge(int bw, int bh, int iw, int ih, int x, int y, void *dst, ptrdiff_t dst_stride, const void *ref,
                       ptrdiff_t ref_stride, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !dst || !ref || bw < 1 || bh < 1 || bw > 256 || bh > 256 || iw < 1 || ih < 1) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    auto clip = [](int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; };
    // the reference pixels the block can reach: the clamped rectangle
    const int ry0 = clip(y, 0, ih - 1), ry1 = clip(y + bh - 1, 0, ih - 1) + 1;
    const int rx0 = clip(x, 0, iw - 1), rx1 = clip(x + bw - 1, 0, iw - 1) + 1;
    uint8_t *win = g_call.scratch, *dout = win + (1 << 19);
    if (int e = win_in(win, (const uint8_t *)ref + (ptrdiff_t)ry0 * ref_stride + (ptrdiff_t)rx0 * px, ref_stride, 0,
                       ry1 - ry0, 0, (ptrdiff_t)(rx1 - rx0) * px, s))
        return e;
    mi::McCallArgs a;
    memset(&a, 0, sizeof(a));
    a.src = win;
    a.src_stride = (int64_t)(rx1 - rx0) * px;
    a.dst = dout;
    a.dst_stride = (int64_t)bw * px;
    a.w = bw; a.h = bh; a.mx = x; a.my = y; a.iw = iw; a.ih = ih;
    mc_call_bd(a, bpc, bitdepth_max);
    if (mi::launch_mc_call(a, 2, s)) return -EIO;
    return win_out(dst, dst_stride, dout, 0, bh, 0, (ptrdiff_t)bw * px, s);
}

int mi_dsp_mc_warp8x8(int prep, void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                      const int16_t *abcd, int mx, int my, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !dst || !src || !abcd) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    int16_t hb[4];
    if (hipMemcpy(hb, abcd, sizeof(hb), hipMemcpyDefault) != hipSuccess) return -EIO;
    uint8_t *win = g_call.scratch, *dout = win + 4096;
    const int r0 = -3, r1 = 12;
    const ptrdiff_t b0 = -3 * px, b1 = 12 * px;
    if (int e = win_in(win, src, src_stride, r0, r1, b0, b1, s)) return e;
    mi::McCallArgs a;
    memset(&a, 0, sizeof(a));
    a.src = win + (size_t)(-r0) * (b1 - b0) - b0;
    a.src_stride = b1 - b0;
    a.dst = dout;
    a.dst_stride = 8 * px;
    a.tmp1 = (int16_t *)dout;
    a.prep = prep;
    a.w = 8; a.h = 8; a.mx = mx; a.my = my;
    for (int i = 0; i < 4; i++) a.abcd[i] = hb[i];
    mc_call_bd(a, bpc, bitdepth_max);
    if (mi::launch_mc_call(a, 3, s)) return -EIO;
    // warp8x8t: dst is the int16 intermediate with stride dst_stride (in elements, as the
    // reference's tmp_stride); warp8x8: pixels
    if (prep) return win_out(dst, dst_stride * 2, dout, 0, 8, 0, 16, s);
    return win_out(dst, dst_stride, dout, 0, 8, 0, 8 * px, s);
}

int mi_dsp_mc_resize(void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride, int dst_w, int h,
                     int src_w, int dx, int mx0, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !dst || !src || dst_w < 1 || h < 1 || src_w < 1 || dst_w > 8192 || src_w > 8192 || h > 64 ||
        mx0 < 0 || mx0 >= (1 << 14))
        return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    if ((size_t)(src_w + dst_w) * h * px > (1u << 20)) return -EINVAL;
    hipStream_t s = g_call.stream;
    uint8_t *win = g_call.scratch, *dout = win + (size_t)src_w * h * px;
    if (int e = win_in(win, src, src_stride, 0, h, 0, (ptrdiff_t)src_w * px, s)) return e;
    mi::McCallArgs a;
    memset(&a, 0, sizeof(a));
    a.src = win;
    a.src_stride = (int64_t)src_w * px;
    a.dst = dout;
    a.dst_stride = (int64_t)dst_w * px;
    a.w = dst_w; a.h = h; a.iw = src_w; a.mx = mx0; a.weight = dx;
    mc_call_bd(a, bpc, bitdepth_max);
    if (mi::launch_mc_call(a, 4, s)) return -EIO;
    return win_out(dst, dst_stride, dout, 0, h, 0, (ptrdiff_t)dst_w * px, s);
}

int mi_dsp_mc_scaled(int prep, int filter2d, void *dst, ptrdiff_t dst_stride, const void *src, ptrdiff_t src_stride,
                     int w, int h, int mx, int my, int dx, int dy, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !dst || !src || filter2d < 0 || filter2d > 9 || !mc_dims_ok(w, h) || mx < 0 || mx >= 1024 || my < 0 ||
        my >= 1024 || dx < 1 || dy < 1 || dx > 2048 || dy > 2048)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    const int px = bpc == 8 ? 1 : 2;
    hipStream_t s = g_call.stream;
    // source reach: rows -3 .. ((h-1)*dy + my >> 10) + 4, columns -3 .. ((w-1)*dx + mx >> 10) + 4
    const int r0 = -3, r1 = (((h - 1) * dy + my) >> 10) + 5;
    const ptrdiff_t b0 = -3 * px, b1 = (ptrdiff_t)((((w - 1) * dx + mx) >> 10) + 5) * px;
    if ((size_t)(r1 - r0) * (b1 - b0) > (1u << 19)) return -EINVAL;
    uint8_t *win = g_call.scratch, *dout = win + (1 << 19);
    if (int e = win_in(win, src, src_stride, r0, r1, b0, b1, s)) return e;
    mi::McCallArgs a;
    memset(&a, 0, sizeof(a));
    a.src = win + (size_t)(-r0) * (b1 - b0) - b0;
    a.src_stride = b1 - b0;
    a.dst = dout;
    a.dst_stride = (int64_t)w * px;
    a.tmp1 = (int16_t *)dout;
    a.prep = prep;
    a.w = w; a.h = h; a.mx = mx; a.my = my; a.dx = dx; a.dy = dy; a.filter2d = filter2d;
    mc_call_bd(a, bpc, bitdepth_max);
    if (mi::launch_mc_call(a, 5, s)) return -EIO;
    if (prep) {
        if (hipMemcpyAsync(dst, dout, (size_t)w * h * 2, hipMemcpyDefault, s) != hipSuccess) return -EIO;
        return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO;
    }
    return win_out(dst, dst_stride, dout, 0, h, 0, (ptrdiff_t)w * px, s);
}

// ---- lr table (src/looprestoration.rs:91-107): wiener, sgr[kind] on one unit ----
namespace {
// Stage the unit's pixels (columns 0 .. w + 3*have_right), the lpf rows 0, 1, 6, 7 (columns
// -3*have_left .. w + 3*have_right) and left[h][4] into one pitch-P buffer (column 3 = x 0),
// filter, and write the w x h result back over p.
int lr_call(mi::LrCallArgs &a, void *p, ptrdiff_t stride, const void *left, const void *lpf, int w, int h,
            int edges, int bitdepth_max, int bpc) {
    const int px = bpc == 8 ? 1 : 2;
    const bool hl = edges & 1, hr = edges & 2, ht = edges & 4, hb = edges & 8;
    if ((hl && !left) || ((ht || hb) && !lpf)) return -EINVAL;
    hipStream_t s = g_call.stream;
    const ptrdiff_t P = (ptrdiff_t)(w + 6) * px;
    uint8_t *dp = g_call.scratch, *dlpf = dp + 64 * P, *dleft = dlpf + 8 * P, *dout = dleft + 64 * 4 * 2;
    auto rows = [&](uint8_t *dst, const void *src, int r, ptrdiff_t c0, ptrdiff_t c1) -> int {
        return hipMemcpyAsync(dst + r * P + 3 * px + c0, (const uint8_t *)src + r * stride + c0, c1 - c0,
                              hipMemcpyDefault, s) == hipSuccess ? 0 : -EIO;
    };
    const ptrdiff_t c1 = (ptrdiff_t)(w + (hr ? 3 : 0)) * px, lc0 = hl ? -3 * px : 0;
    int e = 0;
    for (int r = 0; r < h && !e; r++) e = rows(dp, p, r, 0, c1);
    if (ht) for (int r = 0; r < 2 && !e; r++) e = rows(dlpf, lpf, r, lc0, c1);
    if (hb) for (int r = 6; r < 8 && !e; r++) e = rows(dlpf, lpf, r, lc0, c1);
    if (!e && hl) e = copy_in(dleft, left, (size_t)h * 4 * px, s);
    if (e) return e;
    a.p = dp + 3 * px;
    a.lpf = dlpf + 3 * px;
    a.left = dleft;
    a.out = dout;
    a.ps = P / px;
    a.w = w;
    a.h = h;
    a.edges = edges;
    a.bd = bpc;
    (void)bitdepth_max;
    if (mi::launch_lr_call(a, bpc, s)) return -EIO;
    return win_out(p, stride, dout, 0, h, 0, (ptrdiff_t)w * px, s);
}
bool lr_dims_ok(int w, int h) { return w >= 1 && w <= 384 && h >= 1 && h <= 64; }
}  // namespace

int mi_dsp_lr_wiener(void *p, ptrdiff_t stride, const void *left, const void *lpf, int w, int h, const void *params,
                     int edges, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !p || !params || !lr_dims_ok(w, h) || edges < 0 || edges > 15) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    int16_t f[2][8];
    if (hipMemcpy(f, params, sizeof(f), hipMemcpyDefault) != hipSuccess) return -EIO;
    mi::LrCallArgs a;
    memset(&a, 0, sizeof(a));
    a.tp.wiener = true;
    for (int k = 0; k < 7; k++) { a.tp.fh[k] = f[0][k]; a.tp.fv[k] = f[1][k]; }
    if (bpc == 8) a.tp.fh[3] += 128;   // the reference adds the 8-bit centre tap separately
    return lr_call(a, p, stride, left, lpf, w, h, edges, bitdepth_max, bpc);
}

int mi_dsp_lr_sgr(int kind, void *p, ptrdiff_t stride, const void *left, const void *lpf, int w, int h,
                  const void *params, int edges, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || kind < 0 || kind > 2 || !p || !params || !lr_dims_ok(w, h) || edges < 0 || edges > 15) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    struct { uint32_t s0, s1; int16_t w0, w1; } sp;   // LooprestorationParams_sgr
    if (hipMemcpy(&sp, params, sizeof(sp), hipMemcpyDefault) != hipSuccess) return -EIO;
    mi::LrCallArgs a;
    memset(&a, 0, sizeof(a));
    a.tp.wiener = false;
    a.tp.s0 = kind != 1 ? (int)sp.s0 : 0;
    a.tp.s1 = kind != 0 ? (int)sp.s1 : 0;
    a.tp.w0 = sp.w0;
    a.tp.w1 = sp.w1;
    if ((kind != 1 && !a.tp.s0) || (kind != 0 && !a.tp.s1)) return -EINVAL;
    return lr_call(a, p, stride, left, lpf, w, h, edges, bitdepth_max, bpc);
}


// ---- film-grain table (src/filmgrain.rs:41-198): generate_grain_y / _uv, fgy / fguv_32x32xn ----
namespace {
constexpr int kGW = 82, kGH = 73, kGP = 88;   // template width / height, device pitch (fg.hip)
constexpr size_t kFgLutB = 3 * kGH * kGP * 2, kFgSclB = 3 * 4096;
size_t al256(size_t n) { return (n + 255) & ~(size_t)255; }

int fg_read_data(MiFilmGrainData &d, const MiFilmGrainData *data) {
    if (hipMemcpy(&d, data, sizeof(d), hipMemcpyDefault) != hipSuccess) return -EIO;
    return fg_data_ok(&d) ? 0 : -EINVAL;
}
// caller's GrainLut<Entry> rows (82 entries: int8 at 8 bits, int16 above) <-> int16 [73][82]
int fg_lut_read(int16_t *t, const void *buf, int bpc) {
    if (bpc == 8) {
        int8_t b[kGH * kGW];
        if (hipMemcpy(b, buf, sizeof(b), hipMemcpyDefault) != hipSuccess) return -EIO;
        for (int i = 0; i < kGH * kGW; i++) t[i] = b[i];
        return 0;
    }
    return hipMemcpy(t, buf, kGH * kGW * 2, hipMemcpyDefault) == hipSuccess ? 0 : -EIO;
}
int fg_lut_write(void *buf, const int16_t *t, int bpc) {
    if (bpc == 8) {
        int8_t b[kGH * kGW];
        for (int i = 0; i < kGH * kGW; i++) b[i] = (int8_t)t[i];
        return hipMemcpy(buf, b, sizeof(b), hipMemcpyDefault) == hipSuccess ? 0 : -EIO;
    }
    return hipMemcpy(buf, t, kGH * kGW * 2, hipMemcpyDefault) == hipSuccess ? 0 : -EIO;
}
// run the template generator and fetch plane pl's template into t [73][82]
int fg_generate(mi::FgArgs &a, int pl, int16_t *t) {
    hipStream_t s = g_call.stream;
    a.lut = (int16_t *)g_call.scratch;
    a.scaling = g_call.scratch + kFgLutB;
    if (mi::launch_fg(a, s, true, false)) return -EIO;
    static int16_t dev[kGH * kGP];
    if (hipMemcpyAsync(dev, a.lut + pl * kGH * kGP, sizeof(dev), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    for (int r = 0; r < kGH; r++) memcpy(t + r * kGW, dev + r * kGP, kGW * 2);
    return 0;
}
// the caller's template -> device slot pl (pitch 88)
int fg_lut_in(int16_t *dlut, int pl, const void *grain_lut, int bpc, hipStream_t s) {
    static int16_t t[kGH * kGW], dev[kGH * kGP];
    if (int e = fg_lut_read(t, grain_lut, bpc)) return e;
    memset(dev, 0, sizeof(dev));
    for (int r = 0; r < kGH; r++) memcpy(dev + r * kGP, t + r * kGW, kGW * 2);
    if (hipMemcpyAsync(dlut + pl * kGH * kGP, dev, sizeof(dev), hipMemcpyHostToDevice, s) != hipSuccess) return -EIO;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO;   // dev is reused
}
int layout_ok(int layout) { return layout >= 1 && layout <= 3; }

// fgy (plane 0) / fguv (plane 1 + uv): one 32-row strip through the frame apply kernel
int fg_strip(int pl, int layout, void *dst_row, const void *src_row, ptrdiff_t stride, const MiFilmGrainData *data,
             size_t pw, const uint8_t *scaling, const void *grain_lut, int bh, int row_num, const void *luma_row,
             ptrdiff_t luma_stride, int is_id, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    const int sx = pl && layout != 3, sy = pl && layout == 1;
    if (!bpc || !dst_row || !src_row || !data || !scaling || !grain_lut || (pl && (!luma_row || !layout_ok(layout))) ||
        pw < 1 || pw > 8192 || bh < 1 || bh > (32 >> sy) || row_num < 0)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    if (int e = fg_tables()) return e;
    mi::FgArgs a;
    memset(&a, 0, sizeof(a));
    if (int e = fg_read_data(a.data, data)) return e;
    const int px = bpc == 8 ? 1 : 2;
    const size_t P = al256(pw * px), lw = pw << sx, LP = al256(lw * px);
    const int lrows = pl ? ((bh - 1) << sy) + 1 : 0;
    const int nblocks = (int)((pw + (32 >> sx) - 1) / (32 >> sx));
    const size_t o_scl = kFgLutB, o_off = o_scl + kFgSclB, o_src = o_off + al256(2 * nblocks),
                 o_luma = o_src + P * bh, total = o_luma + LP * lrows;
    if (int e = g_call.reserve(total)) return e;
    hipStream_t s = g_call.stream;
    uint8_t *S = g_call.scratch;
    a.lut = (int16_t *)S;
    a.scaling = S + o_scl;
    a.offsets = S + o_off;
    if (int e = fg_lut_in(a.lut, pl, grain_lut, bpc, s)) return e;
    int e = copy_in(a.scaling + pl * 4096, scaling, (size_t)1 << bpc, s);
    if (!e && pl) e = copy_in(a.scaling, scaling, (size_t)1 << bpc, s);   // the slot read under chroma_scaling_from_luma
    for (int r = 0; r < bh && !e; r++)
        if (hipMemcpyAsync(S + o_src + r * P, (const uint8_t *)src_row + r * stride, pw * px, hipMemcpyDefault, s) !=
            hipSuccess)
            e = -EIO;
    for (int y = 0; pl && y < bh && !e; y++)
        if (hipMemcpyAsync(S + o_luma + (size_t)(y << sy) * LP, (const uint8_t *)luma_row + (y << sy) * luma_stride,
                           lw * px, hipMemcpyDefault, s) != hipSuccess)
            e = -EIO;
    if (e) return e;
    a.bpc = bpc;
    a.layout = pl ? layout : 0;
    a.ss_x = pl && layout != 3;
    a.ss_y = pl && layout == 1;
    a.w = (int)lw;
    a.h = bh << sy;
    a.is_id = is_id;
    const bool prev = a.data.overlap_flag && row_num > 0;
    a.nrows = prev ? 2 : 1;
    a.row0 = prev ? row_num - 1 : row_num;
    a.row_off = prev ? 1 : 0;
    a.nblocks = nblocks;
    a.src[0] = S + (pl ? o_luma : o_src);
    a.stride[0] = pl ? (int64_t)LP : (int64_t)P;
    a.src[pl] = S + o_src;
    a.dst[pl] = S + o_src;
    a.stride[pl] = (int64_t)P;
    a.pw[pl] = (int)pw;
    a.ph[pl] = bh;
    a.chunks[pl] = (int)((pw + 511) / 512);
    a.grain[pl] = 1;
    const int nb = (a.chunks[pl] * bh + 4 * mi::kFgItems - 1) / (4 * mi::kFgItems);
    for (int q = 0; q < 4; q++) a.blk_start[q] = q <= pl ? 0 : nb;
    if (mi::launch_fg_call(a, s)) return -EIO;
    for (int r = 0; r < bh && !e; r++)
        if (hipMemcpyAsync((uint8_t *)dst_row + r * stride, S + o_src + r * P, pw * px, hipMemcpyDefault, s) != hipSuccess)
            e = -EIO;
    if (hipStreamSynchronize(s) != hipSuccess) return -EIO;
    return e;
}
}  // namespace

int mi_dsp_fg_generate_grain_y(void *buf, const MiFilmGrainData *data, int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !buf || !data) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    if (int e = fg_tables()) return e;
    mi::FgArgs a;
    memset(&a, 0, sizeof(a));
    if (int e = fg_read_data(a.data, data)) return e;
    a.bpc = bpc;
    static int16_t t[kGH * kGW];
    if (int e = fg_generate(a, 0, t)) return e;
    return fg_lut_write(buf, t, bpc);
}

int mi_dsp_fg_generate_grain_uv(int layout, void *buf, const void *buf_y, const MiFilmGrainData *data, int uv,
                                int bitdepth_max) {
    const int bpc = bpc_of(bitdepth_max);
    if (!bpc || !layout_ok(layout) || !buf || !buf_y || !data || uv < 0 || uv > 1) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_call.mu);
    if (int e = g_call.init()) return e;
    if (int e = fg_tables()) return e;
    mi::FgArgs a;
    memset(&a, 0, sizeof(a));
    if (int e = fg_read_data(a.data, data)) return e;
    static int16_t ty[kGH * kGW], t[kGH * kGW], out[kGH * kGW];
    if (int e = fg_lut_read(ty, buf_y, bpc)) return e;
    int16_t *dly = (int16_t *)(g_call.scratch + kFgLutB + kFgSclB);
    if (hipMemcpy(dly, ty, sizeof(ty), hipMemcpyHostToDevice) != hipSuccess) return -EIO;
    a.bpc = bpc;
    a.layout = layout;
    a.ss_x = layout != 3;
    a.ss_y = layout == 1;
    a.lut_y = dly;
    a.uv_only = 1 + uv;
    if (int e = fg_generate(a, 1 + uv, t)) return e;
    // only the chroma template's own cw x chh corner is written, as the reference does
    if (int e = fg_lut_read(out, buf, bpc)) return e;
    const int cw = a.ss_x ? 44 : kGW, chh = a.ss_y ? 38 : kGH;
    for (int r = 0; r < chh; r++) memcpy(out + r * kGW, t + r * kGW, cw * 2);
    return fg_lut_write(buf, out, bpc);
}

int mi_dsp_fgy_32x32xn(void *dst_row, const void *src_row, ptrdiff_t stride, const MiFilmGrainData *data, size_t pw,
                       const uint8_t *scaling, const void *grain_lut, int bh, int row_num, int bitdepth_max) {
    return fg_strip(0, 0, dst_row, src_row, stride, data, pw, scaling, grain_lut, bh, row_num, nullptr, 0, 0,
                    bitdepth_max);
}

int mi_dsp_fguv_32x32xn(int layout, void *dst_row, const void *src_row, ptrdiff_t stride,
                        const MiFilmGrainData *data, size_t pw, const uint8_t *scaling, const void *grain_lut, int bh,
                        int row_num, const void *luma_row, ptrdiff_t luma_stride, int uv_pl, int is_id,
                        int bitdepth_max) {
    if (uv_pl < 0 || uv_pl > 1) return -EINVAL;
    return fg_strip(1 + uv_pl, layout, dst_row, src_row, stride, data, pw, scaling, grain_lut, bh, row_num, luma_row,
                    luma_stride, is_id, bitdepth_max);
}

}  // extern "C"
} // extern "C"

namespace mi_internal {

// mi_intra_recon, and the strip form frame_exec.cpp uses for a single frame: with nstrips > 1
// the frame's blocks are grouped by strip (strip q = blocks [strip_start[q], strip_start[q+1]),
// each in dependency order), deps index the whole frame, and queue q (strip q) runs on XCD q.
int intra_recon(MiCtx *ctx, const MiIntraFrame *frames, int nframes, const int32_t *strip_start, int nstrips,
                unsigned flags, void *stream, bool granules) {
    if (!ctx || !frames || nframes < 1 || nframes > mi::kIrMaxFrames) return fail(ctx, -EINVAL);
    if (nstrips > 1 && (nframes != 1 || nstrips > 8 || !strip_start)) return fail(ctx, -EINVAL);
    const int bpc = frames[0].pic.bpc;
    if (bpc != 8 && bpc != 10 && bpc != 12) return fail(ctx, -EINVAL);
    size_t total = 0;
    for (int f = 0; f < nframes; f++) {
        const MiIntraFrame &fr = frames[f];
        if (fr.pic.bpc != bpc || fr.n < 0 || (fr.n && (!fr.blocks || !fr.tx || !fr.dep_start || !fr.coef)))
            return fail(ctx, -EINVAL);
        total += (size_t)fr.n;
    }
    if (nstrips > 1)
        for (int q = 0; q < nstrips; q++)
            if (strip_start[0] != 0 || strip_start[q + 1] < strip_start[q] || strip_start[nstrips] != frames[0].n)
                return fail(ctx, -EINVAL);
    if (int e = ctx_words(ctx, (hipStream_t)stream)) return fail(ctx, e);
    if (total > ctx->ir_done_n) {
        // an earlier launch on this context's stream may still poll the old flags
        if (ctx->ir_done && hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return fail(ctx, -EIO);
        if (ctx->ir_done) (void)hipFree(ctx->ir_done);
        ctx->ir_done = nullptr;
        ctx->ir_done_n = 0;
        if (hipMalloc(&ctx->ir_done, total * sizeof(uint32_t)) != hipSuccess) return fail(ctx, -ENOMEM);
        // stream-ordered, as ctx_words
        if (hipMemsetAsync(ctx->ir_done, 0, total * sizeof(uint32_t), (hipStream_t)stream) != hipSuccess)
            return fail(ctx, -EIO);
        ctx->ir_done_n = total;
    }
    if (++ctx->ir_epoch == 0) ctx->ir_epoch = 1;   // done words hold the epoch of the last call
    hipStream_t s = (hipStream_t)stream;
    mi::IntraReconArgs a;
    memset(&a, 0, sizeof(a));
    // edge granules: one region per frame (mi::gran_count), zeroed once when (re)allocated
    std::vector<uint32_t> goff(nframes, 0);
    if (granules) {
        size_t ng = 0;
        for (int f = 0; f < nframes; f++) {
            const MiPicture &pic = frames[f].pic;
            goff[f] = (uint32_t)ng;
            ng += mi::gran_count((pic.w + 127) & ~127, (pic.h + 127) & ~127, pic.layout == 1 || pic.layout == 2,
                                 pic.layout == 1, pic.layout ? 3 : 1);
        }
        if (ng > 0xffffffffull) return fail(ctx, -EINVAL);
        if (ng > ctx->ir_gran_n) {
            if (ctx->ir_gran && hipStreamSynchronize(s) != hipSuccess) return fail(ctx, -EIO);
            if (ctx->ir_gran) (void)hipFree(ctx->ir_gran);
            ctx->ir_gran = nullptr;
            ctx->ir_gran_n = 0;
            if (hipMalloc((void **)&ctx->ir_gran, ng * 8) != hipSuccess) return fail(ctx, -ENOMEM);
            if (hipMemsetAsync(ctx->ir_gran, 0, ng * 8, s) != hipSuccess) return fail(ctx, -EIO);
            ctx->ir_gran_n = ng;
        }
        a.gran = ctx->ir_gran;
    }
    const int nq = nstrips > 1 ? nstrips : nframes;
    size_t off = 0;
    for (int q = 0; q < nq; q++) {
        const MiIntraFrame &fr = frames[nstrips > 1 ? 0 : q];
        const int s0 = nstrips > 1 ? strip_start[q] : 0;
        mi::IntraReconFrame &d = a.fr[q];
        for (int p = 0; p < 3; p++) d.ip.dst[p] = (uint8_t *)fr.pic.data[p];
        d.ip.stride[0] = fr.pic.stride[0];
        d.ip.stride[1] = fr.pic.stride[1];
        d.ip.iblocks = fr.blocks + s0;
        d.ip.ac = fr.ac;
        d.ip.idx = fr.idx;
        d.ip.pal = (const uint8_t *)fr.pal;
        d.ip.bpc = bpc;
        d.ip.bdmax = (1 << bpc) - 1;
        d.tx = fr.tx + s0;
        d.coef = (uint8_t *)fr.coef;
        d.dep_start = fr.dep_start + s0;
        d.deps = fr.deps;
        d.done = ctx->ir_done + off;
        d.base = s0;
        d.head = ctx->ir_words + q;
        d.n = nstrips > 1 ? strip_start[q + 1] - s0 : fr.n;
        d.pw = (uint16_t)((fr.pic.w + 127) & ~127);
        d.ph = (uint16_t)((fr.pic.h + 127) & ~127);
        d.ss_hor = fr.pic.layout == 1 || fr.pic.layout == 2;
        d.ss_ver = fr.pic.layout == 1;
        d.nplanes = fr.pic.layout ? 3 : 1;
        d.goff = goff[nstrips > 1 ? 0 : q];
        if (nstrips <= 1) off += (size_t)fr.n;
    }
    // queue heads and XCD worker ranks start from 0 in stream order
    if (hipMemsetAsync(ctx->ir_words, 0, 64 * sizeof(int), s) != hipSuccess ||
        hipMemsetAsync(ctx->ir_words + 72, 0, 8 * sizeof(int), s) != hipSuccess)
        return fail(ctx, -EIO);
    a.xcd_rank = ctx->ir_words + 72;
    a.err = ctx->ir_words + 64;
    a.desc_err = ctx->ir_words + 65;
#ifdef MI_IR_DEBUG
    static int *dbg = nullptr;
    if (!dbg && hipHostMalloc((void **)&dbg, 65536 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return fail(ctx, -ENOMEM);
    memset(dbg, 0, 65536 * sizeof(int));
    int *ddbg = nullptr;
    (void)hipHostGetDevicePointer((void **)&ddbg, dbg, 0);
    a.dbg = ddbg;
    setenv("MI_IR_DBG_PTR", std::to_string((uintptr_t)dbg).c_str(), 1);
#endif
    static const bool tl_env = getenv("MI_IR_TIMELINE") != nullptr;
    if (tl_env) {
        if (ctx->ir_tl_n < ctx->ir_done_n) {
            if (ctx->ir_tl) (void)hipFree(ctx->ir_tl);
            ctx->ir_tl = nullptr;
            ctx->ir_tl_n = 0;
            if (hipMalloc((void **)&ctx->ir_tl, ctx->ir_done_n * 128) != hipSuccess) return fail(ctx, -ENOMEM);
            ctx->ir_tl_n = ctx->ir_done_n;
        }
        a.tl = (uintptr_t)ctx->ir_tl - (uintptr_t)ctx->ir_done * 32;
    }
    a.epoch = ctx->ir_epoch;
    a.nframes = nq;
    a.zero_coefs = (flags & MI_ITX_KEEP_COEFS) ? 0 : 1;
    // one-wave workers per XCD (VGPRs allow 2 per SIMD = 256 per XCD, LDS 7 per CU): one per
    // ~96 units of the busiest XCD's first queue, 128 to 192 (a worker that arrives after its
    // block's producer finished adds to the chain: 4K intra frames gain 25 % from 128 to 192;
    // 352x288 frames lose 15 % at 64), plus 64 per extra queue the XCD serves
    const int per_xcd = (nq + 7) / 8;
    int n_xcd = 0;
    for (int q = 0; q < nq && q < 8; q++) n_xcd = std::max(n_xcd, a.fr[q].n);
    const int wpx = std::min(256, std::max(128, std::min(192, n_xcd / 96)) + 64 * (per_xcd - 1));
    return mi::launch_intra_recon(a, bpc, wpx, s) ? fail(ctx, -EIO) : 0;
}

}  // namespace mi_internal
