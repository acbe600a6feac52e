// output.cpp — displayed pictures from the device to the host (include/mi_av1out.h).
//
// rav1d hands the caller a picture with film grain applied on the fly (src/lib.rs
// output_picture_ready -> rav1d_apply_grain, src/fg_apply.rs:272-284); the CPU decoder's
// pictures already live in host memory. Here the reconstructed picture lives in HBM, so the
// output step is also the device-to-host transfer: the grain kernel (fg.hip) stores its result
// straight into pinned, device-mapped host memory, one pass over the picture instead of a
// grain pass into HBM followed by a copy. Without grain the visible area is copied by DMA.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstring>

#include "mi_av1out.h"

namespace {

// dav1d's default-allocator geometry (src/picture.rs:98-115), as the device pictures use
void geometry(int w, int h, int layout, int bpc, ptrdiff_t stride[2], size_t rows[2]) {
    const int pxb = bpc == 8 ? 1 : 2, ss_hor = layout == 1 || layout == 2, ss_ver = layout == 1;
    const int aw = (w + 127) & ~127, ah = (h + 127) & ~127;
    stride[0] = (ptrdiff_t)aw * pxb;
    if (stride[0] % 1024 == 0) stride[0] += 64;
    stride[1] = (ptrdiff_t)(aw >> ss_hor) * pxb;
    if (stride[1] % 1024 == 0) stride[1] += 64;
    rows[0] = (size_t)ah;
    rows[1] = (size_t)(ah >> ss_ver);
}

bool valid(const MiPicture *p) {
    return p && p->data[0] && p->w > 0 && p->h > 0 && p->layout >= 0 && p->layout <= 3 &&
           (p->bpc == 8 || p->bpc == 10 || p->bpc == 12) && (!p->layout || (p->data[1] && p->data[2]));
}

}  // namespace

extern "C" {

int mi_host_picture_alloc(int w, int h, int layout, int bpc, MiPicture *pic) {
    if (!pic || w <= 0 || h <= 0 || w > 65536 || h > 65536 || layout < 0 || layout > 3 ||
        (bpc != 8 && bpc != 10 && bpc != 12))
        return -EINVAL;
    memset(pic, 0, sizeof(*pic));
    ptrdiff_t stride[2];
    size_t rows[2];
    geometry(w, h, layout, bpc, stride, rows);
    const size_t ybytes = ((size_t)stride[0] * rows[0] + 63) & ~(size_t)63;
    const size_t cbytes = layout ? ((size_t)stride[1] * rows[1] + 63) & ~(size_t)63 : 0;
    void *mem = nullptr;
    // pinned + mapped: kernels store into it over PCIe, the host reads it after a sync
    if (hipHostMalloc(&mem, ybytes + 2 * cbytes, hipHostMallocMapped) != hipSuccess || !mem) return -ENOMEM;
    uint8_t *b = (uint8_t *)mem;
    pic->data[0] = b;
    pic->data[1] = layout ? b + ybytes : nullptr;
    pic->data[2] = layout ? b + ybytes + cbytes : nullptr;
    pic->stride[0] = stride[0];
    pic->stride[1] = stride[1];
    pic->w = w;
    pic->h = h;
    pic->layout = layout;
    pic->bpc = bpc;
    return 0;
}

void mi_host_picture_free(MiPicture *pic) {
    if (!pic || !pic->data[0]) return;
    (void)hipHostFree(pic->data[0]);
    memset(pic, 0, sizeof(*pic));
}

int mi_output_picture(MiCtx *ctx, const MiPicture *in, const MiPicture *out, const MiFilmGrainData *fg,
                      int mtrx_identity, void *stream) {
    if (!ctx || !valid(in) || !valid(out)) return -EINVAL;
    if (in->w != out->w || in->h != out->h || in->layout != out->layout || in->bpc != out->bpc ||
        in->stride[0] != out->stride[0] || in->stride[1] != out->stride[1])
        return -EINVAL;
    if (fg) return mi_film_grain_frame(ctx, in, out, fg, mtrx_identity, stream);
    hipStream_t s = (hipStream_t)stream;
    const int hbd = in->bpc > 8, ss_hor = in->layout == 1 || in->layout == 2, ss_ver = in->layout == 1;
    for (int p = 0; p < (in->layout ? 3 : 1); p++) {
        const int pw = p ? (in->w + ss_hor) >> ss_hor : in->w, ph = p ? (in->h + ss_ver) >> ss_ver : in->h;
        const size_t st = (size_t)in->stride[p ? 1 : 0];
        if (hipMemcpy2DAsync(out->data[p], st, in->data[p], st, (size_t)pw << hbd, (size_t)ph,
                             hipMemcpyDeviceToHost, s) != hipSuccess)
            return -EIO;
    }
    return 0;
}

}  // extern "C"
