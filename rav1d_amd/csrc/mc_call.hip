// mc_call.hip — single-call motion-compensation kernels behind the table-compatible entry
// points (mi_dsp_mc_*): mc[10] / mct[10] (8-tap and bilinear put / prep), avg, w_avg, mask,
// w_mask[3], blend, blend_v, blend_h, warp8x8 / warp8x8t, emu_edge, resize and mc_scaled /
// mct_scaled of Rav1dMCDSPContext (rav1d src/mc.rs:
// 1174-1338; C src/mc_tmpl.c:52-845). One lane per output pixel (per mask sample for
// w_mask); the per-call path exists for drop-in parity, the frame path is mc.hip.
#include "common.h"

namespace mi {

__constant__ int8_t k_subpel_c[6][15][8] = {
#include "tables/mc_subpel_filters.inc"
};
__constant__ uint8_t k_obmc_c[64] = {
#include "tables/obmc_masks.inc"
};
__constant__ int8_t k_warp_c[193][8] = {
#include "tables/mc_warp_filter.inc"
};
__constant__ int8_t k_resize_c[64][8] = {
#include "tables/resize_filter.inc"
};

__device__ __forceinline__ int rnd_c(int v, int sh) { return (v + ((1 << sh) >> 1)) >> sh; }
__device__ __forceinline__ int clip_c(int v, int lo, int hi) { return min(max(v, lo), hi); }

template <typename Px>
__device__ __forceinline__ int ld(const uint8_t *p, int64_t stride, int y, int x) {
    return reinterpret_cast<const Px *>(p + y * stride)[x];
}
template <typename Px>
__device__ __forceinline__ void st(uint8_t *p, int64_t stride, int y, int x, int v) {
    reinterpret_cast<Px *>(p + y * stride)[x] = (Px)v;
}

// filter2d -> (type_h, type_v): 0 regular, 1 smooth, 2 sharp; w / h <= 4 use the 4-tap sets
__device__ __forceinline__ const int8_t *sub_h(int f2d, int mx, int w) {
    const int t = (int)((0x111222000ull >> (4 * f2d)) & 15);
    return !mx ? nullptr : w > 4 ? k_subpel_c[t][mx - 1] : k_subpel_c[3 + (t & 1)][mx - 1];
}
__device__ __forceinline__ const int8_t *sub_v(int f2d, int my, int h) {
    const int t = (int)((0x210210210ull >> (4 * f2d)) & 15);
    return !my ? nullptr : h > 4 ? k_subpel_c[t][my - 1] : k_subpel_c[3 + (t & 1)][my - 1];
}

template <typename Px>
__global__ __launch_bounds__(256) void mc_call_pp_kernel(McCallArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.w * a.h) return;
    const int y = i / a.w, x = i % a.w, ib = a.ib, bias = a.bias;
    const uint8_t *s = a.src;
    const int64_t ss = a.src_stride;
    int out;            // put: the pixel; prep: the int16 intermediate
    if (a.filter2d == 9) {            // bilinear (mc_tmpl.c:380-500)
        auto bil = [&](int yy, int xx, int m, int dy, int dx) {
            const int p = ld<Px>(s, ss, yy, xx);
            return 16 * p + m * (ld<Px>(s, ss, yy + dy, xx + dx) - p);
        };
        if (a.mx && a.my) {
            const int m0 = rnd_c(bil(y, x, a.mx, 0, 1), 4 - ib), m1 = rnd_c(bil(y + 1, x, a.mx, 0, 1), 4 - ib);
            const int v = 16 * m0 + a.my * (m1 - m0);
            out = a.prep ? rnd_c(v, 4) - bias : clip_c(rnd_c(v, 4 + ib), 0, a.bdmax);
        } else if (a.mx) {
            const int p = rnd_c(bil(y, x, a.mx, 0, 1), 4 - ib);
            out = a.prep ? p - bias : clip_c((p + ((1 << ib) >> 1)) >> ib, 0, a.bdmax);
        } else if (a.my) {
            const int v = bil(y, x, a.my, 1, 0);
            out = a.prep ? rnd_c(v, 4 - ib) - bias : clip_c(rnd_c(v, 4), 0, a.bdmax);
        } else {
            const int p = ld<Px>(s, ss, y, x);
            out = a.prep ? (p << ib) - bias : p;
        }
    } else {                          // 8-tap (mc_tmpl.c:100-290)
        const int8_t *fh = sub_h(a.filter2d, a.mx, a.w), *fv = sub_v(a.filter2d, a.my, a.h);
        auto hsum = [&](int yy) {
            int v = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) v += fh[k] * ld<Px>(s, ss, yy, x + k - 3);
            return v;
        };
        if (fh && fv) {
            int v = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) v += fv[k] * rnd_c(hsum(y + k - 3), 6 - ib);
            out = a.prep ? rnd_c(v, 6) - bias : clip_c(rnd_c(v, 6 + ib), 0, a.bdmax);
        } else if (fh) {
            const int v = hsum(y);
            out = a.prep ? rnd_c(v, 6 - ib) - bias : clip_c((v + 32 + ((1 << (6 - ib)) >> 1)) >> 6, 0, a.bdmax);
        } else if (fv) {
            int v = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) v += fv[k] * ld<Px>(s, ss, y + k - 3, x);
            out = a.prep ? rnd_c(v, 6 - ib) - bias : clip_c(rnd_c(v, 6), 0, a.bdmax);
        } else {
            const int p = ld<Px>(s, ss, y, x);
            out = a.prep ? (p << ib) - bias : p;
        }
    }
    if (a.prep) a.tmp1[y * a.w + x] = (int16_t)out;
    else st<Px>(a.dst, a.dst_stride, y, x, out);
}

// avg (op 0), w_avg (1), mask (2), blend (4), blend_v (5), blend_h (6): one lane per pixel;
// w_mask (3): one lane per mask sample (its 1, 2 or 4 pixels)
template <typename Px>
__global__ __launch_bounds__(256) void mc_call_comb_kernel(McCallArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int w = a.w, h = a.h, ib = a.ib, bias = a.bias;
    if (a.op == 3) {
        const int mw = w >> a.ss_hor, mh = h >> a.ss_ver;
        if (i >= mw * mh) return;
        const int my = i / mw, mx = i % mw;
        const int sh = ib + 6, r = (32 << ib) + bias * 64;
        const int mask_sh = a.bpc + ib - 4, mask_rnd = 1 << (mask_sh - 5);
        int msum = 0;
        for (int dy = 0; dy <= a.ss_ver; dy++)
            for (int dx = 0; dx <= a.ss_hor; dx++) {
                const int y = (my << a.ss_ver) + dy, x = (mx << a.ss_hor) + dx;
                const int t1 = a.tmp1[y * w + x], t2 = a.tmp2[y * w + x];
                const int m = min(38 + ((abs(t1 - t2) + mask_rnd) >> mask_sh), 64);
                st<Px>(a.dst, a.dst_stride, y, x, clip_c((t1 * m + t2 * (64 - m) + r) >> sh, 0, a.bdmax));
                msum += m;
            }
        // w_mask_420: (m + n + m' + n' + 2 - sign) >> 2; _422: (m + n + 1 - sign) >> 1; _444: m
        const int v = a.ss_ver ? (msum + 2 - a.sign) >> 2 : a.ss_hor ? (msum + 1 - a.sign) >> 1 : msum;
        a.mask_out[my * mw + mx] = (uint8_t)v;
        return;
    }
    if (i >= w * h) return;
    const int y = i / w, x = i % w;
    if (a.op >= 4) {
        int m;
        if (a.op == 4) m = a.mask[y * w + x];
        else if (a.op == 5) { if (x >= (w * 3) >> 2) return; m = k_obmc_c[w + x]; }
        else { if (y >= (h * 3) >> 2) return; m = k_obmc_c[h + y]; }
        const int d = ld<Px>(a.dst, a.dst_stride, y, x);
        const int t = reinterpret_cast<const Px *>(a.src)[y * w + x];
        st<Px>(a.dst, a.dst_stride, y, x, (d * (64 - m) + t * m + 32) >> 6);
        return;
    }
    const int t1 = a.tmp1[y * w + x], t2 = a.tmp2[y * w + x];
    int v;
    if (a.op == 0) v = (t1 + t2 + (1 << ib) + bias * 2) >> (ib + 1);
    else if (a.op == 1) v = (t1 * a.weight + t2 * (16 - a.weight) + (8 << ib) + bias * 16) >> (ib + 4);
    else {
        const int m = a.mask[y * w + x];
        v = (t1 * m + t2 * (64 - m) + (32 << ib) + bias * 64) >> (ib + 6);
    }
    st<Px>(a.dst, a.dst_stride, y, x, clip_c(v, 0, a.bdmax));
}

// emu_edge (mc_tmpl.c:798-845): the bw x bh block at (x, y) of an iw x ih reference with
// clamped coordinates; src = the staged clamped rectangle, its origin at (clip(x), clip(y))
template <typename Px>
__global__ __launch_bounds__(256) void mc_call_emu_kernel(McCallArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.w * a.h) return;
    const int yy = i / a.w, xx = i % a.w;
    const int sy = clip_c(a.my + yy, 0, a.ih - 1) - clip_c(a.my, 0, a.ih - 1);
    const int sx = clip_c(a.mx + xx, 0, a.iw - 1) - clip_c(a.mx, 0, a.iw - 1);
    st<Px>(a.dst, a.dst_stride, yy, xx, ld<Px>(a.src, a.src_stride, sy, sx));
}

// put / prep scaled (mc_tmpl.c:201-227, 291-330, 445-470, 528-560): positions in 1/1024 pel,
// step dx / dy; output (y, x) reads source row ((my + y*dy) >> 10) and column
// ((mx + x*dx) >> 10) with filter phases from the low 10 bits (closed form of the reference's
// running position; mx, my < 1024)
template <typename Px>
__global__ __launch_bounds__(256) void mc_call_scaled_kernel(McCallArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.w * a.h) return;
    const int y = i / a.w, x = i % a.w, ib = a.ib, bias = a.bias;
    const int px_ = a.mx + x * a.dx, py_ = a.my + y * a.dy;
    const int ioff = px_ >> 10, imx = px_ & 0x3ff, row = py_ >> 10, imy = py_ & 0x3ff;
    const uint8_t *s = a.src;
    const int64_t ss = a.src_stride;
    int out;
    if (a.filter2d == 9) {
        auto mid = [&](int r) {
            const int p0 = ld<Px>(s, ss, r, ioff), p1 = ld<Px>(s, ss, r, ioff + 1);
            return rnd_c(16 * p0 + (imx >> 6) * (p1 - p0), 4 - ib);
        };
        const int m0 = mid(row), m1 = mid(row + 1);
        const int v = 16 * m0 + (imy >> 6) * (m1 - m0);
        out = a.prep ? rnd_c(v, 4) - bias : clip_c(rnd_c(v, 4 + ib), 0, a.bdmax);
    } else {
        const int8_t *fh = sub_h(a.filter2d, imx >> 6, a.w), *fv = sub_v(a.filter2d, imy >> 6, a.h);
        auto mid = [&](int r) {
            if (!fh) return ld<Px>(s, ss, r, ioff) << ib;
            int v = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) v += fh[k] * ld<Px>(s, ss, r, ioff + k - 3);
            return rnd_c(v, 6 - ib);
        };
        if (fv) {
            int v = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) v += fv[k] * mid(row + k - 3);
            out = a.prep ? rnd_c(v, 6) - bias : clip_c(rnd_c(v, 6 + ib), 0, a.bdmax);
        } else {
            const int m = mid(row);
            out = a.prep ? m - bias : clip_c((m + ((1 << ib) >> 1)) >> ib, 0, a.bdmax);
        }
    }
    if (a.prep) a.tmp1[y * a.w + x] = (int16_t)out;
    else st<Px>(a.dst, a.dst_stride, y, x, out);
}

// warp8x8 / warp8x8t (mc_tmpl.c:714-796): 15 horizontally filtered rows of 8 in LDS (the
// filter phase steps by abcd[0] along x and abcd[1] per row), then the vertical pass (abcd[2]
// along x, abcd[3] per row). src at the block origin, rows / columns -3 .. 11 readable.
template <typename Px>
__global__ __launch_bounds__(64) void mc_call_warp_kernel(McCallArgs a) {
    __shared__ int mid[15 * 8];
    const int lane = threadIdx.x, ib = a.ib;
    for (int i = lane; i < 15 * 8; i += 64) {
        const int y = i >> 3, x = i & 7;
        const int tmx = a.mx + y * a.abcd[1] + x * a.abcd[0];
        const int8_t *F = k_warp_c[64 + ((tmx + 512) >> 10)];
        int v = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) v += F[k] * ld<Px>(a.src, a.src_stride, y - 3, x + k - 3);
        mid[i] = rnd_c(v, 7 - ib);
    }
    __syncthreads();
    const int y = lane >> 3, x = lane & 7;
    const int tmy = a.my + y * a.abcd[3] + x * a.abcd[2];
    const int8_t *F = k_warp_c[64 + ((tmy + 512) >> 10)];
    int v = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) v += F[k] * mid[(y + k) * 8 + x];
    if (a.prep) a.tmp1[y * a.w + x] = (int16_t)(rnd_c(v, 7) - a.bias);
    else st<Px>(a.dst, a.dst_stride, y, x, clip_c(rnd_c(v, 7 + ib), 0, a.bdmax));
}

// resize (mc_tmpl.c:847-875): output x reads source column -1 + ((mx0 + x * dx) >> 14) with
// filter phase ((mx0 + x * dx) & 0x3fff) >> 8, columns clamped to [0, src_w)
template <typename Px>
__global__ __launch_bounds__(256) void mc_call_resize_kernel(McCallArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.w * a.h) return;
    const int y = i / a.w, x = i % a.w;
    const int64_t pos = (int64_t)a.mx + (int64_t)x * a.weight;   // weight: dx
    const int sx = -1 + (int)(pos >> 14), ph = (int)(pos & 0x3fff) >> 8;
    const int8_t *F = k_resize_c[ph];
    int v = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) v += F[k] * ld<Px>(a.src, a.src_stride, y, clip_c(sx - 3 + k, 0, a.iw - 1));
    st<Px>(a.dst, a.dst_stride, y, x, clip_c((-v + 64) >> 7, 0, a.bdmax));
}

int launch_mc_call(const McCallArgs &a, int kind, hipStream_t s) {
    const int n = kind == 1 && a.op == 3 ? (a.w >> a.ss_hor) * (a.h >> a.ss_ver) : a.w * a.h;
    const dim3 g((n + 255) / 256);
    if (kind == 3) {
        if (a.bpc == 8) mc_call_warp_kernel<uint8_t><<<1, 64, 0, s>>>(a);
        else mc_call_warp_kernel<uint16_t><<<1, 64, 0, s>>>(a);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (kind == 5) {
        if (a.bpc == 8) mc_call_scaled_kernel<uint8_t><<<g, 256, 0, s>>>(a);
        else mc_call_scaled_kernel<uint16_t><<<g, 256, 0, s>>>(a);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (kind == 4) {
        if (a.bpc == 8) mc_call_resize_kernel<uint8_t><<<g, 256, 0, s>>>(a);
        else mc_call_resize_kernel<uint16_t><<<g, 256, 0, s>>>(a);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (a.bpc == 8) {
        if (kind == 0) mc_call_pp_kernel<uint8_t><<<g, 256, 0, s>>>(a);
        else if (kind == 1) mc_call_comb_kernel<uint8_t><<<g, 256, 0, s>>>(a);
        else mc_call_emu_kernel<uint8_t><<<g, 256, 0, s>>>(a);
    } else {
        if (kind == 0) mc_call_pp_kernel<uint16_t><<<g, 256, 0, s>>>(a);
        else if (kind == 1) mc_call_comb_kernel<uint16_t><<<g, 256, 0, s>>>(a);
        else mc_call_emu_kernel<uint16_t><<<g, 256, 0, s>>>(a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
