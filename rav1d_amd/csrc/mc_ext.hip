// mc_ext.hip — the less frequent inter-prediction paths on gfx950: scaled references,
// warped motion, compound combine from intermediates, and super-resolution.
//
// Replaces, per frame, the mc() scaled branch (rav1d src/recon.rs:2124-2202) with
// mc_scaled / mct_scaled (src/mc.rs put_8tap_scaled:212, prep_8tap_scaled:351, bilin :496,
// :608; C mc_tmpl.c), warp_affine's warp8x8 / warp8x8t calls (recon.rs:2311-2400; mc.rs
// :885, :962), the avg / w_avg / mask / w_mask step when a side was warped or scaled
// (recon.rs:3292-3331), and rav1d_filter_sbrow_resize's mc.resize (recon.rs:4215-4285;
// mc.rs:1114).
//
// These paths are rare in streams (reference scaling, global/local warp, superres), so the
// kernels favour one simple, divergence-free shape each over the main path's packing:
//   scaled:  one 64-lane workgroup per unit, one lane per output pixel, the 8 intermediate
//            rows it needs filtered in registers (8 x 8 taps + 8 taps); also OBMC laps whose
//            neighbour's reference is scaled (blended like mc_kernel's laps);
//   warp:    four 8x8 blocks per 256-lane workgroup; the 15x15 window and the warp filter
//            table staged in LDS, lane (r, c) filters intermediate rows r and r + 8, then
//            output (r, c);
//   combine: one 64-lane workgroup per unit, lane per pixel (per mask sample for w_mask);
//   resize:  one lane per output pixel, 256 per workgroup along a row.
#include "common.h"

namespace mi {

__constant__ int8_t k_subpel_x[6][15][8] = {
#include "tables/mc_subpel_filters.inc"
};
__constant__ int8_t k_warp[193][8] = {
#include "tables/mc_warp_filter.inc"
};
__constant__ int8_t k_resize[64][8] = {
#include "tables/resize_filter.inc"
};
__constant__ uint8_t k_obmc_s[64] = {
#include "tables/obmc_masks.inc"
};

__device__ __forceinline__ int rnd2(int v, int sh) { return (v + ((1 << sh) >> 1)) >> sh; }
__device__ __forceinline__ int f2d_th(int f) { return (int)((0x111222000ull >> (4 * f)) & 15); }
__device__ __forceinline__ int f2d_tv(int f) { return (int)((0x210210210ull >> (4 * f)) & 15); }

template <typename Px>
__device__ __forceinline__ int px_at(const uint8_t *base, int64_t stride, int iw, int ih, int y, int x) {
    y = min(max(y, 0), ih - 1);
    x = min(max(x, 0), iw - 1);
    return reinterpret_cast<const Px *>(base + (int64_t)y * stride)[x];
}

// ---------------------------------------------------------------------------------------
// scaled references
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int scale_fac(int ref_sz, int this_sz) { return ((ref_sz << 14) + (this_sz >> 1)) / this_sz; }

template <typename Px>
__global__ __launch_bounds__(64) void mc_scaled_kernel(McArgs a, const MiMcBlock *units, int cur_w, int cur_h) {
    const MiMcBlock b = units[blockIdx.x];
    const int p = b.plane, r = b.ref[0];
    const int ssh = p && a.layout != 3, ssv = p && a.layout == 1;
    // f->svc[r] (decode.rs:4776-4790) from the picture sizes, then mc()'s positions
    const int sx = scale_fac(a.ref_w[r][0], cur_w), sy = scale_fac(a.ref_h[r][0], cur_h);
    const int stx = (sx + 8) >> 4, sty = (sy + 8) >> 4;
    const int opy = (b.y << 4) + b.mvy[0] * (1 << !ssv), opx = (b.x << 4) + b.mvx[0] * (1 << !ssh);
    const int64_t tx = (int64_t)opx * sx + (int64_t)(sx - 0x4000) * 8;
    const int64_t ty = (int64_t)opy * sy + (int64_t)(sy - 0x4000) * 8;
    const int pos_x = (int)(tx < 0 ? -((-tx + 128) >> 8) : (tx + 128) >> 8) + 32;
    const int pos_y = (int)(ty < 0 ? -((-ty + 128) >> 8) : (ty + 128) >> 8) + 32;
    const int left = pos_x >> 10, top = pos_y >> 10, mx = pos_x & 0x3ff, my = pos_y & 0x3ff;
    const uint8_t *base = a.ref[r][p];
    const int64_t rs = a.ref_stride[r][p ? 1 : 0];
    const int iw = a.ref_w[r][p], ih = a.ref_h[r][p];
    const bool prep = b.comp == MI_MC_PREP;
    const int ib = a.ib, w = b.w, h = b.h, n = w * h;
    const int64_t ds = a.dst_stride[p ? 1 : 0];
    const bool bilin = b.filter2d == 9;
    const int th = f2d_th(b.filter2d), tv = f2d_tv(b.filter2d);
    for (int i = threadIdx.x; i < n; i += 64) {
        const int y = i / w, x = i - y * w;
        const int px = mx + x * stx, ioff = px >> 10, phx = (px & 0x3ff) >> 6;
        const int py = my + y * sty, row = py >> 10, phy = (py & 0x3ff) >> 6;
        const int cx = left + ioff, cy = top + row;
        int v;
        if (bilin) {
            // bilin_scaled (mc_tmpl.c:445-470, 528-560)
            int mid[2];
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int s0 = px_at<Px>(base, rs, iw, ih, cy + k, cx), s1 = px_at<Px>(base, rs, iw, ih, cy + k, cx + 1);
                mid[k] = rnd2(16 * s0 + phx * (s1 - s0), 4 - ib);
            }
            const int s = 16 * mid[0] + phy * (mid[1] - mid[0]);
            v = prep ? rnd2(s, 4) - a.bias : min(max(rnd2(s, 4 + ib), 0), a.bdmax);
        } else {
            // put/prep_8tap_scaled (mc_tmpl.c:201-227, 291-330)
            const int8_t *fh = phx ? k_subpel_x[w > 4 ? th : 3 + (th & 1)][phx - 1] : nullptr;
            const int8_t *fv = phy ? k_subpel_x[h > 4 ? tv : 3 + (tv & 1)][phy - 1] : nullptr;
            int mid[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int yy = cy - 3 + k;
                if (fh) {
                    int s = 0;
#pragma unroll
                    for (int j = 0; j < 8; j++) s += fh[j] * px_at<Px>(base, rs, iw, ih, yy, cx - 3 + j);
                    mid[k] = rnd2(s, 6 - ib);
                } else {
                    mid[k] = px_at<Px>(base, rs, iw, ih, yy, cx) << ib;
                }
            }
            if (fv) {
                int s = 0;
#pragma unroll
                for (int k = 0; k < 8; k++) s += fv[k] * mid[k];
                v = prep ? rnd2(s, 6) - a.bias : min(max(rnd2(s, 6 + ib), 0), a.bdmax);
            } else {
                v = prep ? mid[3] - a.bias : min(max((mid[3] + ((1 << ib) >> 1)) >> ib, 0), a.bdmax);
            }
        }
        Px *d = reinterpret_cast<Px *>(a.dst[p] + (int64_t)(b.y + y) * ds) + b.x + x;
        if (prep) {
            a.tmp[b.mask_off + i] = (int16_t)v;
        } else if (b.comp == MI_MC_OBMC_H || b.comp == MI_MC_OBMC_V) {
            // an OBMC lap from a scaled reference, blended as blend_h / blend_v (mc_tmpl.c)
            const bool above = b.comp == MI_MC_OBMC_H;
            if (above ? y < ((b.param * 3) >> 2) : x < ((w * 3) >> 2)) {
                const int m = k_obmc_s[above ? b.param + y : w + x];
                *d = (Px)((*d * (64 - m) + v * m + 32) >> 6);
            }
        } else {
            *d = (Px)v;
        }
    }
}

int launch_mc_scaled(const McArgs &a, const MiMcBlock *units, int n, int cur_w, int cur_h, hipStream_t s) {
    if (n <= 0) return 0;
    if (a.bpc == 8) mc_scaled_kernel<uint8_t><<<n, 64, 0, s>>>(a, units, cur_w, cur_h);
    else mc_scaled_kernel<uint16_t><<<n, 64, 0, s>>>(a, units, cur_w, cur_h);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------------------------------
// warped motion: warp_affine_8x8_c / _8x8t_c (mc_tmpl.c:714-796)
// ---------------------------------------------------------------------------------------
template <typename Px>
__global__ __launch_bounds__(256) void mc_warp_kernel(McArgs a, const MiWarpBlock *blocks, int n) {
    __shared__ int8_t filt[193 * 8];
    __shared__ int16_t win[4][15 * 16];
    __shared__ int16_t mid[4][15 * 8];
    for (int i = threadIdx.x; i < 193 * 8; i += 256) filt[i] = (&k_warp[0][0])[i];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bi = blockIdx.x * 4 + wv;
    const bool on = bi < n;
    const MiWarpBlock b = blocks[on ? bi : 0];
    const int p = b.plane, r = b.ref;
    const uint8_t *base = a.ref[r][p];
    const int64_t rs = a.ref_stride[r][p ? 1 : 0];
    const int iw = a.ref_w[r][p], ih = a.ref_h[r][p];
    // 15 x 15 window from (dx - 3, dy - 3), clamped (== emu_edge, recon.rs:2357-2370)
    for (int e = lane; e < 15 * 15; e += 64) {
        const int yy = e / 15, xx = e - yy * 15;
        win[wv][yy * 16 + xx] = (int16_t)px_at<Px>(base, rs, iw, ih, b.dy - 3 + yy, b.dx - 3 + xx);
    }
    __syncthreads();
    const int ib = a.ib;
    const int rr = lane >> 3, c = lane & 7;
    const int alpha = b.abcd[0], beta = b.abcd[1], gamma = b.abcd[2], delta = b.abcd[3];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int y = rr + 8 * k;
        if (y < 15) {
            const int tmx = b.mx + y * beta + c * alpha;
            const int8_t *F = filt + 8 * (64 + ((tmx + 512) >> 10));
            const int16_t *s = &win[wv][y * 16 + c];
            int sum = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) sum += F[j] * s[j];
            mid[wv][y * 8 + c] = (int16_t)rnd2(sum, 7 - ib);
        }
    }
    __syncthreads();
    if (!on) return;
    const int tmy = b.my + rr * delta + c * gamma;
    const int8_t *F = filt + 8 * (64 + ((tmy + 512) >> 10));
    int sum = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) sum += F[j] * mid[wv][(rr + j) * 8 + c];
    if (b.prep) {
        a.tmp[b.tmp_off + rr * b.tmp_stride + c] = (int16_t)(rnd2(sum, 7) - a.bias);
    } else {
        const int64_t ds = a.dst_stride[p ? 1 : 0];
        reinterpret_cast<Px *>(a.dst[p] + (int64_t)(b.y + rr) * ds)[b.x + c] =
            (Px)min(max(rnd2(sum, 7 + ib), 0), a.bdmax);
    }
}

int launch_mc_warp(const McArgs &a, const MiWarpBlock *blocks, int n, hipStream_t s) {
    if (n <= 0) return 0;
    const int g = (n + 3) / 4;
    if (a.bpc == 8) mc_warp_kernel<uint8_t><<<g, 256, 0, s>>>(a, blocks, n);
    else mc_warp_kernel<uint16_t><<<g, 256, 0, s>>>(a, blocks, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------------------------------
// compound combine from two intermediates: avg / w_avg / mask / w_mask (mc_tmpl.c:561-712)
// ---------------------------------------------------------------------------------------
template <typename Px>
__global__ __launch_bounds__(64) void mc_combine_kernel(McArgs a, const MiMcCombine *units) {
    const MiMcCombine u = units[blockIdx.x];
    const int p = u.plane, w = u.w, h = u.h, ib = a.ib, sign = u.param >> 7;
    const int16_t *t[2] = { a.tmp + u.tmp_off[sign], a.tmp + u.tmp_off[!sign] };   // t1, t2 of mask / w_mask
    const int64_t ds = a.dst_stride[p ? 1 : 0];
    uint8_t *dst = a.dst[p] + (int64_t)u.y * ds;
    auto put = [&](int y, int x, int v) {
        reinterpret_cast<Px *>(dst + (int64_t)y * ds)[u.x + x] = (Px)min(max(v, 0), a.bdmax);
    };
    if (u.comp == MI_MC_SEG) {
        // lane per mask sample: (1 << msh) x (1 << msv) pixels
        const int msh = a.seg_ss_hor, msv = a.seg_ss_ver, mw = w >> msh, mh = h >> msv;
        const int mask_sh = a.bpc + ib - 4, mask_rnd = 1 << (mask_sh - 5);
        const int sh = ib + 6, rnd = (32 << ib) + a.bias * 64;
        for (int i = threadIdx.x; i < mw * mh; i += 64) {
            const int my = i / mw, mx = i - my * mw;
            int msum = 0;
            for (int dy = 0; dy <= msv; dy++)
                for (int dx = 0; dx <= msh; dx++) {
                    const int y = (my << msv) + dy, x = (mx << msh) + dx;
                    const int t1 = t[0][y * w + x], t2 = t[1][y * w + x];
                    const int m = min(38 + ((abs(t1 - t2) + mask_rnd) >> mask_sh), 64);
                    put(y, x, (t1 * m + t2 * (64 - m) + rnd) >> sh);
                    msum += m;
                }
            int mv = msum;
            if (msh && msv) mv = (msum + 2 - sign) >> 2;
            else if (msh) mv = (msum + 1 - sign) >> 1;
            a.masks[u.mask_off + i] = (uint8_t)mv;
        }
        return;
    }
    const uint8_t *mk = a.masks + u.mask_off;
    for (int i = threadIdx.x; i < w * h; i += 64) {
        const int y = i / w, x = i - y * w;
        const int t0 = a.tmp[u.tmp_off[0] + i], t1 = a.tmp[u.tmp_off[1] + i];
        int v;
        if (u.comp == MI_MC_AVG) {
            v = (t0 + t1 + (1 << ib) + a.bias * 2) >> (ib + 1);
        } else if (u.comp == MI_MC_WAVG) {
            const int wt = u.param & 31;
            v = (t0 * wt + t1 * (16 - wt) + (8 << ib) + a.bias * 16) >> (ib + 4);
        } else {
            const int m = mk[i];
            v = (t[0][i] * m + t[1][i] * (64 - m) + (32 << ib) + a.bias * 64) >> (ib + 6);
        }
        put(y, x, v);
    }
}

int launch_mc_combine(const McArgs &a, const MiMcCombine *units, int n, hipStream_t s) {
    if (n <= 0) return 0;
    if (a.bpc == 8) mc_combine_kernel<uint8_t><<<n, 64, 0, s>>>(a, units);
    else mc_combine_kernel<uint16_t><<<n, 64, 0, s>>>(a, units);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------------------------------
// super-resolution: resize_c (mc_tmpl.c:847-875) over every row of every plane
// ---------------------------------------------------------------------------------------
template <typename Px>
__global__ __launch_bounds__(256) void superres_kernel(SuperresArgs a) {
    int b = blockIdx.x;
    const int chunk = b % a.chunks;
    b /= a.chunks;
    int p = 0;
    while (p + 1 < a.nplanes && b >= a.h[p]) b -= a.h[p++];
    const int y = b, x = chunk * 256 + threadIdx.x;
    if (x >= a.dst_w[p]) return;
    const int step = a.step[p ? 1 : 0], start = a.start[p ? 1 : 0];
    const int64_t pos = (int64_t)start + (int64_t)x * step;
    const int src_x = -1 + (int)(pos >> 14), mx = (int)(pos & 0x3fff);
    const int8_t *F = k_resize[mx >> 8];
    const Px *src = reinterpret_cast<const Px *>(a.src[p] + (int64_t)y * a.src_stride[p ? 1 : 0]);
    const int sw = a.src_w[p];
    int s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += F[k] * (int)src[min(max(src_x - 3 + k, 0), sw - 1)];
    reinterpret_cast<Px *>(a.dst[p] + (int64_t)y * a.dst_stride[p ? 1 : 0])[x] =
        (Px)min(max((-s + 64) >> 7, 0), (1 << a.bpc) - 1);
}

int launch_superres(const SuperresArgs &a, hipStream_t s) {
    int rows = 0;
    for (int p = 0; p < a.nplanes; p++) rows += a.h[p];
    const int g = rows * a.chunks;
    if (g <= 0) return 0;
    if (a.bpc == 8) superres_kernel<uint8_t><<<g, 256, 0, s>>>(a);
    else superres_kernel<uint16_t><<<g, 256, 0, s>>>(a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
