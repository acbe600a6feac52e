// ipred.hip — batched intra prediction on gfx950.
//
// Replaces the DSP intra_pred[14], cfl_pred[4] and pal_pred of Rav1dIntraPredDSPContext
// (rav1d src/ipred.rs:163-169; C ipred_tmpl.c). A launch predicts many blocks whose edges are
// already gathered (the reference's rav1d_prepare_intra_edges output, src/ipred_prepare.rs:
// 118-204): each MiIpredBlock names its topleft sample in an edge buffer laid out as the
// reference's (topleft[1 + i] top row, topleft[-(1 + i)] left column). Blocks of one launch
// must be independent (one intra wavefront step, or the per-call entry).
//
// One wave per block. Smooth/paeth/V/H/DC are per-pixel maps (DC sums by wave reduction).
// Z1/Z2/Z3 first build the filtered or upsampled edge in LDS (filter_edge / upsample_edge,
// ipred_tmpl.c:362-406), then every pixel interpolates independently: the reference's
// "pixel_set ... break" tails are the per-pixel rule base >= max_base (base grows along the
// row). FILTER_PRED (recursive 4x2 taps) runs as an anti-diagonal wavefront of 4x2 sub-blocks
// over an LDS copy of the block.
#include "common.h"

namespace mi {

__constant__ uint8_t k_sm_weights[128] = {
#include "tables/sm_weights.inc"
};
__constant__ uint16_t k_dr_intra_derivative[44] = {
#include "tables/dr_intra_derivative.inc"
};
__constant__ int8_t k_filter_intra_taps[5][64] = {
#include "tables/filter_intra_taps.inc"
};

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ int filter_strength(int wh, int angle, int is_sm) {
    if (is_sm) {
        if (wh <= 8) { if (angle >= 64) return 2; if (angle >= 40) return 1; }
        else if (wh <= 16) { if (angle >= 48) return 2; if (angle >= 20) return 1; }
        else if (wh <= 24) { if (angle >= 4) return 3; }
        else return 3;
    } else {
        if (wh <= 8) { if (angle >= 56) return 1; }
        else if (wh <= 16) { if (angle >= 40) return 1; }
        else if (wh <= 24) { if (angle >= 32) return 3; if (angle >= 16) return 2; if (angle >= 8) return 1; }
        else if (wh <= 32) { if (angle >= 32) return 3; if (angle >= 4) return 2; return 1; }
        else return 3;
    }
    return 0;
}

__device__ __forceinline__ int upsample_on(int wh, int angle, int is_sm) { return angle < 40 && wh <= (16 >> is_sm); }

// filter_edge: out[i] for i in [0, sz), lanes in parallel; in_ is the edge base, samples in
// index range [from, to) (clamped).
template <typename Px>
__device__ void filter_edge_par(int *out, int sz, int lim_from, int lim_to, const Px *in_, int from, int to, int strength) {
    const int k0 = strength == 3 ? 2 : 0, k1 = strength == 1 ? 4 : strength == 2 ? 5 : 4;
    const int k2 = strength == 1 ? 8 : strength == 2 ? 6 : 4;
    for (int i = threadIdx.x; i < sz; i += 64) {
        if (i < lim_from || i >= lim_to) {
            out[i] = in_[min(max(i, from), to - 1)];
        } else {
            int s = k0 * in_[min(max(i - 2, from), to - 1)] + k1 * in_[min(max(i - 1, from), to - 1)] +
                    k2 * in_[min(max(i, from), to - 1)] + k1 * in_[min(max(i + 1, from), to - 1)] +
                    k0 * in_[min(max(i + 2, from), to - 1)];
            out[i] = (s + 8) >> 4;
        }
    }
}

// upsample_edge: out[0 .. 2 hsz - 2]
template <typename Px>
__device__ void upsample_edge_par(int *out, int hsz, const Px *in_, int from, int to, int bdmax) {
    for (int i = threadIdx.x; i < hsz; i += 64) {
        out[i * 2] = in_[min(max(i, from), to - 1)];
        if (i < hsz - 1) {
            const int s = -in_[min(max(i - 1, from), to - 1)] + 9 * in_[min(max(i, from), to - 1)] +
                          9 * in_[min(max(i + 1, from), to - 1)] - in_[min(max(i + 2, from), to - 1)];
            out[i * 2 + 1] = min(max((s + 8) >> 4, 0), bdmax);
        }
    }
}

// Predict one block from its gathered edge `tl` (global edge buffer or LDS). eb / ft: LDS
// scratch for the directional edge and the filter-intra image.
template <typename Px>
__device__ __forceinline__ void predict_block(const IpredArgs &a, const MiIpredBlock &b, const Px *tl, int *eb, Px *ft) {
    const int lane = threadIdx.x;
    const int w = b.w, h = b.h, n = w * h;
    const int64_t st = a.stride[b.plane ? 1 : 0];
    uint8_t *dst = a.dst[b.plane] + (int64_t)b.y * st + (int64_t)b.x * sizeof(Px);
    const int bdmax = a.bdmax;
    // inter-intra (MI_IPRED_II): blend into the inter prediction with the block's mask
    // (mc.blend, mc_tmpl.c:621-630); the address is formed before the uniform branch
    const bool ii = b.mode & MI_IPRED_II;
    const uint8_t *iim = a.idx + b.aux_off;
    auto put = [&](int y, int x, int v) {
        Px *d = reinterpret_cast<Px *>(dst + (int64_t)y * st) + x;
        if (ii) {
            const int m = iim[y * w + x];
            v = (*d * (64 - m) + v * m + 32) >> 6;
        }
        *d = (Px)v;
    };
    const int mode = b.mode & ~MI_IPRED_II;

    if (mode >= MI_IPRED_PAL) {                      // pal_pred: palette at edge_off, indices in idx
        const uint8_t *idx = a.idx + b.aux_off;
        for (int i = lane; i < n; i += 64) put(i / w, i % w, tl[idx[i]]);
        return;
    }
    const bool cfl = mode >= MI_IPRED_CFL;
    const int m = cfl ? mode - MI_IPRED_CFL : mode;
    if (m == 0 || m == 3 || m == 4 || m == 5) {
        // DC family (ipred_tmpl.c:86-218) -> splat or CfL
        int dc;
        if (m == 5) {
            dc = (bdmax + 1) >> 1;
        } else {
            int s = 0;
            if (m != 3) for (int i = lane; i < w; i += 64) s += tl[1 + i];
            if (m != 4) for (int i = lane; i < h; i += 64) s += tl[-(1 + i)];
            s = wave_sum(s);
            if (m == 4) dc = (s + (w >> 1)) >> __ffs(w) - 1;
            else if (m == 3) dc = (s + (h >> 1)) >> __ffs(h) - 1;
            else {
                unsigned d = ((unsigned)s + ((w + h) >> 1)) >> (__ffs(w + h) - 1);
                if (w != h) {
                    const bool q = w > h * 2 || h > w * 2;
                    if (a.bpc == 8) d = (d * (q ? 0x3334u : 0x5556u)) >> 16;
                    else d = (d * (q ? 0x6667u : 0xAAABu)) >> 17;
                }
                dc = (int)d;
            }
        }
        if (!cfl) {
            for (int i = lane; i < n; i += 64) put(i / w, i % w, dc);
        } else {
            const int16_t *ac = a.ac + b.aux_off;
            const int alpha = b.alpha;
            for (int i = lane; i < n; i += 64) {
                const int diff = alpha * ac[i];
                const int mag = (abs(diff) + 32) >> 6;
                put(i / w, i % w, min(max(dc + (diff < 0 ? -mag : mag), 0), bdmax));
            }
        }
        return;
    }
    // V, H, PAETH, SMOOTH, SMOOTH_V, SMOOTH_H: the (wave-uniform) mode selects one loop;
    // no per-pixel mode branch (a merged per-pixel three-way branch here was miscompiled by
    // hipcc 7.2: the store address was left undefined on one path)
    if (m == 1) {
        for (int i = lane; i < n; i += 64) put(i / w, i % w, tl[1 + i % w]);
        return;
    }
    if (m == 2) {
        for (int i = lane; i < n; i += 64) put(i / w, i % w, tl[-(1 + i / w)]);
        return;
    }
    if (m == 12) {
        const int c = tl[0];
        for (int i = lane; i < n; i += 64) {
            const int y = i / w, x = i % w;
            const int top = tl[1 + x], left = tl[-(1 + y)];
            const int base = left + top - c;
            const int ld = abs(left - base), td = abs(top - base), tld = abs(c - base);
            put(y, x, ld <= td && ld <= tld ? left : td <= tld ? top : c);
        }
        return;
    }
    if (m == 9) {
        const int right = tl[w], bottom = tl[-h];
        for (int i = lane; i < n; i += 64) {
            const int y = i / w, x = i % w;
            const int wv = k_sm_weights[h + y], wh = k_sm_weights[w + x];
            put(y, x, (wv * tl[1 + x] + (256 - wv) * bottom + wh * tl[-(1 + y)] + (256 - wh) * right + 256) >> 9);
        }
        return;
    }
    if (m == 10) {
        const int bottom = tl[-h];
        for (int i = lane; i < n; i += 64) {
            const int y = i / w, x = i % w;
            const int wv = k_sm_weights[h + y];
            put(y, x, (wv * tl[1 + x] + (256 - wv) * bottom + 128) >> 8);
        }
        return;
    }
    if (m == 11) {
        const int right = tl[w];
        for (int i = lane; i < n; i += 64) {
            const int y = i / w, x = i % w;
            const int wh = k_sm_weights[w + x];
            put(y, x, (wh * tl[-(1 + y)] + (256 - wh) * right + 128) >> 8);
        }
        return;
    }
    const int is_sm = (b.angle >> 9) & 1, eef = b.angle >> 10, angle = b.angle & 511;
    if (m == 6) {
        // Z1 (ipred_tmpl.c:408-460)
        int dx = k_dr_intra_derivative[angle >> 1];
        const int up = eef ? upsample_on(w + h, 90 - angle, is_sm) : 0;
        const int fs = !up && eef ? filter_strength(w + h, 90 - angle, is_sm) : 0;
        int max_base_x;
        if (up) {
            upsample_edge_par<Px>(eb, w + h, tl + 1, -1, w + min(w, h), bdmax);
            max_base_x = 2 * (w + h) - 2;
            dx <<= 1;
        } else if (fs) {
            filter_edge_par<Px>(eb, w + h, 0, w + h, tl + 1, -1, w + min(w, h), fs);
            max_base_x = w + h - 1;
        } else {
            for (int i = lane; i < w + h; i += 64) eb[i] = tl[1 + i];
            max_base_x = w + min(w, h) - 1;
        }
        __syncthreads();
        const int base_inc = 1 + up;
        for (int i = lane; i < n; i += 64) {
            const int y = i / w, x = i % w;
            const int xpos = (y + 1) * dx, frac = xpos & 0x3E, base = (xpos >> 6) + x * base_inc;
            put(y, x, base < max_base_x ? (eb[base] * (64 - frac) + eb[base + 1] * frac + 32) >> 6 : eb[max_base_x]);
        }
        return;
    }
    if (m == 7) {
        // Z2 (ipred_tmpl.c:462-540): eb[64 + k] = topleft[k], k in [-2h, 2w]
        int dy = k_dr_intra_derivative[(angle - 90) >> 1];
        int dx = k_dr_intra_derivative[(180 - angle) >> 1];
        const int up_left = eef ? upsample_on(w + h, 180 - angle, is_sm) : 0;
        const int up_above = eef ? upsample_on(w + h, angle - 90, is_sm) : 0;
        int *const t = eb + 64;
        if (up_above) {
            upsample_edge_par<Px>(t, w + 1, tl, 0, w + 1, bdmax);
            dx <<= 1;
        } else {
            const int fs = eef ? filter_strength(w + h, angle - 90, is_sm) : 0;
            if (fs) filter_edge_par<Px>(t + 1, w, 0, b.max_w, tl + 1, -1, w, fs);
            else for (int i = lane; i < w; i += 64) t[1 + i] = tl[1 + i];
        }
        if (up_left) {
            upsample_edge_par<Px>(t - 2 * h, h + 1, tl - h, 0, h + 1, bdmax);
            dy <<= 1;
        } else {
            const int fs = eef ? filter_strength(w + h, 180 - angle, is_sm) : 0;
            if (fs) filter_edge_par<Px>(t - h, h, h - b.max_h, h, tl - h, 0, h + 1, fs);
            else for (int i = lane; i < h; i += 64) t[-h + i] = tl[-h + i];
        }
        __syncthreads();
        if (lane == 0) t[0] = tl[0];
        __syncthreads();
        // both interpolations are evaluated (clamped LDS indices) and selected: no per-pixel branch
        const int base_inc_x = 1 + up_above;
        const int lo = 64 - (1 + up_left);           // eb index of left[0]
        for (int i = lane; i < n; i += 64) {
            const int y = i / w, x = i % w;
            const int xpos = ((1 + up_above) << 6) - (y + 1) * dx;
            const int base_x = (xpos >> 6) + x * base_inc_x, frac_x = xpos & 0x3E;
            const int ti = min(max(64 + base_x, 0), 2 * 128);
            const int vt = eb[ti] * (64 - frac_x) + eb[ti + 1] * frac_x;
            const int ypos = (y << (6 + up_left)) - (x + 1) * dy;
            const int base_y = ypos >> 6, frac_y = ypos & 0x3E;
            const int li = min(max(lo - base_y, 1), 2 * 128 + 1);
            const int vl = eb[li] * (64 - frac_y) + eb[li - 1] * frac_y;
            put(y, x, ((base_x >= 0 ? vt : vl) + 32) >> 6);
        }
        return;
    }
    if (m == 8) {
        // Z3 (ipred_tmpl.c:542-616): lv(k) = left[-k]
        int dy = k_dr_intra_derivative[(270 - angle) >> 1];
        const int up = eef ? upsample_on(w + h, angle - 180, is_sm) : 0;
        const int fs = !up && eef ? filter_strength(w + h, angle - 180, is_sm) : 0;
        int max_base_y, lbase;
        if (up) {
            upsample_edge_par<Px>(eb, w + h, tl - (w + h), max(w - h, 0), w + h + 1, bdmax);
            lbase = 2 * (w + h) - 2;
            max_base_y = 2 * (w + h) - 2;
            dy <<= 1;
        } else if (fs) {
            filter_edge_par<Px>(eb, w + h, 0, w + h, tl - (w + h), max(w - h, 0), w + h + 1, fs);
            lbase = w + h - 1;
            max_base_y = w + h - 1;
        } else {
            // left = &topleft[-1]: store eb[lbase - k] = topleft[-1 - k], k in [0, w + h]
            lbase = w + h;
            for (int k = lane; k <= w + h; k += 64) eb[lbase - k] = tl[-1 - k];
            max_base_y = h + min(w, h) - 1;
        }
        __syncthreads();
        const int base_inc = 1 + up;
        for (int i = lane; i < n; i += 64) {
            const int y = i / w, x = i % w;
            const int ypos = (x + 1) * dy, frac = ypos & 0x3E, base = (ypos >> 6) + y * base_inc;
            put(y, x, base < max_base_y ? (eb[lbase - base] * (64 - frac) + eb[lbase - base - 1] * frac + 32) >> 6
                                        : eb[lbase - max_base_y]);
        }
        return;
    }
    // FILTER_PRED (ipred_tmpl.c:618-655): 4x2 sub-blocks, anti-diagonal wavefront
    {
        const int8_t *flt = k_filter_intra_taps[b.angle & 511];
        const int nbx = w >> 2, nby = h >> 1;
        const int sb = lane >> 3, o = lane & 7, yy = o >> 2, xx = o & 3;
        for (int d = 0; d < nbx + nby - 1; d++) {
            // sub-blocks on this diagonal: by from max(0, d - nbx + 1) .. min(d, nby - 1)
            const int by0 = max(0, d - nbx + 1), by1 = min(d, nby - 1);
            for (int k0 = by0; k0 <= by1; k0 += 8) {
                const int by = k0 + sb, bx = d - by;
                if (by <= by1) {
                    const int x = bx * 4, y = by * 2;
                    int p[7];
                    p[0] = y ? (x ? (int)ft[(y - 1) * w + x - 1] : (int)tl[-y]) : (int)tl[x];
#pragma unroll
                    for (int k = 0; k < 4; k++) p[1 + k] = y ? (int)ft[(y - 1) * w + x + k] : (int)tl[1 + x + k];
#pragma unroll
                    for (int k = 0; k < 2; k++) p[5 + k] = x ? (int)ft[(y + k) * w + x - 1] : (int)tl[-(1 + y + k)];
                    const int8_t *f = flt + yy * 4 + xx;
                    int acc = 0;
#pragma unroll
                    for (int k = 0; k < 7; k++) acc += f[8 * k] * p[k];
                    ft[(y + yy) * w + x + xx] = (Px)min(max((acc + 8) >> 4, 0), bdmax);
                }
            }
            __syncthreads();
        }
        for (int i = lane; i < n; i += 64) put(i / w, i % w, ft[i]);
    }
}

template <typename Px>
__global__ __launch_bounds__(64) void ipred_kernel(IpredArgs a) {
    __shared__ int eb[2 * 128 + 2];            // prepared edge (Z1/Z3: 2(w+h); Z2: 64 + 64 + 1)
    __shared__ Px ft[32 * 32];                 // FILTER_PRED block image (up to 32x32)
    const MiIpredBlock b = a.blocks[blockIdx.x];
    predict_block<Px>(a, b, reinterpret_cast<const Px *>(a.edges) + b.edge_off, eb, ft);
}

// ---- device-side rav1d_prepare_intra_edges (ipred_prepare.rs:118-204) ----

// av1_intra_prediction_edges needs per implementation mode: LEFT 1, TOP 2, TOP_LEFT 4,
// TOP_RIGHT 8, BOTTOM_LEFT 16 (ipred_prepare.rs:76-115)
__constant__ uint8_t k_needs[14] = { 3, 2, 1, 1, 2, 0, 14, 7, 21, 3, 3, 3, 7, 7 };
__constant__ uint8_t k_mode_angle[8] = { 90, 180, 45, 135, 113, 157, 203, 67 };

template <typename Px>
__global__ __launch_bounds__(64) void intra_kernel(IpredArgs a) {
    __shared__ int eb[2 * 128 + 2];
    __shared__ Px ft[32 * 32];
    __shared__ Px edge[2 * 128 + 1];           // topleft at [128]
    const MiIntraBlock ib = a.iblocks[blockIdx.x];
    const int lane = threadIdx.x;
    const int w = ib.w, h = ib.h, x = ib.x, y = ib.y;
    const bool have_left = ib.flags & MI_INTRA_HAVE_LEFT, have_top = ib.flags & MI_INTRA_HAVE_TOP;
    const int64_t st = a.stride[ib.plane ? 1 : 0];
    const Px *pic = reinterpret_cast<const Px *>(a.dst[ib.plane]);
    auto P = [&](int yy, int xx) -> int { return reinterpret_cast<const Px *>(reinterpret_cast<const uint8_t *>(pic) + (int64_t)yy * st)[xx]; };
    const int bd = a.bpc;

    MiIpredBlock b;
    b.edge_off = 0;
    b.aux_off = ib.aux_off;
    b.x = ib.x;
    b.y = ib.y;
    b.w = ib.w;
    b.h = ib.h;
    b.plane = ib.plane;
    b.max_w = ib.max_w;
    b.max_h = ib.max_h;
    b.alpha = ib.alpha;
    b.pad = 0;
    const int ii = ib.flags & MI_INTRA_II ? MI_IPRED_II : 0;
    if (ib.mode == MI_IPRED_PAL) {
        b.mode = MI_IPRED_PAL;
        b.angle = 0;
        predict_block<Px>(a, b, reinterpret_cast<const Px *>(a.pal) + ib.pal_off, eb, ft);
        return;
    }
    // mode remap (ipred_prepare.rs:148-172): all wave-uniform
    const bool cfl = ib.mode == MI_IPRED_CFL;
    int m = cfl ? 0 : ib.mode, angle = 0;
    if (m >= 1 && m <= 8) {
        angle = k_mode_angle[m - 1] + 3 * ib.angle;
        if (angle <= 90) m = angle < 90 && have_top ? 6 : 1;
        else if (angle < 180) m = 7;
        else m = angle > 180 && have_left ? 8 : 2;
    } else if (m == 0 || m == 12) {
        // av1_mode_conv[mode][have_left][have_top]
        m = m == 0 ? (have_left ? (have_top ? 0 : 3) : (have_top ? 4 : 5))
                   : (have_left ? (have_top ? 12 : 2) : (have_top ? 1 : 5));
    } else if (m == 13) {
        angle = ib.filt_idx;
    }
    const int needs = k_needs[m];
    Px *tl = edge + 128;
    const int tw4 = w >> 2, th4 = h >> 2;
    // left column (+ bottom-left)
    if (needs & 1) {
        const int sz = h;
        if (have_left) {
            const int px_have = min(sz, (int)ib.tile_h - y);
            for (int i = lane; i < sz; i += 64) tl[-1 - i] = (Px)P(y + min(i, px_have - 1), x - 1);
        } else {
            const int v = have_top ? P(y - 1, x) : (1 << bd >> 1) + 1;
            for (int i = lane; i < sz; i += 64) tl[-1 - i] = (Px)v;
        }
        if (needs & 16) {
            const bool hbl = have_left && y + h < (int)ib.tile_h && (ib.flags & MI_INTRA_BOTTOM_LEFT);
            if (hbl) {
                const int px_have = min(sz, (int)ib.tile_h - y - h);
                for (int i = lane; i < sz; i += 64) tl[-1 - sz - i] = (Px)P(y + sz + min(i, px_have - 1), x - 1);
            } else {
                // bottom_left[..] = bottom_left[sz] = the last left sample (written above by this
                // lane set: recompute it instead of reading LDS before the barrier)
                const int last = have_left ? P(y + min(sz, (int)ib.tile_h - y) - 1, x - 1)
                                           : (have_top ? P(y - 1, x) : (1 << bd >> 1) + 1);
                for (int i = lane; i < sz; i += 64) tl[-1 - sz - i] = (Px)last;
            }
        }
    }
    // top row (+ top-right)
    if (needs & 2) {
        const int sz = w;
        if (have_top) {
            const int px_have = min(sz, (int)ib.tile_w - x);
            for (int i = lane; i < sz; i += 64) tl[1 + i] = (Px)P(y - 1, x + min(i, px_have - 1));
        } else {
            const int v = have_left ? P(y, x - 1) : (1 << bd >> 1) - 1;
            for (int i = lane; i < sz; i += 64) tl[1 + i] = (Px)v;
        }
        if (needs & 8) {
            const bool htr = have_top && x + w < (int)ib.tile_w && (ib.flags & MI_INTRA_TOP_RIGHT);
            if (htr) {
                const int px_have = min(sz, (int)ib.tile_w - x - w);
                for (int i = lane; i < sz; i += 64) tl[1 + sz + i] = (Px)P(y - 1, x + sz + min(i, px_have - 1));
            } else {
                const int last = have_top ? P(y - 1, x + min(sz, (int)ib.tile_w - x) - 1)
                                          : (have_left ? P(y, x - 1) : (1 << bd >> 1) - 1);
                for (int i = lane; i < sz; i += 64) tl[1 + sz + i] = (Px)last;
            }
        }
    }
    __syncthreads();
    if ((needs & 4) && lane == 0) {
        int c = have_top ? P(y - 1, x - (have_left ? 1 : 0)) : have_left ? P(y, x - 1) : 1 << bd >> 1;
        if (m == 7 && tw4 + th4 >= 6 && (ib.flags & MI_INTRA_EDGE_FILTER))
            c = ((tl[-1] + tl[1]) * 5 + c * 6 + 8) >> 4;
        tl[0] = (Px)c;
    }
    __syncthreads();
    b.mode = (uint8_t)((cfl ? MI_IPRED_CFL + m : m) | ii);
    b.angle = (uint16_t)(angle | (ib.flags & MI_INTRA_SMOOTH_NB ? 512 : 0) | (ib.flags & MI_INTRA_EDGE_FILTER ? 1024 : 0));
    if (m == 13) b.angle = (uint16_t)ib.filt_idx;
    predict_block<Px>(a, b, tl, eb, ft);
}

int launch_intra(const IpredArgs &a, int n, hipStream_t s) {
    if (n <= 0) return 0;
    if (a.bpc == 8) intra_kernel<uint8_t><<<n, 64, 0, s>>>(a);
    else intra_kernel<uint16_t><<<n, 64, 0, s>>>(a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_ipred(const IpredArgs &a, int n, hipStream_t s) {
    if (n <= 0) return 0;
    if (a.bpc == 8) ipred_kernel<uint8_t><<<n, 64, 0, s>>>(a);
    else ipred_kernel<uint16_t><<<n, 64, 0, s>>>(a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
