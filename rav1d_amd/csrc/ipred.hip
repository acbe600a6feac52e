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
#include "itx_1d.h"

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

// TxfmType -> 1-D kinds (as itx.hip's k_row_kind / k_col_kind; levels.rs TxfmType is VERT_HORZ)
// (2 bits per type, packed in an immediate: a table in memory is a scalar load per block)
//   column: { KD, KA, KD, KA, KF, KD, KF, KA, KF, KI, KD, KI, KA, KI, KF, KI }
//   row:    { KD, KD, KA, KA, KD, KF, KF, KF, KA, KI, KI, KD, KI, KA, KI, KF }
__device__ __forceinline__ int col_kind_ip(int t) { return (int)((0xedce6244u >> (2 * t)) & 3); }
__device__ __forceinline__ int row_kind_ip(int t) { return (int)((0xb73da850u >> (2 * t)) & 3); }

// Sum over the wave by DPP row shifts and row broadcasts (VALU only, no LDS round trips), the
// total read from lane 63
__device__ __forceinline__ int wave_sum_dpp(int v) {
    int s = v;
    s += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    s += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    s += __builtin_amdgcn_update_dpp(0, v, 0x113, 0xf, 0xf, false);   // row_shr:3
    s += __builtin_amdgcn_update_dpp(0, s, 0x114, 0xf, 0xe, false);   // row_shr:4, banks 1-3
    s += __builtin_amdgcn_update_dpp(0, s, 0x118, 0xf, 0xc, false);   // row_shr:8, banks 2-3
    s += __builtin_amdgcn_update_dpp(0, s, 0x142, 0xa, 0xf, false);   // row_bcast:15, rows 1, 3
    s += __builtin_amdgcn_update_dpp(0, s, 0x143, 0xc, 0xf, false);   // row_bcast:31, rows 2-3
    return __builtin_amdgcn_readlane(s, 63);
}

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

// plane base / stride by a (wave-uniform) plane index as selects: an indexed array of a
// register-held argument struct would put the struct in scratch
__device__ __forceinline__ uint8_t *plane_ptr(const IpredArgs &a, int p) {
    return p == 0 ? a.dst[0] : p == 1 ? a.dst[1] : a.dst[2];
}
__device__ __forceinline__ int64_t plane_stride(const IpredArgs &a, int p) { return p ? a.stride[1] : a.stride[0]; }

// DC_PRED / LEFT_DC / TOP_DC (m 0 / 3 / 4) from the sum s of the edge samples they average
// (ipred_tmpl.c:86-160: the 1/3 and 1/5 multipliers of rectangular blocks)
__device__ __forceinline__ int dc_of_sum(int m, int s, int w, int h, int bpc) {
    if (m == 4) return (s + (w >> 1)) >> (__ffs(w) - 1);
    if (m == 3) return (s + (h >> 1)) >> (__ffs(h) - 1);
    unsigned d = ((unsigned)s + ((w + h) >> 1)) >> (__ffs(w + h) - 1);
    if (w != h) {
        const bool q = w > h * 2 || h > w * 2;
        if (bpc == 8) d = (d * (q ? 0x3334u : 0x5556u)) >> 16;
        else d = (d * (q ? 0x6667u : 0xAAABu)) >> 17;
    }
    return (int)d;
}

// Predict one block from its gathered edge `tl` (global edge buffer or LDS). eb / ft: LDS
// scratch for the directional edge and the filter-intra image.
template <typename Px, bool ToLds = false>
__device__ __forceinline__ void predict_block(const IpredArgs &a, const MiIpredBlock &b, const Px *tl, int *eb, Px *ft,
                                              Px *lt = nullptr, const int16_t *acl = nullptr,
                                              const int16_t *res = nullptr, int rdc = 0, int dcs = -1) {
    const int lane = threadIdx.x;
    const int w = b.w, h = b.h, n = w * h;
    // (w is a power of two: row / column of pixel i by shift and mask, not a division)
    const int lw = 31 - __clz(w);
    const int64_t st = plane_stride(a, b.plane);
    uint8_t *dst = plane_ptr(a, b.plane) + (int64_t)b.y * st + (int64_t)b.x * sizeof(Px);
    const int bdmax = a.bdmax;
    // inter-intra (MI_IPRED_II): blend into the inter prediction with the block's mask
    // (mc.blend, mc_tmpl.c:621-630); the address is formed before the uniform branch
    const bool ii = b.mode & MI_IPRED_II;
    const uint8_t *iim = a.idx + b.aux_off;
    // ToLds: the prediction goes to the w x h LDS tile lt (the fused intra reconstruction
    // adds the residual there); otherwise into the picture
    // ToLds: plus the block's residual (res, or the DC-only block's constant rdc), clipped
    auto put = [&](int y, int x, int v) {
        Px *d = ToLds ? lt + y * w + x : reinterpret_cast<Px *>(dst + (int64_t)y * st) + x;
        if (ii) {
            const int m = iim[y * w + x];
            v = (*d * (64 - m) + v * m + 32) >> 6;
        }
        if constexpr (ToLds) v = clampi(v + (res ? (int)res[y * w + x] : rdc), 0, bdmax);
        *d = (Px)v;
    };
    const int mode = b.mode & ~MI_IPRED_II;

    if (mode >= MI_IPRED_PAL) {                      // pal_pred: palette at edge_off, indices in idx
        const uint8_t *idx = a.idx + b.aux_off;
        for (int i = lane; i < n; i += 64) put((i >> lw), (i & (w - 1)), tl[idx[i]]);
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
            if (dcs >= 0) {
                s = dcs;                             // (summed by the caller from its registers)
            } else if (w + h <= 16) {
                // a few samples: every lane sums them itself (broadcast LDS reads), no
                // cross-lane reduction chain
                if (m != 3) for (int i = 0; i < w; i++) s += tl[1 + i];
                if (m != 4) for (int i = 0; i < h; i++) s += tl[-(1 + i)];
            } else {
                if (m != 3) for (int i = lane; i < w; i += 64) s += tl[1 + i];
                if (m != 4) for (int i = lane; i < h; i += 64) s += tl[-(1 + i)];
                s = wave_sum(s);
            }
            dc = dc_of_sum(m, s, w, h, a.bpc);
        }
        if (!cfl) {
            for (int i = lane; i < n; i += 64) put((i >> lw), (i & (w - 1)), dc);
        } else {
            const int16_t *ac = acl ? acl : a.ac + b.aux_off;
            const int alpha = b.alpha;
            for (int i = lane; i < n; i += 64) {
                const int diff = alpha * ac[i];
                const int mag = (abs(diff) + 32) >> 6;
                put((i >> lw), (i & (w - 1)), min(max(dc + (diff < 0 ? -mag : mag), 0), bdmax));
            }
        }
        return;
    }
    // V, H, PAETH, SMOOTH, SMOOTH_V, SMOOTH_H: the (wave-uniform) mode selects one loop;
    // no per-pixel mode branch (a merged per-pixel three-way branch here was miscompiled by
    // hipcc 7.2: the store address was left undefined on one path)
    if (m == 1) {
        for (int i = lane; i < n; i += 64) put((i >> lw), (i & (w - 1)), tl[1 + (i & (w - 1))]);
        return;
    }
    if (m == 2) {
        for (int i = lane; i < n; i += 64) put((i >> lw), (i & (w - 1)), tl[-(1 + (i >> lw))]);
        return;
    }
    if (m == 12) {
        const int c = tl[0];
        for (int i = lane; i < n; i += 64) {
            const int y = (i >> lw), x = (i & (w - 1));
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
            const int y = (i >> lw), x = (i & (w - 1));
            const int wv = k_sm_weights[h + y], wh = k_sm_weights[w + x];
            put(y, x, (wv * tl[1 + x] + (256 - wv) * bottom + wh * tl[-(1 + y)] + (256 - wh) * right + 256) >> 9);
        }
        return;
    }
    if (m == 10) {
        const int bottom = tl[-h];
        for (int i = lane; i < n; i += 64) {
            const int y = (i >> lw), x = (i & (w - 1));
            const int wv = k_sm_weights[h + y];
            put(y, x, (wv * tl[1 + x] + (256 - wv) * bottom + 128) >> 8);
        }
        return;
    }
    if (m == 11) {
        const int right = tl[w];
        for (int i = lane; i < n; i += 64) {
            const int y = (i >> lw), x = (i & (w - 1));
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
            const int y = (i >> lw), x = (i & (w - 1));
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
            const int y = (i >> lw), x = (i & (w - 1));
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
            const int y = (i >> lw), x = (i & (w - 1));
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
        for (int i = lane; i < n; i += 64) put((i >> lw), (i & (w - 1)), ft[i]);
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
// (5 bits per mode: { 3, 2, 1, 1, 2, 0, 14, 7, 21, 3, 3, 3, 7, 7 }; packed immediates, as the
// transform kinds)
__device__ __forceinline__ int needs_of(int m) {
    return m < 12 ? (int)((0x718c753b80208443ull >> (5 * m)) & 31) : (int)(((0x718c753b80208443ull >> 60) | (0xeull << 4)) >> (5 * (m - 12)) & 31);
}
// base angles of the directional modes 1..8 { 90, 180, 45, 135, 113, 157, 203, 67 }
__device__ __forceinline__ int mode_angle(int k) { return (int)((0x43cb9d71872db45aull >> (8 * k)) & 255); }

// cfl_ac (ipred.rs:1326-1432; C ipred_tmpl.c:658-700) by one wave: each AC sample is the sum
// of its 1/2/4 luma pixels scaled to <<3 in total, w_pad / h_pad 4-px groups replicate the last
// real column / row, then the rounded mean is subtracted. Lane i % 64 owns sample i, so the
// caller's reads of ac need no barrier. Sc1: the luma was stored during this launch (fused
// reconstruction), read past L1.
// A pixel read of the persistent kernel's hand-off: the aligned 4-byte word holding it, loaded
// `sc1` (L1-bypassing, agent scope), and the pixel extracted. MI355X_MICROARCH.md's hand-off
// table (row 1) covers 4-, 8- and 16-B `sc1` loads of bytes stored `sc1`, not 1-/2-B loads.
// global (address space 1) `sc1` loads: a generic pointer would make them flat loads, which
// also count in lgkmcnt and are not the `global_` form the hand-off rules name
template <typename T>
__device__ __forceinline__ T ld_sc1(const T *q) {
    typedef __attribute__((address_space(1))) const T *gp;
    return __hip_atomic_load((gp)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename Px>
__device__ __forceinline__ int ld_px_sc1(const Px *q) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(q);
    const uint32_t w = ld_sc1(reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3));
    if constexpr (sizeof(Px) == 1) return (w >> (8 * (a & 3))) & 0xff;
    else return (w >> (8 * (a & 2))) & 0xffff;
}

template <typename Px, bool Sc1>
__device__ __forceinline__ void cfl_ac_wave(int16_t *ac, const uint8_t *ybase, int64_t stride, int w_pad, int h_pad,
                                            int cw, int ch, int ss_hor, int ss_ver) {
    const int lane = threadIdx.x & 63;
    const int rw = cw - 4 * w_pad, rh = ch - 4 * h_pad;   // real (unpadded) extent
    const int64_t ps = stride / (int64_t)sizeof(Px);
    const Px *y = reinterpret_cast<const Px *>(ybase);
    auto L = [&](int64_t o) -> int {
        if constexpr (Sc1) return ld_px_sc1(y + o);
        else return y[o];
    };
    const int sh = 1 + !ss_ver + !ss_hor;
    int sum = 0;
    for (int i = lane; i < cw * ch; i += 64) {
        const int r = min(i / cw, rh - 1), c = min(i % cw, rw - 1);
        const int yy = r << ss_ver, xx = c << ss_hor;
        int s = L(yy * ps + xx);
        if (ss_hor) s += L(yy * ps + xx + 1);
        if (ss_ver) {
            s += L((yy + 1) * ps + xx);
            if (ss_hor) s += L((yy + 1) * ps + xx + 1);
        }
        s <<= sh;
        ac[i] = (int16_t)s;
        sum += s;
    }
    sum = wave_sum(sum);
    const int log2sz = __ffs(cw) - 1 + __ffs(ch) - 1;
    const int mean = (sum + ((1 << log2sz) >> 1)) >> log2sz;
    for (int i = lane; i < cw * ch; i += 64) ac[i] = (int16_t)(ac[i] - mean);
}

// Edge granules of the persistent reconstruction (IntraReconArgs::gran): for one plane, the
// right column of every block at its 4-px column boundary (col[bx * colp + y / 2]: pixels y and
// y + 1 of column 4 * bx - 1) and its bottom row at its row boundary (row[by * rowp + x / 2]:
// pixels x and x + 1 of row 4 * by - 1), each an 8-B {pixel, pixel << 16, epoch << 32} record
// stored by one `sc1` 8-B store: the hand-off of MI355X_MICROARCH.md's data-tagged granules (no
// flag, no second load: a consumer polls the record itself and finds the data with the tag).
#ifndef MI_IR_GRAN_SPIN_LOG2
#define MI_IR_GRAN_SPIN_LOG2 22
#endif
struct GranCtx {
    unsigned long long *col, *row;
    int colp, rowp;
    uint32_t epoch;
    int *err;
};
__device__ __forceinline__ GranCtx gran_ctx(unsigned long long *base, int pw, int ph, int ss_hor, int ss_ver,
                                             int nplanes, int plane, uint32_t epoch, int *err) {
    GranCtx g;
    unsigned long long *q = base;
    for (int p = 0; p < nplanes; p++) {
        const int w = p ? pw >> ss_hor : pw, h = p ? ph >> ss_ver : ph;
        const int colp = h >> 1, rowp = w >> 1;
        if (p == plane) {
            g.col = q;
            g.row = q + (size_t)((w >> 2) + 1) * colp;
            g.colp = colp;
            g.rowp = rowp;
        }
        q += (size_t)((w >> 2) + 1) * colp + (size_t)((h >> 2) + 1) * rowp;
    }
    g.epoch = epoch;
    g.err = err;
    return g;
}
// The edge pixels (yy[k], xx[k]) (use[k]) of the block at (x, y) from the granules: a left-column
// pixel from the column boundary x, a top-row pixel from the row boundary y, the top-left corner
// (only ever sample K-1) from whichever of the two its block wrote. Every lane polls its records
// until each carries this launch's epoch, with two rounds of loads in flight (a record that
// turns valid is seen about half a round trip sooner than by one load at a time); bounded like
// the flag wait.
template <int K>
__device__ __forceinline__ void gran_fetch(const GranCtx &g, int x, int y, const int (&yy)[K], const int (&xx)[K],
                                           const bool (&use)[K], int (&out)[K]) {
    const unsigned long long *pa[K], *pc;
    int sa[K], sc = 0;
    bool ok[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        ok[k] = !use[k];
        sa[k] = 0;
        pa[k] = g.col;                                   // (unused samples: any valid record)
        if (!use[k]) continue;
        if (xx[k] == x - 1) {
            pa[k] = g.col + (x >> 2) * g.colp + (yy[k] >> 1);
            sa[k] = (yy[k] & 1) * 16;
        } else {
            pa[k] = g.row + (y >> 2) * g.rowp + (xx[k] >> 1);
            sa[k] = (xx[k] & 1) * 16;
        }
    }
    // the corner's second record (row boundary y), if sample K-1 is the corner
    const bool corner = use[K - 1] && xx[K - 1] == x - 1 && yy[K - 1] == y - 1;
    pc = pa[K - 1];
    if (corner) {
        pc = g.row + (y >> 2) * g.rowp + ((x - 1) >> 1);
        sc = ((x - 1) & 1) * 16;
    }
    auto ld = [](const unsigned long long *q) { return ld_sc1(q); };
    auto take = [&](const unsigned long long (&v)[K], unsigned long long vc) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            if (ok[k]) continue;
            if ((uint32_t)(v[k] >> 32) == g.epoch) {
                out[k] = (int)((v[k] >> sa[k]) & 0xffff);
                ok[k] = true;
            } else if (k == K - 1 && corner && (uint32_t)(vc >> 32) == g.epoch) {
                out[k] = (int)((vc >> sc) & 0xffff);
                ok[k] = true;
            }
        }
        bool all = true;
#pragma unroll
        for (int k = 0; k < K; k++) all = all && ok[k];
        return __builtin_amdgcn_ballot_w64(!all) == 0;
    };
    unsigned long long v0[K], v1[K], c0, c1;
#pragma unroll
    for (int k = 0; k < K; k++) v0[k] = ld(pa[k]);
    c0 = ld(pc);
    for (unsigned spins = 0;; spins++) {
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < K; k++) v1[k] = ld(pa[k]);
        c1 = ld(pc);
        if (take(v0, c0)) break;
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < K; k++) v0[k] = ld(pa[k]);
        c0 = ld(pc);
        if (take(v1, c1)) break;
        if (spins > (1u << MI_IR_GRAN_SPIN_LOG2)) {
            atomicOr(g.err, 1);
            break;
        }
    }
}

// intra_block's result: MI_IR_TIMELINE stamps, and the value of a plain DC-family block that
// was not written to the tile (-1: the tile holds the block)
struct IntraOut {
    unsigned long long tlx;
    int dcv;
};

// Gather one block's edges from the picture (rav1d_prepare_intra_edges) and predict it, one
// wave. Fused (the persistent reconstruction kernel): neighbour pixels were stored by other
// CUs of this XCD during the launch, so every picture read is an L1-bypassing `sc1` load
// (L2-served), and the prediction goes to the LDS tile lt.
template <typename Px, bool Fused>
__device__ __forceinline__ IntraOut intra_block(const IpredArgs &a, const MiIntraBlock &ib, int *eb, Px *ft, Px *edge,
                                            Px *lt, int16_t *acl, const int16_t *res = nullptr, int rdc = 0,
                                            bool use_gran = false, GranCtx gran = {}, bool tlv = false) {
    const int lane = threadIdx.x;
    // MI_IR_TIMELINE stamps 7..10 (lane k keeps stamp k), returned to the caller
    unsigned long long tlx = 0;
#define TLV(k) do { if (tlv) { const unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); if (lane == (k)) tlx = t_; } } while (0)
    const int w = ib.w, h = ib.h, x = ib.x, y = ib.y;
    const int lw = 31 - __clz(w);                // (w a power of two)
    const bool have_left = ib.flags & MI_INTRA_HAVE_LEFT, have_top = ib.flags & MI_INTRA_HAVE_TOP;
    const int64_t st = plane_stride(a, ib.plane);
    const Px *pic = reinterpret_cast<const Px *>(plane_ptr(a, ib.plane));
    auto P = [&](int yy, int xx) -> int {
        const Px *q = reinterpret_cast<const Px *>(reinterpret_cast<const uint8_t *>(pic) + (int64_t)yy * st) + xx;
        if constexpr (Fused) return ld_px_sc1(q);
        else return *q;
    };
    if constexpr (Fused) {
        // inter-intra blends into the block's existing (inter) pixels, and the residual of an
        // inter-intra block (MI_INTRA_RESID) adds to them: start the tile from them
        if ((ib.flags & MI_INTRA_II) || ib.mode == MI_INTRA_RESID)
            for (int i = lane; i < w * h; i += 64) lt[i] = (Px)P(y + (i >> lw), x + (i & (w - 1)));
    }
    if (ib.mode == MI_INTRA_RESID) {
        if constexpr (Fused)
            for (int i = lane; i < w * h; i += 64) lt[i] = (Px)clampi((int)lt[i] + (res ? (int)res[i] : rdc), 0, a.bdmax);
        return { tlx, -1 };
    }
    const int bd = a.bpc;
    if (ib.mode == MI_INTRA_IBC) {
        // intra block copy: bilinear put_bilin_c (mc_tmpl.c) from the already reconstructed
        // source rectangle of this picture (its owners are this block's dependencies)
        const int mvx = (int16_t)(ib.reserved & 0xffff), mvy = (int16_t)(ib.reserved >> 16);
        const int ssh = ib.filt_idx & 1, ssv = (ib.filt_idx >> 1) & 1;
        const int sx = x + (mvx >> (3 + ssh)), sy = y + (mvy >> (3 + ssv));
        const int mx = (mvx & (15 >> !ssh)) << !ssh, my = (mvy & (15 >> !ssv)) << !ssv;
        const int ibits = bd == 8 ? 4 : 14 - bd, bdmax = (1 << bd) - 1;
        auto rnd = [](int v, int sh) { return (v + ((1 << sh) >> 1)) >> sh; };
        // emu_edge (recon.rs:2052-2083, intrabc: the frame's 8-aligned coded size f.bw*4 >> ss_hor
        // by f.bh*4 >> ss_ver, carried in max_w / max_h) replicates the border: clamping every
        // tap coordinate is the same read
        const int cw = ib.max_w - 1, chh = ib.max_h - 1;
        auto Q = [&](int yy, int xx) { return P(min(max(yy, 0), chh), min(max(xx, 0), cw)); };
        for (int i = lane; i < w * h; i += 64) {
            const int yy = (i >> lw), xx = (i & (w - 1)), py = sy + yy, px = sx + xx;
            const int s00 = Q(py, px);
            int v;
            if (mx && my) {
                const int m0 = rnd(16 * s00 + mx * (Q(py, px + 1) - s00), 4 - ibits);
                const int s10 = Q(py + 1, px);
                const int m1 = rnd(16 * s10 + mx * (Q(py + 1, px + 1) - s10), 4 - ibits);
                v = rnd(16 * m0 + my * (m1 - m0), 4 + ibits);
            } else if (mx) {
                v = (rnd(16 * s00 + mx * (Q(py, px + 1) - s00), 4 - ibits) + ((1 << ibits) >> 1)) >> ibits;
            } else if (my) {
                v = rnd(16 * s00 + my * (Q(py + 1, px) - s00), 4);
            } else {
                v = s00;
            }
            v = min(max(v, 0), bdmax);
            if constexpr (Fused) lt[i] = (Px)clampi(v + (res ? (int)res[i] : rdc), 0, bdmax);
            else reinterpret_cast<Px *>(plane_ptr(a, ib.plane) + (int64_t)(y + yy) * st)[x + xx] = (Px)v;
        }
        return { tlx, -1 };
    }

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
        predict_block<Px, Fused>(a, b, reinterpret_cast<const Px *>(a.pal) + ib.pal_off, eb, ft, lt, nullptr, res, rdc);
        return { tlx, -1 };
    }
    // mode remap (ipred_prepare.rs:148-172): all wave-uniform
    const bool cfl = ib.mode == MI_IPRED_CFL;
    int m = cfl ? 0 : ib.mode, angle = 0;
    if (m >= 1 && m <= 8) {
        angle = mode_angle(m - 1) + 3 * ib.angle;
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
    const int needs = needs_of(m);
    Px *tl = edge + 128;
    const int tw4 = w >> 2, th4 = h >> 2;
    // Every edge sample in one round of loads (w, h <= 64: lane i owns sample i of each
    // edge; for i beyond the edge the clamped address is still inside it): left column,
    // bottom-left, top row, top-right and the corner, then the LDS writes. Unavailable parts
    // are filled as rav1d_prepare_intra_edges does (ipred_prepare.rs:118-204).
    const int i = lane;
    const int half = 1 << bd >> 1;
    // the five edge samples of this lane (left, bottom-left, top, top-right, corner): a pixel
    // position, or a constant where the edge is unavailable (ipred_prepare.rs:118-204)
    int py[5], px[5], v[5] = { 0, 0, 0, 0, 0 };
    bool rd[5] = { false, false, false, false, false };
    auto at = [&](int k, int yy, int xx) { py[k] = yy; px[k] = xx; rd[k] = true; };
#pragma unroll
    for (int k = 0; k < 5; k++) py[k] = px[k] = 0;
    if (needs & 1) {
        if (have_left) at(0, y + min(i, min(h, (int)ib.tile_h - y) - 1), x - 1);
        else if (have_top) at(0, y - 1, x);
        else v[0] = half + 1;
        if (needs & 16) {
            const bool hbl = have_left && y + h < (int)ib.tile_h && (ib.flags & MI_INTRA_BOTTOM_LEFT);
            if (hbl) at(1, y + h + min(i, min(h, (int)ib.tile_h - y - h) - 1), x - 1);
            else if (have_left) at(1, y + min(h, (int)ib.tile_h - y) - 1, x - 1);
            else if (have_top) at(1, y - 1, x);
            else v[1] = half + 1;
        }
    }
    if (needs & 2) {
        if (have_top) at(2, y - 1, x + min(i, min(w, (int)ib.tile_w - x) - 1));
        else if (have_left) at(2, y, x - 1);
        else v[2] = half - 1;
        if (needs & 8) {
            const bool htr = have_top && x + w < (int)ib.tile_w && (ib.flags & MI_INTRA_TOP_RIGHT);
            if (htr) at(3, y - 1, x + w + min(i, min(w, (int)ib.tile_w - x - w) - 1));
            else if (have_top) at(3, y - 1, x + min(w, (int)ib.tile_w - x) - 1);
            else if (have_left) at(3, y, x - 1);
            else v[3] = half - 1;
        }
    }
    if (needs & 4) {
        if (have_top) at(4, y - 1, x - (have_left ? 1 : 0));
        else if (have_left) at(4, y, x - 1);
        else v[4] = half;
    }
    if (Fused && use_gran) {
        gran_fetch<5>(gran, x, y, py, px, rd, v);
        TLV(7);
    } else {
#pragma unroll
        for (int k = 0; k < 5; k++)
            if (rd[k]) v[k] = P(py[k], px[k]);
    }
    TLV(8);
    const int vL = v[0], vBL = v[1], vT = v[2], vTR = v[3], vC = v[4];
    // DC family: the edge sum from the registers (lane i holds left[i] and top[i])
    int dcs = -1;
    if (Fused && (m == 0 || m == 3 || m == 4))
        dcs = wave_sum_dpp((m != 3 && i < w ? vT : 0) + (m != 4 && i < h ? vL : 0));
    // a plain DC-family block is one value: returned, no edge staging and no LDS tile (the
    // caller stores dc + residual directly)
    if (Fused && !cfl && !ii && (m == 0 || m == 3 || m == 4 || m == 5))
        return { tlx, m == 5 ? (1 << bd) >> 1 : dc_of_sum(m, dcs, w, h, bd) };
    if ((needs & 1) && i < h) {
        tl[-1 - i] = (Px)vL;
        if (needs & 16) tl[-1 - h - i] = (Px)vBL;
    }
    if ((needs & 2) && i < w) {
        tl[1 + i] = (Px)vT;
        if (needs & 8) tl[1 + w + i] = (Px)vTR;
    }
    __syncthreads();
    if ((needs & 4) && lane == 0) {
        int c = vC;
        if (m == 7 && tw4 + th4 >= 6 && (ib.flags & MI_INTRA_EDGE_FILTER))
            c = ((tl[-1] + tl[1]) * 5 + c * 6 + 8) >> 4;
        tl[0] = (Px)c;
    }
    __syncthreads();
    TLV(9);
    b.mode = (uint8_t)((cfl ? MI_IPRED_CFL + m : m) | ii);
    b.angle = (uint16_t)(angle | (ib.flags & MI_INTRA_SMOOTH_NB ? 512 : 0) | (ib.flags & MI_INTRA_EDGE_FILTER ? 1024 : 0));
    if (m == 13) b.angle = (uint16_t)ib.filt_idx;
    if (cfl && (ib.flags & MI_INTRA_CFL_AC)) {
        // the AC from the reconstructed luma under the block (its dependencies made it final)
        const int ssh = (ib.reserved >> 16) & 1, ssv = (ib.reserved >> 17) & 1;
        const uint8_t *yb = a.dst[0] + (int64_t)(y << ssv) * a.stride[0] + (int64_t)(x << ssh) * sizeof(Px);
        cfl_ac_wave<Px, Fused>(acl, yb, a.stride[0], ib.reserved & 0xff, (ib.reserved >> 8) & 0xff, w, h, ssh, ssv);
        predict_block<Px, Fused>(a, b, tl, eb, ft, lt, acl, res, rdc, dcs);
        return { tlx, -1 };
    }
    predict_block<Px, Fused>(a, b, tl, eb, ft, lt, nullptr, res, rdc, dcs);
    TLV(10);
    return { tlx, -1 };
}

template <typename Px>
__global__ __launch_bounds__(64) void intra_kernel(IpredArgs a) {
    __shared__ int eb[2 * 128 + 2];
    __shared__ Px ft[32 * 32];
    __shared__ Px edge[2 * 128 + 1];           // topleft at [128]
    __shared__ int16_t acl[32 * 32];           // MI_INTRA_CFL_AC
    intra_block<Px, false>(a, a.iblocks[blockIdx.x], eb, ft, edge, nullptr, acl);
}

// ---- persistent fused intra reconstruction (mi_intra_recon) ----
//
// One launch reconstructs whole intra frames: prediction (intra_block) and the residual
// (inverse transform + add) of every transform block, in dependency order, without a launch
// per wavefront step. Queue f -- a frame, or one vertical strip of a single frame
// (frame_exec.cpp) -- is worked on only by the workgroups the dispatcher placed on XCD f
// (HW_REG_XCC_ID): the `sc1` loads below are served by the reading XCD's L2, which may hold a
// line cached before a neighbouring block sharing it was written, so the readers and writers
// of a line share one L2. Strips keep that true: their boundaries are 128-B line boundaries in
// every plane, and a block that reads a line of another strip also depends on every block
// writing that line, so the first read of such a line on this XCD finds it final. A block's
// pixels are published with the hand-off of MI355X_MICROARCH.md's table row 1: 4-/8-B `sc1`
// stores, the storing wave's vmcnt(0), then one lane's `sc1` done-flag store; readers poll the
// flag and read pixels with 4-B `sc1` loads only. Each worker wave
// takes the next block from the frame's queue (an atomic head over blocks in dependency
// order), waits until every block its edges read has been marked done with this launch's
// epoch, predicts into an LDS tile, adds the residual there and stores the tile. Deadlock-free:
// a block only waits on earlier queue entries, which running workers hold. A wait that
// exceeds ~0.5 s flags the context's device error word and gives up (no hang).

#ifndef MI_IR_SPIN_LOG2
#define MI_IR_SPIN_LOG2 22
#endif

__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

// Inverse transform of one block by one wave, in two halves, both from the coefficients only,
// so both run while the block still waits for its neighbours: itx_rows leaves the
// shifted/clipped rows in tmp, or returns the DC-only block's value; itx_cols leaves the w x h
// residual in res (int16), which the prediction's stores add (predict_block's put). The
// per-block semantics of itx_size (itx.hip): lane j = row j, then column j.
template <int TX, typename Px, typename Cf, typename Lt, bool Wide>
__device__ __forceinline__ int itx_rows(const MiTxBlock &b, Cf *cf, bool zero, int bdmax, Lt *tmp) {
    constexpr TxDim D = tx_dim(TX);
    constexpr int Wd = D.w, Ht = D.h, SH = imin_c(Ht, 32), SW = imin_c(Wd, 32);
    constexpr int LS = Wd + 1;
    constexpr bool Rect2 = (Wd == 2 * Ht) || (Ht == 2 * Wd);
    constexpr int Shift = D.shift, Rnd = (1 << Shift) >> 1;
    const int j = threadIdx.x;
    if (b.eob < 0) return 0;  // no residual (skip / prediction only): the arena is not read
    if (b.txtp == 0 && b.eob < 1) {
        int dc = (int)cf[0];
        if (Rect2) dc = (dc * 181 + 128) >> 8;
        dc = (dc * 181 + 128) >> 8;
        dc = (dc + Rnd) >> Shift;
        dc = (dc * 181 + 128 + 2048) >> 12;
        if (zero && j == 0) cf[0] = 0;
        return dc;
    }
    int row_lo, col_lo;
    if constexpr (sizeof(Px) == 1) { row_lo = -32768; col_lo = -32768; }
    else { row_lo = (int)((unsigned)~bdmax << 7); col_lo = (int)((unsigned)~bdmax << 5); }
    const int row_hi = ~row_lo, col_hi = ~col_lo;
    if (j < SH) {
        int r[Wd];
#pragma unroll
        for (int x = 0; x < Wd; x++) r[x] = 0;
        int cv[SW];
        tx_load_row<SW, SH, Cf>(cf, b.flags, j, cv);
#pragma unroll
        for (int x = 0; x < SW; x++) {
            if constexpr (Rect2) r[x] = (cv[x] * 181 + 128) >> 8;
            else r[x] = cv[x];
        }
        if (zero) tx_zero_row<SW, SH, Cf>(cf, b.flags, j);
        if (TX == 0 && b.txtp == 16) {
            if constexpr (TX == 0) {
#pragma unroll
                for (int x = 0; x < 4; x++) r[x] >>= 2;
                iwht4(r);
#pragma unroll
                for (int x = 0; x < 4; x++) tmp[j * LS + x] = (Lt)r[x];
            }
        } else {
            itx1d<Wide, Wd>(row_kind_ip(b.txtp), r, row_lo, row_hi);
#pragma unroll
            for (int x = 0; x < Wd; x++) tmp[j * LS + x] = (Lt)clampi((r[x] + Rnd) >> Shift, col_lo, col_hi);
        }
    }
    return 0;
}

template <int TX, typename Px, typename Lt, bool Wide>
__device__ __forceinline__ void itx_cols(const MiTxBlock &b, int bdmax, int16_t *res, const Lt *tmp) {
    constexpr TxDim D = tx_dim(TX);
    constexpr int Wd = D.w, Ht = D.h, SH = imin_c(Ht, 32);
    constexpr int LS = Wd + 1;
    const int j = threadIdx.x;
    int col_lo;
    if constexpr (sizeof(Px) == 1) col_lo = -32768;
    else col_lo = (int)((unsigned)~bdmax << 5);
    const int col_hi = ~col_lo;
    if (j < Wd) {
        int c[Ht];
#pragma unroll
        for (int y = 0; y < Ht; y++) c[y] = y < SH ? (int)tmp[y * LS + j] : 0;
        if (TX == 0 && b.txtp == 16) {
            if constexpr (TX == 0) {
                iwht4(c);
#pragma unroll
                for (int y = 0; y < 4; y++) res[y * Wd + j] = (int16_t)clampi(c[y], -32768, 32767);
            }
        } else {
            itx1d<Wide, Ht>(col_kind_ip(b.txtp), c, col_lo, col_hi);
            // (c + 8) >> 4 does NOT always fit int16: the identity column transforms are not
            // clipped (itx_1d.rs:1106-1121), so at 12 bpc identity32 reaches 4 * 131071 and the
            // residual +32768. Saturating is exact: any |r| > 32767 exceeds
            // bdmax, and the pixel clips to the same bound as with the unsaturated int
#pragma unroll
            for (int y = 0; y < Ht; y++) res[y * Wd + j] = (int16_t)clampi((c[y] + 8) >> 4, -32768, 32767);
        }
    }
}

// An opaque copy into a scalar register: the value is then no longer a (rematerialisable)
// kernel-argument load
template <typename T>
__device__ __forceinline__ T sreg(T v) {
    asm volatile("" : "+s"(v));
    return v;
}
// ... for a pointer, through a global-address-space copy, so that its uses stay `global_` /
// `s_load` accesses (a laundered generic pointer would make every access a flat one)
template <typename T>
__device__ __forceinline__ T *sreg(T *v) {
    typedef __attribute__((address_space(1))) T *G;
    G g = (G)v;
    asm volatile("" : "+s"(g));
    return (T *)g;
}
__device__ __forceinline__ IntraReconFrame frame_regs(const IntraReconFrame &g) {
    IntraReconFrame f;
    for (int p = 0; p < 3; p++) f.ip.dst[p] = sreg(g.ip.dst[p]);
    f.ip.stride[0] = sreg(g.ip.stride[0]);
    f.ip.stride[1] = sreg(g.ip.stride[1]);
    f.ip.blocks = nullptr;
    f.ip.edges = nullptr;
    f.ip.ac = sreg(g.ip.ac);
    f.ip.idx = sreg(g.ip.idx);
    f.ip.iblocks = sreg(g.ip.iblocks);
    f.ip.pal = sreg(g.ip.pal);
    f.ip.bpc = sreg(g.ip.bpc);
    f.ip.bdmax = sreg(g.ip.bdmax);
    f.tx = sreg(g.tx);
    f.coef = sreg(g.coef);
    f.dep_start = sreg(g.dep_start);
    f.deps = sreg(g.deps);
    f.done = sreg(g.done);
    f.head = sreg(g.head);
    f.n = sreg(g.n);
    f.base = sreg(g.base);
    f.pw = (uint16_t)sreg((int)g.pw);
    f.ph = (uint16_t)sreg((int)g.ph);
    f.ss_hor = (uint8_t)sreg((int)g.ss_hor);
    f.ss_ver = (uint8_t)sreg((int)g.ss_ver);
    f.nplanes = (uint8_t)sreg((int)g.nplanes);
    f.pad_ = 0;
    f.goff = sreg(g.goff);
    return f;
}

template <typename Px, typename Cf, typename Lt, bool Wide>
__global__ __launch_bounds__(64) void intra_recon_kernel(IntraReconArgs a) {
    __shared__ int eb[2 * 128 + 2];
    __shared__ Px ft[32 * 32];
    __shared__ Px edge[2 * 128 + 1];
    __shared__ int16_t acl[32 * 32];           // MI_INTRA_CFL_AC
    // the row pass's tmp and the block's tile lt share their LDS: tmp lives from the row pass
    // to the column pass (before the dependency wait), lt from the prediction to the stores
    constexpr int kLtB = 64 * 64 * (int)sizeof(Px), kTmpB = 32 * 65 * (int)sizeof(Lt);
    __shared__ __attribute__((aligned(16))) unsigned char lt_tmp[kLtB > kTmpB ? kLtB : kTmpB];
    Px *const lt = reinterpret_cast<Px *>(lt_tmp);
    Lt *const tmp = reinterpret_cast<Lt *>(lt_tmp);
    __shared__ int16_t res[64 * 64];            // the block's residual (itx_cols)
    const unsigned xcc = xcc_id();
#ifdef MI_IR_DEBUG
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(a.dbg + 16 + (xcc & 7), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_fetch_add(a.dbg + 32 + (blockIdx.x & 7), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#define DBG(i, v) __hip_atomic_store(a.dbg + 64 + (i), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
#else
#define DBG(i, v) do {} while (0)
#endif
    // MI_IR_TIMELINE: stamp k of the current unit into lane k's tl_v (one store per unit)
    unsigned long long tl_v = 0;
#define TL(k) do { if (tl_base) { const unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); if (threadIdx.x == (k)) tl_v = t_; } } while (0)
    // queues xcc, xcc + 8, ... (frames, or the strips of one frame) belong to this XCD; its
    // workers are dealt over them round robin
    const int lane = threadIdx.x;
    const int nper = (a.nframes - (int)xcc + 7) >> 3;
    if (nper <= 0) return;
    const int rank = __builtin_amdgcn_readfirstlane(atomicAdd(a.xcd_rank + xcc, lane == 0 ? 1 : 0));
    const int fidx = xcc + 8 * (rank % nper);
    // the queue's descriptor and the launch constants in registers for the whole launch: read
    // at each use they are scalar loads of the kernel arguments, which the descriptors streaming
    // through the scalar cache evict (a miss on the critical path of every block)
    const IntraReconFrame fr = frame_regs(a.fr[fidx]);
    const uint32_t epoch = sreg(a.epoch);
    unsigned long long *const gran = sreg(a.gran);
    int *const err = sreg(a.err), *const desc_err = sreg(a.desc_err);
    const uintptr_t tl_base = sreg(a.tl);
    const int zero_coefs = sreg(a.zero_coefs);
    for (;;) {
        // The block index must be provably wave-uniform and the loop free of lane-divergent
        // branches: otherwise the structurizer may run lanes 1..63 into the next iteration
        // ahead of lane 0's pop (observed: a livelock on the same block)
        // (every lane executes the pop, lane 0 adds 1 and the others 0, so no lane-divergent
        // branch exists at loop level)
        // (popping the next block ahead, to hide the atomic, measured slower: 6.8 -> 8.1 ms
        // per 1080p frame, a worker blocked on its first block also holds the second)
        const int i = __builtin_amdgcn_readfirstlane(atomicAdd(fr.head, lane == 0 ? 1 : 0));
        if (i >= fr.n) return;
        unsigned long long *tl =
            tl_base ? reinterpret_cast<unsigned long long *>(tl_base + (uintptr_t)(fr.done + fr.base + i) * 32) : nullptr;
        TL(0);
        DBG(i, 1);
        const MiIntraBlock ib = fr.ip.iblocks[i];
        const MiTxBlock tb = fr.tx[i];
        {
            // a descriptor the reference could never issue (plane / rectangle outside the
            // picture, a residual of another size or position, an illegal transform type) is
            // skipped, reported, and still marked done so that no worker waits on it forever
            const int sh = ib.plane ? fr.ss_hor : 0, sv = ib.plane ? fr.ss_ver : 0;
            const TxDim td = tx_dim(tb.tx < 19 ? tb.tx : 0);
            const bool ok_ = ib.plane < fr.nplanes && ib.x + ib.w <= (fr.pw >> sh) && ib.y + ib.h <= (fr.ph >> sv) &&
                            tb.tx < 19 && td.w == ib.w && td.h == ib.h && tb.x == ib.x && tb.y == ib.y &&
                            tb.plane == ib.plane && (tb.eob < 0 || (tb.txtp < 17 && ((itx_legal_types(tb.tx) >> tb.txtp) & 1) &&
                                                                    tx_flags_ok(tb.flags, imin_c(td.w, 32), imin_c(td.h, 32), tb.coef_off, sizeof(Cf) == 4)));
            const bool ok = __builtin_amdgcn_readfirstlane((int)ok_) != 0;
            if (!ok) {
                if (lane == 0) {
                    atomicOr(desc_err, 2);
                    __hip_atomic_store(fr.done + fr.base + i, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                continue;
            }
        }
        // the residual's row pass needs only the coefficients: before the dependency wait
        Cf *cf = reinterpret_cast<Cf *>(fr.coef) + tb.coef_off;
        int dc = 0;
        switch (tb.tx) {
#define CASE(n) case n: dc = itx_rows<n, Px, Cf, Lt, Wide>(tb, cf, zero_coefs, fr.ip.bdmax, tmp); break;
            CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9)
            CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16) CASE(17) CASE(18)
#undef CASE
        default: break;
        }
        // the column pass too (the residual), unless the block is DC-only (a constant dc)
        const bool dconly = tb.eob < 0 || (tb.txtp == 0 && tb.eob < 1);
        if (!dconly) {
            __syncthreads();
            switch (tb.tx) {
#define CASE(n) case n: itx_cols<n, Px, Lt, Wide>(tb, fr.ip.bdmax, res, tmp); break;
                CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9)
                CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16) CASE(17) CASE(18)
#undef CASE
            default: break;
            }
        }
        TL(1);
        // wait for the blocks this one's edges read; wave-uniform loop exits (a ballot). With
        // edge granules only CfL (its luma) and intra block copy (its source) read pixels of
        // other blocks outside the granules
        const int d0 = fr.dep_start[i];
        const int d1 = gran && ib.mode != MI_IPRED_CFL && ib.mode != MI_INTRA_IBC ? d0 : fr.dep_start[i + 1];
        for (int base = d0; base < d1; base += 64) {
            const int d = base + lane;
            const uint32_t *flag = fr.done + (d < d1 ? fr.deps[d] : 0);
            bool ok = d >= d1;
            for (unsigned spins = 0;; spins++) {
                if (!ok) ok = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
                if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
                if (spins > (1u << MI_IR_SPIN_LOG2)) {
                    atomicOr(err, 1);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        DBG(i, 2);
        TL(2);
        GranCtx gc = {};
        if (gran)
            gc = gran_ctx(gran + fr.goff, fr.pw, fr.ph, fr.ss_hor, fr.ss_ver, fr.nplanes, ib.plane, epoch, err);
        int dcv;
        {
            const IntraOut o = intra_block<Px, true>(fr.ip, ib, eb, ft, edge, lt, acl, dconly ? nullptr : res, dc,
                                                     gran != nullptr, gc, tl_base != 0);
            dcv = o.dcv;
            if (lane >= 7 && lane <= 10) tl_v = o.tlx;
        }
        // pixel (yy, xx) of the reconstructed block: the LDS tile, or a DC-family block's value
        // plus the residual (res was complete before the dependency wait's barrier)
        const bool direct = dcv >= 0;
        const int bdmax_ = fr.ip.bdmax;
        auto pix = [&](int yy, int xx) -> uint32_t {
            if (direct) return (uint32_t)clampi(dcv + (dconly ? dc : (int)res[yy * ib.w + xx]), 0, bdmax_);
            return lt[yy * ib.w + xx];
        };
        if (!direct) __syncthreads();
        DBG(i, 3);
        TL(3);
        TL(4);
        if (gran) {
            // the edges later blocks read, as granules: right column (lanes 0..h/2-1), bottom
            // row (lanes 32..32+w/2-1), before the tile's own stores
            const int w = ib.w, h = ib.h;
            unsigned long long *gd = nullptr;
            uint32_t p0 = 0, p1 = 0;
            if (lane < (h >> 1)) {
                const int r = 2 * lane;
                p0 = pix(r, w - 1);
                p1 = pix(r + 1, w - 1);
                gd = gc.col + ((ib.x + w) >> 2) * gc.colp + ((ib.y + r) >> 1);
            } else if (lane >= 32 && lane - 32 < (w >> 1)) {
                const int c = 2 * (lane - 32);
                p0 = pix(h - 1, c);
                p1 = pix(h - 1, c + 1);
                gd = gc.row + ((ib.y + h) >> 2) * gc.rowp + ((ib.x + c) >> 1);
            }
            if (gd)
                __hip_atomic_store(gd, (unsigned long long)(p0 | (p1 << 16)) | ((unsigned long long)epoch << 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // store the reconstructed tile: 4-pixel chunks, 4-B (8 bpc) / 8-B (hbd) `sc1` stores
        {
            const int w = ib.w, h = ib.h, cpr = w >> 2, lcpr = 29 - __clz(w);
            const int64_t st = plane_stride(fr.ip, ib.plane);
            uint8_t *base = plane_ptr(fr.ip, ib.plane) + (int64_t)ib.y * st + (int64_t)ib.x * sizeof(Px);
            for (int c = lane; c < h * cpr; c += 64) {
                const int yy = c >> lcpr, xx = (c & (cpr - 1)) * 4;
                const uint32_t q0 = pix(yy, xx), q1 = pix(yy, xx + 1), q2 = pix(yy, xx + 2), q3 = pix(yy, xx + 3);
                if constexpr (sizeof(Px) == 2)
                    __hip_atomic_store(reinterpret_cast<uint64_t *>(base + yy * st + xx * 2),
                                       (uint64_t)(q0 | (q1 << 16)) | ((uint64_t)(q2 | (q3 << 16)) << 32),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    __hip_atomic_store(reinterpret_cast<uint32_t *>(base + yy * st + xx),
                                       q0 | (q1 << 8) | (q2 << 16) | (q3 << 24), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        DBG(i, 7);
        TL(5);
        // hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, table row 1): every byte
        // stored `sc1`, the storing wave drains its stores, then ONE lane stores the flag `sc1`
        // (agent scope); consumers poll it with `sc1` loads and read the pixels with 4-B `sc1`
        // loads (ld_px_sc1). Each worker workgroup is one wave.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        DBG(i, 8);
        __syncthreads();
        DBG(i, 4);
        if (lane == 0) __hip_atomic_store(fr.done + fr.base + i, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        TL(6);
        if (tl && lane < 16) tl[lane] = tl_v;   // (stamps kept in lane k's register until here)
    }
#undef TL
}

// After the persistent launch, in stream order: every frame's queue head must have passed its
// block count (a frame whose XCD received no workgroup would be left untouched). Sets bit 2 of
// the sticky error word mi_frame_end reports, so a failure of any launch is seen, not only of
// the last one.
__global__ __launch_bounds__(64) void intra_recon_check_kernel(IntraReconArgs a) {
    const int f = threadIdx.x;
    if (f < a.nframes && *a.fr[f].head < a.fr[f].n) atomicOr(a.err, 4);
}

int launch_intra_recon(const IntraReconArgs &a, int bpc, int wg_per_xcd, hipStream_t s) {
    const int n = 8 * wg_per_xcd;
    if (bpc == 8) intra_recon_kernel<uint8_t, int16_t, int16_t, false><<<n, 64, 0, s>>>(a);
    else if (bpc == 10) intra_recon_kernel<uint16_t, int32_t, int16_t, false><<<n, 64, 0, s>>>(a);
    else intra_recon_kernel<uint16_t, int32_t, int32_t, true><<<n, 64, 0, s>>>(a);
    intra_recon_check_kernel<<<1, 64, 0, s>>>(a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---- cfl_ac (ipred.rs:1326-1432; C ipred_tmpl.c:658-700) ----
// The chroma block's AC of the (subsampled) luma: each sample is the sum of its 1/2/4 luma
// pixels scaled to <<3 total, w_pad / h_pad 4-px groups replicated from the last real
// column / row, then the rounded mean subtracted. One wave, the mean by a wave reduction.
template <typename Px>
__global__ __launch_bounds__(64) void cfl_ac_kernel(CflAcArgs a) {
    cfl_ac_wave<Px, false>(a.ac, a.y, a.stride, a.w_pad, a.h_pad, a.cw, a.ch, a.ss_hor, a.ss_ver);
}

int launch_cfl_ac(const CflAcArgs &a, int bpc, hipStream_t s) {
    if (bpc == 8) cfl_ac_kernel<uint8_t><<<1, 64, 0, s>>>(a);
    else cfl_ac_kernel<uint16_t><<<1, 64, 0, s>>>(a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
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
