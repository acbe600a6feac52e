// mc.hip — frame-batched motion compensation on gfx950.
//
// Replaces the per-block `mc()` driver and compound dispatch of recon (rav1d src/recon.rs:
// 2025-2203, 3236-3428; C recon_tmpl.c:962-1011, 1836-1921) and the DSP mc[10]/mct[10]
// (8-tap and bilinear put/prep), avg, w_avg, mask, w_mask (src/mc.rs; C mc_tmpl.c).
//
// One wave per prediction unit (a block's rectangle in one plane, up to 128x128). The unit is
// cut into tiles of TW = min(w, 64) columns; the wave's 64 lanes form G = 64 / TW groups of
// TW lanes, each group owning up to 16 consecutive rows, so a tile has TH = min(h, 16 G) rows.
// Per tile and reference: the (TH+7) x (TW+7) reference window is staged in LDS with clamped
// coordinates (identical to emu_edge's edge replication, mc_tmpl.c:798-845), the horizontal
// pass writes TH+7 rows of intermediates to LDS, and each lane runs the vertical pass down its
// column with an 8-entry register window. Compound predictions keep both references' prep
// values in registers and blend them before a single coalesced store.
#include "common.h"

namespace mi {

__constant__ int8_t k_subpel[6][15][8] = {
#include "tables/mc_subpel_filters.inc"
};

constexpr int kWinMax = 1640;    // max (TH+7)*(TW+7) over unit shapes (23*71, 71*23, 39*39)
constexpr int kMidMax = 1480;    // max (TH+7)*TW (23*64, 71*16, 39*32)

// filter2d (Filter2d, horizontal/vertical order) -> subpel filter types (0 regular, 1 smooth, 2 sharp)
__device__ __forceinline__ int f2d_type_h(int f) { return (int)((0x111222000ull >> (4 * f)) & 15); }
__device__ __forceinline__ int f2d_type_v(int f) { return (int)((0x210210210ull >> (4 * f)) & 15); }

// Taps of one direction: 8 ints (bilinear as [0,0,0,16-m,m,0,0,0]); has = filter present.
struct Taps {
    int f[8];
    bool has;
};

__device__ __forceinline__ Taps make_taps(int m, int n, int type, bool bilin) {
    Taps t;
    t.has = m != 0;
#pragma unroll
    for (int k = 0; k < 8; k++) t.f[k] = 0;
    if (!t.has) return t;
    if (bilin) {
        t.f[3] = 16 - m;
        t.f[4] = m;
    } else {
        const int row = n > 4 ? type : 3 + (type & 1);
#pragma unroll
        for (int k = 0; k < 8; k++) t.f[k] = k_subpel[row][m - 1][k];
    }
    return t;
}

struct McUnit {
    int x, y, w, h, plane, filter2d, nref, comp, param;
    int mvx[2], mvy[2], ref[2];
    uint32_t mask_off;
};

__device__ __forceinline__ McUnit load_unit(const MiMcBlock *b) {
    McUnit u;
    u.x = b->x; u.y = b->y; u.w = b->w; u.h = b->h;
    u.plane = b->plane; u.filter2d = b->filter2d;
    u.mvx[0] = b->mvx[0]; u.mvx[1] = b->mvx[1];
    u.mvy[0] = b->mvy[0]; u.mvy[1] = b->mvy[1];
    u.ref[0] = b->ref[0]; u.ref[1] = b->ref[1];
    u.nref = b->ref[1] >= 0 ? 2 : 1;
    u.comp = b->comp; u.param = b->param;
    u.mask_off = b->mask_off;
    return u;
}

template <typename Px>
__device__ __forceinline__ int ldpx(const uint8_t *base, int64_t stride, int y, int x) {
    return reinterpret_cast<const Px *>(base + (int64_t)y * stride)[x];
}

// One reference's prediction for the tile (tx0, ty0) of unit u: put (pixel) or prep (int16
// intermediate) values for this lane's rows, out[q] for row g*R + q, column c.
template <typename Px, bool PREP>
__device__ __forceinline__ void predict_tile(const McArgs &a, const McUnit &u, int i, int tx0, int ty0,
                                             int TW, int TH, int R, int16_t *win, int16_t *mid, int out[16]) {
    const int lane = threadIdx.x;
    const int p = u.plane;
    const int ssh = p && a.layout != 3, ssv = p && a.layout == 1;
    const int r = u.ref[i];
    const int mvx = u.mvx[i], mvy = u.mvy[i];
    const int mx = (mvx & (15 >> !ssh)) << !ssh, my = (mvy & (15 >> !ssv)) << !ssv;
    const int dx = u.x + (mvx >> (3 + ssh)) + tx0, dy = u.y + (mvy >> (3 + ssv)) + ty0;
    const uint8_t *ref = a.ref[r][p];
    const int64_t rs = a.ref_stride[r][p ? 1 : 0];
    const int iw = a.ref_w[r][p], ih = a.ref_h[r][p];
    const bool bilin = u.filter2d == 9;
    const Taps fh = make_taps(mx, u.w, bilin ? 0 : f2d_type_h(u.filter2d), bilin);
    const Taps fv = make_taps(my, u.h, bilin ? 0 : f2d_type_v(u.filter2d), bilin);
    const int SH = bilin ? 4 : 6, ib = a.ib;

    // stage the window: rows dy-3 .. dy+TH+3, cols dx-3 .. dx+TW+3, clamped to the plane
    const int WC = TW + 7, WR = TH + 7, NW = WC * WR;
    const uint32_t inv = (1u << 20) / WC + 1;          // (k * inv) >> 20 == k / WC for k < 2^20 / WC^2
    __syncthreads();                                   // previous users of win / mid are done
    for (int k = lane; k < NW; k += 64) {
        const int rr = (int)(((uint32_t)k * inv) >> 20), cc = k - rr * WC;
        const int yy = min(max(dy - 3 + rr, 0), ih - 1), xx = min(max(dx - 3 + cc, 0), iw - 1);
        win[k] = (int16_t)ldpx<Px>(ref, rs, yy, xx);
    }
    __syncthreads();

    const int c = lane & (TW - 1), g = lane / TW;
    const int r0 = g * R;
    if (fh.has) {
        // horizontal pass: mid[rr][cc] for rr in [0, WR) when a vertical filter follows,
        // else only this lane's rows 3 .. TH+2 are needed (computed directly below)
        if (fv.has) {
            for (int k = lane; k < WR * TW; k += 64) {
                const int rr = k / TW, cc = k & (TW - 1);
                const int16_t *w = win + rr * WC + cc;
                int s = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) s += fh.f[t] * w[t];
                mid[k] = (int16_t)((s + ((1 << (SH - ib)) >> 1)) >> (SH - ib));
            }
            __syncthreads();
            if (r0 < TH) {
                int v[8];
                const int16_t *m = mid + r0 * TW + c;
#pragma unroll
                for (int t = 0; t < 7; t++) v[t] = m[t * TW];
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    if (q < R) {
                        v[7] = m[(q + 7) * TW];
                        int s = 0;
#pragma unroll
                        for (int t = 0; t < 8; t++) s += fv.f[t] * v[t];
                        out[q] = PREP ? ((s + ((1 << SH) >> 1)) >> SH) - a.bias
                                      : min(max((s + ((1 << (SH + ib)) >> 1)) >> (SH + ib), 0), a.bdmax);
#pragma unroll
                        for (int t = 0; t < 7; t++) v[t] = v[t + 1];
                    }
                }
            }
        } else if (r0 < TH) {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                if (q < R) {
                    const int16_t *w = win + (r0 + q + 3) * WC + c;
                    int s = 0;
#pragma unroll
                    for (int t = 0; t < 8; t++) s += fh.f[t] * w[t];
                    const int px = (s + ((1 << (SH - ib)) >> 1)) >> (SH - ib);
                    out[q] = PREP ? px - a.bias : min(max((px + ((1 << ib) >> 1)) >> ib, 0), a.bdmax);
                }
            }
        }
    } else if (r0 < TH) {
        if (fv.has) {
            int v[8];
            const int16_t *w = win + r0 * WC + c + 3;
#pragma unroll
            for (int t = 0; t < 7; t++) v[t] = w[t * WC];
#pragma unroll
            for (int q = 0; q < 16; q++) {
                if (q < R) {
                    v[7] = w[(q + 7) * WC];
                    int s = 0;
#pragma unroll
                    for (int t = 0; t < 8; t++) s += fv.f[t] * v[t];
                    out[q] = PREP ? ((s + ((1 << (SH - ib)) >> 1)) >> (SH - ib)) - a.bias
                                  : min(max((s + ((1 << SH) >> 1)) >> SH, 0), a.bdmax);
#pragma unroll
                    for (int t = 0; t < 7; t++) v[t] = v[t + 1];
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; q++)
                if (q < R) {
                    const int px = win[(r0 + q + 3) * WC + c + 3];
                    out[q] = PREP ? (px << ib) - a.bias : px;
                }
        }
    }
}

template <typename Px>
__global__ __launch_bounds__(64) void mc_kernel(McArgs a, int first) {
    __shared__ int16_t win[kWinMax];
    __shared__ int16_t mid[kMidMax];
    __shared__ uint8_t mtile[1024];            // SEG: per-pixel blend weights of the tile (TH*TW <= 1024)
    const McUnit u = load_unit(&a.blocks[first + blockIdx.x]);
    const int lane = threadIdx.x;
    const int TW = min(u.w, 64), G = 64 / TW, TH = min(u.h, 16 * G);
    const int R = (TH + G - 1) / G;
    const int c = lane & (TW - 1), g = lane / TW, r0 = g * R;
    const int p = u.plane;
    const int64_t ds = a.dst_stride[p ? 1 : 0];
    uint8_t *dst = a.dst[p];
    const int sign = u.param >> 7;

    for (int ty0 = 0; ty0 < u.h; ty0 += TH) {
        for (int tx0 = 0; tx0 < u.w; tx0 += TW) {
            int o0[16], o1[16];
            if (u.nref == 1) {
                predict_tile<Px, false>(a, u, 0, tx0, ty0, TW, TH, R, win, mid, o0);
#pragma unroll
                for (int q = 0; q < 16; q++)
                    if (q < R && r0 + q < TH)
                        reinterpret_cast<Px *>(dst + (int64_t)(u.y + ty0 + r0 + q) * ds)[u.x + tx0 + c] = (Px)o0[q];
                continue;
            }
            predict_tile<Px, true>(a, u, 0, tx0, ty0, TW, TH, R, win, mid, o0);
            predict_tile<Px, true>(a, u, 1, tx0, ty0, TW, TH, R, win, mid, o1);
            const int ib = a.ib;
            if (u.comp == MI_MC_SEG) {
                // w_mask (mc_tmpl.c:661-712): per-pixel weight from |t1 - t2| (t1 = tmp[sign])
                const int mask_sh = a.bpc + ib - 4, mask_rnd = 1 << (mask_sh - 5);
                const int sh = ib + 6, rnd = (32 << ib) + a.bias * 64;
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    if (q < R && r0 + q < TH) {
                        const int t1 = sign ? o1[q] : o0[q], t2 = sign ? o0[q] : o1[q];
                        const int m = min(38 + ((abs(t1 - t2) + mask_rnd) >> mask_sh), 64);
                        mtile[(r0 + q) * TW + c] = (uint8_t)m;
                        o0[q] = min(max((t1 * m + t2 * (64 - m) + rnd) >> sh, 0), a.bdmax);
                    }
                }
                __syncthreads();
                // chroma-resolution mask (w_mask_444/422/420 by the chroma layout)
                const int msh = a.seg_ss_hor, msv = a.seg_ss_ver;
                const int mw = TW >> msh, mh = TH >> msv, mstride = u.w >> msh;
                uint8_t *mo = a.masks + u.mask_off + (ty0 >> msv) * mstride + (tx0 >> msh);
                for (int k = lane; k < mw * mh; k += 64) {
                    const int yy = k / mw, xx = k - yy * mw;
                    const uint8_t *m0 = mtile + (yy << msv) * TW + (xx << msh);
                    int v;
                    if (msh && msv) v = (m0[0] + m0[1] + m0[TW] + m0[TW + 1] + 2 - sign) >> 2;
                    else if (msh) v = (m0[0] + m0[1] + 1 - sign) >> 1;
                    else v = m0[0];
                    mo[yy * mstride + xx] = (uint8_t)v;
                }
            } else {
                const uint8_t *mk = a.masks + u.mask_off;
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    if (q < R && r0 + q < TH) {
                        int v;
                        if (u.comp == MI_MC_AVG) {
                            v = (o0[q] + o1[q] + (1 << ib) + a.bias * 2) >> (ib + 1);
                        } else if (u.comp == MI_MC_WAVG) {
                            const int wt = u.param & 31;
                            v = (o0[q] * wt + o1[q] * (16 - wt) + (8 << ib) + a.bias * 16) >> (ib + 4);
                        } else {
                            const int m = mk[(ty0 + r0 + q) * u.w + tx0 + c];
                            const int t1 = sign ? o1[q] : o0[q], t2 = sign ? o0[q] : o1[q];
                            v = (t1 * m + t2 * (64 - m) + (32 << ib) + a.bias * 64) >> (ib + 6);
                        }
                        o0[q] = min(max(v, 0), a.bdmax);
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 16; q++)
                if (q < R && r0 + q < TH)
                    reinterpret_cast<Px *>(dst + (int64_t)(u.y + ty0 + r0 + q) * ds)[u.x + tx0 + c] = (Px)o0[q];
        }
    }
}

int launch_mc(const McArgs &a, int first, int count, hipStream_t s) {
    if (count <= 0) return 0;
    if (a.bpc == 8) mc_kernel<uint8_t><<<count, 64, 0, s>>>(a, first);
    else mc_kernel<uint16_t><<<count, 64, 0, s>>>(a, first);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
