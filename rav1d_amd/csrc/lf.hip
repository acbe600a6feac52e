// lf.hip — whole-frame deblocking on gfx950.
//
// Replaces rav1d_loopfilter_sbrow_cols/_rows (rav1d src/lf_apply.rs:597-834) and the DSP
// loop_filter_sb[2][2] (src/loopfilter.rs:396-985; C src/loopfilter_tmpl.c:37-250).
//
// Two launches per frame: every column edge of every plane, then every row edge. Within one
// direction the AV1 edge set has disjoint read/write footprints (a filter of width wd needs
// blocks >= wd/2.. on both sides: SURVEY.md App. B.2), so each direction is one fully
// parallel in-place pass and the result equals the reference's sbrow interleaving.
//
// One lane = one pixel line crossing one 4-px edge unit (the reference decides fm/flat/hev per
// line, loopfilter.rs:396-721). Column-edge lanes: 64 consecutive units of one pixel row per
// wave (each lane touches a 16-px window; the wave sweeps ~512 contiguous bytes of the row).
// Row-edge lanes: 64 consecutive pixel columns per wave (every access a coalesced row read).
#include "common.h"

namespace mi {


template <typename Px>
__device__ __forceinline__ void filter_line(Px *q0p, int64_t s, int wd, int E, int I, int H,
                                            int bdm8, int bdmax) {
    const int F = 1 << bdm8;
    E <<= bdm8; I <<= bdm8; H <<= bdm8;
    const int p1 = q0p[-2 * s], p0 = q0p[-s], q0 = q0p[0], q1 = q0p[s];
    int p2 = 0, q2 = 0, p3 = 0, q3 = 0;
    bool fm = abs(p1 - p0) <= I && abs(q1 - q0) <= I && abs(p0 - q0) * 2 + (abs(p1 - q1) >> 1) <= E;
    if (wd > 4) {
        p2 = q0p[-3 * s]; q2 = q0p[2 * s];
        fm = fm && abs(p2 - p1) <= I && abs(q2 - q1) <= I;
        if (wd > 6) {
            p3 = q0p[-4 * s]; q3 = q0p[3 * s];
            fm = fm && abs(p3 - p2) <= I && abs(q3 - q2) <= I;
        }
    }
    if (!fm) return;
    bool flat_in = false, flat_out = false;
    if (wd >= 6) flat_in = abs(p2 - p0) <= F && abs(p1 - p0) <= F && abs(q1 - q0) <= F && abs(q2 - q0) <= F;
    if (wd >= 8) flat_in = flat_in && abs(p3 - p0) <= F && abs(q3 - q0) <= F;
    if (wd == 16 && flat_in) {
        const int p6 = q0p[-7 * s], p5 = q0p[-6 * s], p4 = q0p[-5 * s];
        const int q4 = q0p[4 * s], q5 = q0p[5 * s], q6 = q0p[6 * s];
        flat_out = abs(p6 - p0) <= F && abs(p5 - p0) <= F && abs(p4 - p0) <= F &&
                   abs(q4 - q0) <= F && abs(q5 - q0) <= F && abs(q6 - q0) <= F;
        if (flat_out) {
            // 13-output smoother: each output is a 16-weight window over p6..q6 with the
            // outermost sample repeated (loopfilter.rs wd16 branch)
            int v[14] = { p6, p5, p4, p3, p2, p1, p0, q0, q1, q2, q3, q4, q5, q6 };
            int o[12];
#pragma unroll
            for (int k = 0; k < 12; k++) {
                // output position k corresponds to v[k+1] (p5..q5)
                int sum = 8;
#pragma unroll
                for (int t = -6; t <= 6; t++) {
                    int idx = k + 1 + t;
                    idx = idx < 0 ? 0 : idx > 13 ? 13 : idx;
                    sum += v[idx] * ((t >= -1 && t <= 1) ? 2 : 1);
                }
                o[k] = sum >> 4;
            }
#pragma unroll
            for (int k = 0; k < 6; k++) q0p[-(6 - k) * s] = (Px)o[k];
#pragma unroll
            for (int k = 0; k < 6; k++) q0p[k * s] = (Px)o[6 + k];
            return;
        }
    }
    if (wd >= 8 && flat_in) {
        q0p[-3 * s] = (Px)((3 * p3 + 2 * p2 + p1 + p0 + q0 + 4) >> 3);
        q0p[-2 * s] = (Px)((2 * p3 + p2 + 2 * p1 + p0 + q0 + q1 + 4) >> 3);
        q0p[-1 * s] = (Px)((p3 + p2 + p1 + 2 * p0 + q0 + q1 + q2 + 4) >> 3);
        q0p[0] = (Px)((p2 + p1 + p0 + 2 * q0 + q1 + q2 + q3 + 4) >> 3);
        q0p[s] = (Px)((p1 + p0 + q0 + 2 * q1 + q2 + 2 * q3 + 4) >> 3);
        q0p[2 * s] = (Px)((p0 + q0 + q1 + 2 * q2 + 3 * q3 + 4) >> 3);
    } else if (wd == 6 && flat_in) {
        q0p[-2 * s] = (Px)((3 * p2 + 2 * p1 + 2 * p0 + q0 + 4) >> 3);
        q0p[-1 * s] = (Px)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
        q0p[0] = (Px)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
        q0p[s] = (Px)((p0 + 2 * q0 + 2 * q1 + 3 * q2 + 4) >> 3);
    } else {
        const int dlo = -(128 << bdm8), dhi = (128 << bdm8) - 1;
        const bool hev = abs(p1 - p0) > H || abs(q1 - q0) > H;
        int f = hev ? min(max(p1 - q1, dlo), dhi) : 0;
        f = min(max(3 * (q0 - p0) + f, dlo), dhi);
        const int f1 = min(f + 4, dhi) >> 3;
        const int f2 = min(f + 3, dhi) >> 3;
        q0p[-s] = (Px)min(max(p0 + f2, 0), bdmax);
        q0p[0] = (Px)min(max(q0 - f1, 0), bdmax);
        if (!hev) {
            const int g = (f1 + 1) >> 1;
            q0p[-2 * s] = (Px)min(max(p1 + g, 0), bdmax);
            q0p[s] = (Px)min(max(q1 - g, 0), bdmax);
        }
    }
}

__device__ __forceinline__ int lvl_at(const LfArgs &a, int uy, int ux, int slot) {
    return (a.level[(int64_t)uy * a.b4_stride + ux] >> (8 * slot)) & 0xff;
}

// ---- column edges (filtering along rows) ----
// E/I limits of the frame's sharpness (Av1FilterLUT) staged in LDS: lanes index them with
// their own level, which would otherwise be divergent reads of the kernel-argument segment.
__device__ __forceinline__ void stage_lut(const LfArgs &a, uint8_t *le, uint8_t *li) {
    if (threadIdx.x < 64) { le[threadIdx.x] = a.lim_e[threadIdx.x]; li[threadIdx.x] = a.lim_i[threadIdx.x]; }
    __syncthreads();
}

template <typename Px>
__global__ __launch_bounds__(256) void lf_cols_kernel(LfArgs a) {
    __shared__ uint8_t le[64], li[64];
    stage_lut(a, le, li);
    const int b = xcd_block(blockIdx.x, gridDim.x);
    const int p = b < a.blk_start[1] ? 0 : b < a.blk_start[2] ? 1 : 2;
    const int lb = b - a.blk_start[p];
    const int bx = (a.units_x[p] + 63) >> 6;
    const int ux = (lb % bx) * 64 + (threadIdx.x & 63);
    const int y = (lb / bx) * 4 + (threadIdx.x >> 6);
    if (ux >= a.units_x[p] || y >= a.rows[p] || ux == 0) return;
    const int uy = y >> 2;
    int wd, slot;
    if (p == 0) {
        const int X = ux >> 5, x = ux & 31, Y = uy >> 5, yy = uy & 31;
        const int half = yy >> 4;
        if (half && a.h4 - 32 * Y <= 16) return;
        const unsigned bit = 1u << (yy & 15);
        const uint16_t (*m)[2] = a.masks[Y * a.sb128w + X].filter_y[0][x];
        wd = (m[2][half] & bit) ? 16 : (m[1][half] & bit) ? 8 : (m[0][half] & bit) ? 4 : 0;
        slot = 0;
        if (ux >= a.w4) return;
    } else {
        if (!a.filter_uv) return;
        const int csw = 32 >> a.ss_hor, csh = 32 >> a.ss_ver, hb = 16 >> a.ss_ver;
        const int X = ux / csw, x = ux % csw, Y = uy / csh, yy = uy % csh;
        const int half = yy >= hb;
        if (half && a.h4 - 32 * Y <= 16) return;
        if (x >= ((min(32, a.w4 - X * 32) + a.ss_hor) >> a.ss_hor)) return;
        const unsigned bit = 1u << (yy - half * hb);
        const uint16_t (*m)[2] = a.masks[Y * a.sb128w + X].filter_uv[0][x];
        wd = (m[1][half] & bit) ? 6 : (m[0][half] & bit) ? 4 : 0;
        slot = 1 + p;
    }
    if (!wd) return;
    int L = lvl_at(a, uy, ux, slot);
    if (!L) L = lvl_at(a, uy, ux - 1, slot);
    if (!L) return;
    if (ux * 4 < (wd == 16 ? 7 : wd / 2)) return;   // malformed mask: never reached for valid AV1
    Px *q0 = reinterpret_cast<Px *>(a.plane[p] + (int64_t)y * a.stride[p]) + ux * 4;
    filter_line<Px>(q0, 1, wd, le[L], li[L], L >> 4, a.bdm8, a.bdmax);
}

// ---- row edges (filtering along columns) ----
template <typename Px>
__global__ __launch_bounds__(256) void lf_rows_kernel(LfArgs a) {
    __shared__ uint8_t le[64], li[64];
    stage_lut(a, le, li);
    const int b = xcd_block(blockIdx.x, gridDim.x);
    const int p = b < a.blk_start[1] ? 0 : b < a.blk_start[2] ? 1 : 2;
    const int lb = b - a.blk_start[p];
    const int bx = (a.units_x[p] + 63) >> 6;
    const int x = (lb % bx) * 64 + (threadIdx.x & 63);       // pixel column
    const int uy = (lb / bx) * 4 + (threadIdx.x >> 6);       // unit row
    if (x >= a.units_x[p] || uy >= a.rows[p] || uy == 0) return;
    const int ux = x >> 2;
    int wd, slot;
    if (p == 0) {
        if (uy >= a.h4) return;
        const int X = ux >> 5, xx = ux & 31, Y = uy >> 5, y = uy & 31;
        const int half = xx >> 4;
        const unsigned bit = 1u << (xx & 15);
        const uint16_t (*m)[2] = a.masks[Y * a.sb128w + X].filter_y[1][y];
        wd = (m[2][half] & bit) ? 16 : (m[1][half] & bit) ? 8 : (m[0][half] & bit) ? 4 : 0;
        slot = 1;
    } else {
        if (!a.filter_uv) return;
        const int csw = 32 >> a.ss_hor, csh = 32 >> a.ss_ver, hb = 16 >> a.ss_hor;
        const int X = ux / csw, xx = ux % csw, Y = uy / csh, y = uy % csh;
        if (y >= ((min(a.h4 - 32 * Y, 32) + a.ss_ver) >> a.ss_ver)) return;
        const int half = xx >= hb;
        const unsigned bit = 1u << (xx - half * hb);
        const uint16_t (*m)[2] = a.masks[Y * a.sb128w + X].filter_uv[1][y];
        wd = (m[1][half] & bit) ? 6 : (m[0][half] & bit) ? 4 : 0;
        slot = 1 + p;
    }
    if (!wd) return;
    int L = lvl_at(a, uy, ux, slot);
    if (!L) L = lvl_at(a, uy - 1, ux, slot);
    if (!L) return;
    if (uy * 4 < (wd == 16 ? 7 : wd / 2)) return;
    const int64_t ps = a.stride[p] / (int64_t)sizeof(Px);
    Px *q0 = reinterpret_cast<Px *>(a.plane[p] + (int64_t)uy * 4 * a.stride[p]) + x;
    filter_line<Px>(q0, ps, wd, le[L], li[L], L >> 4, a.bdm8, a.bdmax);
}

int launch_deblock(const LfArgs &cols, const LfArgs &rows, int bpc, hipStream_t s) {
    const int nc = cols.blk_start[3], nr = rows.blk_start[3];
    if (bpc == 8) {
        if (nc) hipLaunchKernelGGL(lf_cols_kernel<uint8_t>, dim3(nc), dim3(256), 0, s, cols);
        if (nr) hipLaunchKernelGGL(lf_rows_kernel<uint8_t>, dim3(nr), dim3(256), 0, s, rows);
    } else {
        if (nc) hipLaunchKernelGGL(lf_cols_kernel<uint16_t>, dim3(nc), dim3(256), 0, s, cols);
        if (nr) hipLaunchKernelGGL(lf_rows_kernel<uint16_t>, dim3(nr), dim3(256), 0, s, rows);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
