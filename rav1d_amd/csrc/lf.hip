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

MI_KTL_DEFINE(lf)

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

// ---- fused, out-of-place deblock: one workgroup per 64x64 plane tile ----
//
// The tile plus a halo (16 px left/right, 12 rows above, 12 below) is staged in LDS once with
// 16-B loads. All column edges whose footprint reaches the tile's columns are filtered over
// every staged row, then all row edges whose footprint reaches the tile's rows over the
// tile's columns, then the tile is stored with 16-B stores. This is "all column edges, then
// all row edges" restricted to the tile, so the result equals the
// two-pass kernels above. Out of place because a tile's halo must hold pre-filter pixels
// while the neighbouring tile writes its own.
//
// Halo sizes: a row edge at e reads rows e-7..e+6 and writes e-6..e+5, so the row edges that
// touch rows [y0, y0+64) are e in [y0-4, y0+68] (19 edges) and read rows [y0-11, y0+74]:
// those rows must be column-filtered first; column edges e in [x0-4, x0+68] (19) read
// columns [x0-11, x0+74].
constexpr int kLfRows = kLfTH + 24;       // staged rows: y0-12 .. y0+TH+11
constexpr int kLfCols = kLfTW + 32;       // staged columns: x0-16 .. x0+TW+15
constexpr int kLfEdgesV = kLfTW / 4 + 3;  // column edges reaching the tile
constexpr int kLfEdgesH = kLfTH / 4 + 3;  // row edges reaching the tile

// The inputs of one edge unit's code, fetched with independent loads (no load depends on
// another) so that a lane's units are all in flight at once.
struct LfEdgeRaw {
    uint16_t m[3];     // mask words for width index 0..2 (chroma: 0..1)
    uint32_t lv, lvp;  // level word of the unit and of its left (dir 0) / upper (dir 1) neighbour
    uint16_t bit;      // 0: the reference never filters this unit
    uint8_t slot, luma;
};

// Column (dir 0) or row (dir 1) edge at 4-px unit (ux, uy) of plane p: the per-lane logic of
// lf_cols/rows_kernel, split into fetch and decode.
__device__ __forceinline__ LfEdgeRaw lf_edge_fetch(const LfTileArgs &a, int p, int dir, int ux, int uy) {
    LfEdgeRaw r;
    r.bit = 0; r.luma = p == 0; r.slot = p == 0 ? dir : 1 + p;
    r.m[0] = r.m[1] = r.m[2] = 0; r.lv = r.lvp = 0;
    if (ux <= 0 && dir == 0) return r;
    if (uy <= 0 && dir == 1) return r;
    if (ux < 0 || uy < 0) return r;
    const uint16_t *m = nullptr;
    int half = 0;
    unsigned bit = 0;
    if (dir == 0) {
        if (ux >= KARG_OF(LfTileArgs, cols_ux, p) || uy * 4 >= KARG_OF(LfTileArgs, cols_rows, p)) return r;
        if (p == 0) {
            const int X = ux >> 5, x = ux & 31, Y = uy >> 5, yy = uy & 31;
            half = yy >> 4;
            if (half && a.h4 - 32 * Y <= 16) return r;
            bit = 1u << (yy & 15);
            m = &a.masks[Y * a.sb128w + X].filter_y[0][x][0][0];
        } else {
            // csw = 32 >> ss_hor units per SB column, csh = 32 >> ss_ver, half = 16 >> ss_ver
            const int lw = 5 - a.ss_hor, lh = 5 - a.ss_ver, hb = 16 >> a.ss_ver;
            const int X = ux >> lw, x = ux & ((1 << lw) - 1), Y = uy >> lh, yy = uy & ((1 << lh) - 1);
            half = yy >= hb;
            if (half && a.h4 - 32 * Y <= 16) return r;
            if (x >= ((min(32, a.w4 - X * 32) + a.ss_hor) >> a.ss_hor)) return r;
            bit = 1u << (yy - half * hb);
            m = &a.masks[Y * a.sb128w + X].filter_uv[0][x][0][0];
        }
    } else {
        if (ux * 4 >= KARG_OF(LfTileArgs, rows_px, p) || uy >= KARG_OF(LfTileArgs, rows_uy, p)) return r;
        if (p == 0) {
            const int X = ux >> 5, xx = ux & 31, Y = uy >> 5, y = uy & 31;
            half = xx >> 4;
            bit = 1u << (xx & 15);
            m = &a.masks[Y * a.sb128w + X].filter_y[1][y][0][0];
        } else {
            const int lw = 5 - a.ss_hor, lh = 5 - a.ss_ver, hb = 16 >> a.ss_hor;
            const int X = ux >> lw, xx = ux & ((1 << lw) - 1), Y = uy >> lh, y = uy & ((1 << lh) - 1);
            if (y >= ((min(a.h4 - 32 * Y, 32) + a.ss_ver) >> a.ss_ver)) return r;
            half = xx >= hb;
            bit = 1u << (xx - half * hb);
            m = &a.masks[Y * a.sb128w + X].filter_uv[1][y][0][0];
        }
    }
    r.bit = (uint16_t)bit;
    r.m[0] = m[half];
    r.m[1] = m[2 + half];
    if (p == 0) r.m[2] = m[4 + half];
    const uint32_t *lv = a.level + (int64_t)uy * a.b4_stride + ux;
    r.lv = lv[0];
    r.lvp = lv[dir ? -a.b4_stride : -1];
    return r;
}

// (wd << 8) | L, or 0 when the unit is not filtered
__device__ __forceinline__ int lf_edge_decode(const LfEdgeRaw &r, int dir, int ux, int uy) {
    if (!r.bit) return 0;
    const int wd = r.luma ? ((r.m[2] & r.bit) ? 16 : (r.m[1] & r.bit) ? 8 : (r.m[0] & r.bit) ? 4 : 0)
                          : ((r.m[1] & r.bit) ? 6 : (r.m[0] & r.bit) ? 4 : 0);
    if (!wd) return 0;
    int L = (r.lv >> (8 * r.slot)) & 0xff;
    if (!L) L = (r.lvp >> (8 * r.slot)) & 0xff;
    if (!L) return 0;
    if ((dir ? uy : ux) * 4 < (wd == 16 ? 7 : wd / 2)) return 0;
    return (wd << 8) | L;
}

// The filter of one pixel line on registers: v[8] = q0, v[7] = p0, v[1] = p6, v[14] = q6
// (loopfilter.rs:396-721), for a compile-time width. Returns false when the line is unchanged.
template <int wd>
__device__ __forceinline__ bool filter_regs(int (&v)[16], int E, int I, int H, int bdm8, int bdmax) {
    const int F = 1 << bdm8;
    E <<= bdm8; I <<= bdm8; H <<= bdm8;
    const int p1 = v[6], p0 = v[7], q0 = v[8], q1 = v[9];
    bool fm = abs(p1 - p0) <= I && abs(q1 - q0) <= I && abs(p0 - q0) * 2 + (abs(p1 - q1) >> 1) <= E;
    const int p2 = v[5], q2 = v[10], p3 = v[4], q3 = v[11];
    if constexpr (wd > 4) fm = fm && abs(p2 - p1) <= I && abs(q2 - q1) <= I;
    if constexpr (wd > 6) fm = fm && abs(p3 - p2) <= I && abs(q3 - q2) <= I;
    if (!fm) return false;
    bool flat_in = false;
    if constexpr (wd >= 6) flat_in = abs(p2 - p0) <= F && abs(p1 - p0) <= F && abs(q1 - q0) <= F && abs(q2 - q0) <= F;
    if constexpr (wd >= 8) flat_in = flat_in && abs(p3 - p0) <= F && abs(q3 - q0) <= F;
    if constexpr (wd == 16) if (flat_in) {
        const bool flat_out = abs(v[1] - p0) <= F && abs(v[2] - p0) <= F && abs(v[3] - p0) <= F &&
                              abs(v[12] - q0) <= F && abs(v[13] - q0) <= F && abs(v[14] - q0) <= F;
        if (flat_out) {
            // 13-tap smoother: the output at v[j] (j = 2..13) is S_j >> 4 with
            // S_j = sum_{t=-6..6} v[clamp(j+t, 1, 14)] + v[j-1] + v[j] + v[j+1]; S_{j+1} - S_j =
            // v[clamp(j+7)] - v[clamp(j-6)] + v[j+2] - v[j-1], so one running sum serves all 12
            int o[12];
            int s = 8 + 6 * v[1] + v[2] + v[3] + v[4] + v[5] + v[6] + v[7] + v[8] + v[1] + v[2] + v[3];
#pragma unroll
            for (int k = 0; k < 12; k++) {
                const int j = k + 2;
                o[k] = s >> 4;
                if (k < 11) {
                    const int hi = j + 7 > 14 ? 14 : j + 7, lo = j - 6 < 1 ? 1 : j - 6;
                    s += v[hi] - v[lo] + v[j + 2] - v[j - 1];
                }
            }
#pragma unroll
            for (int k = 0; k < 12; k++) v[2 + k] = o[k];
            return true;
        }
    }
    if (wd >= 8 && flat_in) {
        v[5] = (3 * p3 + 2 * p2 + p1 + p0 + q0 + 4) >> 3;
        v[6] = (2 * p3 + p2 + 2 * p1 + p0 + q0 + q1 + 4) >> 3;
        v[7] = (p3 + p2 + p1 + 2 * p0 + q0 + q1 + q2 + 4) >> 3;
        v[8] = (p2 + p1 + p0 + 2 * q0 + q1 + q2 + q3 + 4) >> 3;
        v[9] = (p1 + p0 + q0 + 2 * q1 + q2 + 2 * q3 + 4) >> 3;
        v[10] = (p0 + q0 + q1 + 2 * q2 + 3 * q3 + 4) >> 3;
    } else if (wd == 6 && flat_in) {
        v[6] = (3 * p2 + 2 * p1 + 2 * p0 + q0 + 4) >> 3;
        v[7] = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3;
        v[8] = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3;
        v[9] = (p0 + 2 * q0 + 2 * q1 + 3 * q2 + 4) >> 3;
    } else {
        const int dlo = -(128 << bdm8), dhi = (128 << bdm8) - 1;
        const bool hev = abs(p1 - p0) > H || abs(q1 - q0) > H;
        int f = hev ? min(max(p1 - q1, dlo), dhi) : 0;
        f = min(max(3 * (q0 - p0) + f, dlo), dhi);
        const int f1 = min(f + 4, dhi) >> 3;
        const int f2 = min(f + 3, dhi) >> 3;
        v[7] = min(max(p0 + f2, 0), bdmax);
        v[8] = min(max(q0 - f1, 0), bdmax);
        if (!hev) {
            const int g = (f1 + 1) >> 1;
            v[6] = min(max(p1 + g, 0), bdmax);
            v[9] = min(max(q1 - g, 0), bdmax);
        }
    }
    return true;
}

// ---- two pixel lines per lane in packed 16-bit arithmetic ----
//
// The two lines of a lane belong to one edge unit, so they share the filter width and level.
// Every value of the filter fits 16 bits (12-bit pixels: differences within +-4095, the 8-tap
// sums within 8 * 4095 + 4; the 16-weight sums of the 13-tap smoother within 65528, so they are
// shifted as unsigned), and the branches of loopfilter.rs:396-721 become per-half masks
// (0xffff where a condition holds, from the sign of a difference) merged with v_bfi_b32.
// This halves the VALU issue of the filter, which bounds the tile kernel.
typedef short lf_s2 __attribute__((ext_vector_type(2)));
typedef unsigned short lf_u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ lf_s2 pk_splat(int x) { return lf_s2{(short)x, (short)x}; }
__device__ __forceinline__ lf_s2 pk_absd(lf_s2 a, lf_s2 b) {
    const lf_s2 d = a - b;
    return __builtin_elementwise_max(d, -d);
}
__device__ __forceinline__ lf_s2 pk_max(lf_s2 a, lf_s2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ lf_s2 pk_min(lf_s2 a, lf_s2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ lf_s2 pk_clamp(lf_s2 a, lf_s2 lo, lf_s2 hi) { return pk_min(pk_max(a, lo), hi); }
// per half: m ? a : b, for m in {0, 0xffff}
__device__ __forceinline__ lf_s2 pk_sel(lf_s2 m, lf_s2 a, lf_s2 b) {
    const uint32_t mu = __builtin_bit_cast(uint32_t, m);
    return __builtin_bit_cast(lf_s2, (mu & __builtin_bit_cast(uint32_t, a)) | (~mu & __builtin_bit_cast(uint32_t, b)));
}
__device__ __forceinline__ uint32_t pk_bits(lf_s2 m) { return __builtin_bit_cast(uint32_t, m); }
// sum >> 4 of a non-negative 16-bit sum (up to 65535)
__device__ __forceinline__ lf_s2 pk_shr4u(lf_s2 s) { return __builtin_bit_cast(lf_s2, __builtin_bit_cast(lf_u2, s) >> (unsigned short)4); }

// v[8] = q0, v[7] = p0 (as filter_regs), two lines per element. Lines whose filter mask is
// clear are returned unchanged.
template <int WD>
__device__ __forceinline__ void filter_pk(lf_s2 (&v)[16], int E, int I, int H, int bdm8, int bdmax) {
    const lf_s2 F = pk_splat(1 << bdm8), zero = pk_splat(0), bmax = pk_splat(bdmax);
    const lf_s2 Es = pk_splat(E << bdm8), Is = pk_splat(I << bdm8), Hs = pk_splat(H << bdm8);
    const lf_s2 p3 = v[4], p2 = v[5], p1 = v[6], p0 = v[7], q0 = v[8], q1 = v[9], q2 = v[10], q3 = v[11];
    const lf_s2 a10 = pk_max(pk_absd(p1, p0), pk_absd(q1, q0));
    // fm <=> every limit minus its distance is >= 0: sign of the minimum
    lf_s2 t = pk_min(Is - a10, Es - (pk_absd(p0, q0) * (short)2 + (pk_absd(p1, q1) >> (short)1)));
    if constexpr (WD > 4) t = pk_min(t, Is - pk_max(pk_absd(p2, p1), pk_absd(q2, q1)));
    if constexpr (WD > 6) t = pk_min(t, Is - pk_max(pk_absd(p3, p2), pk_absd(q3, q2)));
    const lf_s2 fm = ~(t >> (short)15);                  // 0xffff: the line is filtered
    if (!pk_bits(fm)) return;
    lf_s2 narrow = fm;                                   // lines taking the 4-tap filter
    lf_s2 flat = zero;
    if constexpr (WD >= 6) {
        lf_s2 d = pk_max(pk_max(pk_absd(p2, p0), pk_absd(q2, q0)), a10);
        if constexpr (WD >= 8) d = pk_max(d, pk_max(pk_absd(p3, p0), pk_absd(q3, q0)));
        flat = fm & ~((F - d) >> (short)15);             // fm && flat_in
        narrow = fm & ~flat;
    }
    if (pk_bits(narrow)) {
        const lf_s2 dlo = pk_splat(-(128 << bdm8)), dhi = pk_splat((128 << bdm8) - 1);
        const lf_s2 hev = (Hs - a10) >> (short)15;       // 0xffff: |p1-p0| or |q1-q0| > H
        lf_s2 f = pk_clamp(p1 - q1, dlo, dhi) & hev;
        f = pk_clamp((q0 - p0) * (short)3 + f, dlo, dhi);
        const lf_s2 f1 = pk_min(f + (short)4, dhi) >> (short)3;
        const lf_s2 f2 = pk_min(f + (short)3, dhi) >> (short)3;
        const lf_s2 g = (f1 + (short)1) >> (short)1;
        v[7] = pk_sel(narrow, pk_clamp(p0 + f2, zero, bmax), v[7]);
        v[8] = pk_sel(narrow, pk_clamp(q0 - f1, zero, bmax), v[8]);
        const lf_s2 nh = narrow & ~hev;
        v[6] = pk_sel(nh, pk_clamp(p1 + g, zero, bmax), v[6]);
        v[9] = pk_sel(nh, pk_clamp(q1 - g, zero, bmax), v[9]);
    }
    if constexpr (WD == 6) {
        if (pk_bits(flat)) {
            const lf_s2 c4 = pk_splat(4);
            v[6] = pk_sel(flat, (p2 * (short)3 + p1 * (short)2 + p0 * (short)2 + q0 + c4) >> (short)3, v[6]);
            v[7] = pk_sel(flat, (p2 + p1 * (short)2 + p0 * (short)2 + q0 * (short)2 + q1 + c4) >> (short)3, v[7]);
            v[8] = pk_sel(flat, (p1 + p0 * (short)2 + q0 * (short)2 + q1 * (short)2 + q2 + c4) >> (short)3, v[8]);
            v[9] = pk_sel(flat, (p0 + q0 * (short)2 + q1 * (short)2 + q2 * (short)3 + c4) >> (short)3, v[9]);
        }
    }
    if constexpr (WD >= 8) {
        lf_s2 flat8 = flat;
        if constexpr (WD == 16) {
            if (pk_bits(flat)) {
                const lf_s2 d = pk_max(pk_max(pk_max(pk_absd(v[1], p0), pk_absd(v[2], p0)), pk_max(pk_absd(v[3], p0), pk_absd(v[12], q0))),
                                       pk_max(pk_absd(v[13], q0), pk_absd(v[14], q0)));
                const lf_s2 flat16 = flat & ~((F - d) >> (short)15);
                flat8 = flat & ~flat16;
                if (pk_bits(flat16)) {
                    // the running 16-weight sum of filter_regs, as unsigned 16-bit
                    lf_s2 o[12];
                    lf_s2 s = pk_splat(8) + v[1] * (short)7 + v[2] * (short)2 + v[3] * (short)2 + v[4] + v[5] + v[6] + v[7] + v[8];
#pragma unroll
                    for (int k = 0; k < 12; k++) {
                        const int j = k + 2;
                        o[k] = pk_shr4u(s);
                        if (k < 11) {
                            const int hi = j + 7 > 14 ? 14 : j + 7, lo = j - 6 < 1 ? 1 : j - 6;
                            s += v[hi] - v[lo] + v[j + 2] - v[j - 1];
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 12; k++) v[2 + k] = pk_sel(flat16, o[k], v[2 + k]);
                }
            }
        }
        if (pk_bits(flat8)) {
            const lf_s2 c4 = pk_splat(4);
            const lf_s2 n5 = (p3 * (short)3 + p2 * (short)2 + p1 + p0 + q0 + c4) >> (short)3;
            const lf_s2 n6 = (p3 * (short)2 + p2 + p1 * (short)2 + p0 + q0 + q1 + c4) >> (short)3;
            const lf_s2 n7 = (p3 + p2 + p1 + p0 * (short)2 + q0 + q1 + q2 + c4) >> (short)3;
            const lf_s2 n8 = (p2 + p1 + p0 + q0 * (short)2 + q1 + q2 + q3 + c4) >> (short)3;
            const lf_s2 n9 = (p1 + p0 + q0 + q1 * (short)2 + q2 + q3 * (short)2 + c4) >> (short)3;
            const lf_s2 n10 = (p0 + q0 + q1 + q2 * (short)2 + q3 * (short)3 + c4) >> (short)3;
            v[5] = pk_sel(flat8, n5, v[5]);
            v[6] = pk_sel(flat8, n6, v[6]);
            v[7] = pk_sel(flat8, n7, v[7]);
            v[8] = pk_sel(flat8, n8, v[8]);
            v[9] = pk_sel(flat8, n9, v[9]);
            v[10] = pk_sel(flat8, n10, v[10]);
        }
    }
}

// Pixel pairs <-> packed lanes. Column edges: a lane holds rows r and r + 1 of one edge unit
// (low half = row r), gathered from the two rows' 4-pixel quads with v_perm_b32.
template <typename Px>
__device__ __forceinline__ void pk_load_quad(const Px *w0, const Px *w1, int q, lf_s2 *o) {
    if constexpr (sizeof(Px) == 2) {
        const uint2 d = reinterpret_cast<const uint2 *>(w0)[q], e = reinterpret_cast<const uint2 *>(w1)[q];
        o[0] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(e.x, d.x, 0x05040100u));
        o[1] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(e.x, d.x, 0x07060302u));
        o[2] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(e.y, d.y, 0x05040100u));
        o[3] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(e.y, d.y, 0x07060302u));
    } else {
        const uint32_t d = reinterpret_cast<const uint32_t *>(w0)[q], e = reinterpret_cast<const uint32_t *>(w1)[q];
        o[0] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(e, d, 0x0c040c00u));
        o[1] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(e, d, 0x0c050c01u));
        o[2] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(e, d, 0x0c060c02u));
        o[3] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(e, d, 0x0c070c03u));
    }
}
// rows r / r + 1 of the pixel pair (v[k], v[k + 1]) as one dword (u16) or halfword (u8) each
__device__ __forceinline__ uint32_t pk_row_lo(lf_s2 a, lf_s2 b) {
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x05040100u);
}
__device__ __forceinline__ uint32_t pk_row_hi(lf_s2 a, lf_s2 b) {
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x07060302u);
}
__device__ __forceinline__ uint16_t pk_row_lo8(lf_s2 a, lf_s2 b) {
    return (uint16_t)__builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x0c0c0400u);
}
__device__ __forceinline__ uint16_t pk_row_hi8(lf_s2 a, lf_s2 b) {
    return (uint16_t)__builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x0c0c0602u);
}

template <int WD, typename Px, int P>
__device__ __forceinline__ void lf_col_pair(Px *t, int e, int i, const uint8_t *le,
                                            const uint8_t *li, int bdm8, int bdmax) {
    {
        const int u = e >> 6, L = e & 63;
        const int r = (u / kLfEdgesV) * 4 + 2 * (i & 1), k = u % kLfEdgesV;
        Px *w0 = &t[r * P + 4 + 4 * k], *w1 = w0 + P;
        constexpr int q0 = WD == 16 ? 0 : 1, q1 = WD == 16 ? 4 : 3;   // quads loaded
        lf_s2 v[16];
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = pk_splat(0);
#pragma unroll
        for (int q = q0; q < q1; q++) pk_load_quad<Px>(w0, w1, q, &v[4 * q]);
        filter_pk<WD>(v, le[L], li[L], L >> 4, bdm8, bdmax);
        if constexpr (WD >= 8) {
#pragma unroll
            for (int q = q0; q < q1; q++) {
                if constexpr (sizeof(Px) == 2) {
                    reinterpret_cast<uint2 *>(w0)[q] = make_uint2(pk_row_lo(v[4 * q], v[4 * q + 1]), pk_row_lo(v[4 * q + 2], v[4 * q + 3]));
                    reinterpret_cast<uint2 *>(w1)[q] = make_uint2(pk_row_hi(v[4 * q], v[4 * q + 1]), pk_row_hi(v[4 * q + 2], v[4 * q + 3]));
                } else {
                    reinterpret_cast<uint32_t *>(w0)[q] = pk_row_lo8(v[4 * q], v[4 * q + 1]) | ((uint32_t)pk_row_lo8(v[4 * q + 2], v[4 * q + 3]) << 16);
                    reinterpret_cast<uint32_t *>(w1)[q] = pk_row_hi8(v[4 * q], v[4 * q + 1]) | ((uint32_t)pk_row_hi8(v[4 * q + 2], v[4 * q + 3]) << 16);
                }
            }
        } else {
            if constexpr (sizeof(Px) == 2) {
                reinterpret_cast<uint32_t *>(w0)[3] = pk_row_lo(v[6], v[7]);
                reinterpret_cast<uint32_t *>(w0)[4] = pk_row_lo(v[8], v[9]);
                reinterpret_cast<uint32_t *>(w1)[3] = pk_row_hi(v[6], v[7]);
                reinterpret_cast<uint32_t *>(w1)[4] = pk_row_hi(v[8], v[9]);
            } else {
                reinterpret_cast<uint16_t *>(w0)[3] = pk_row_lo8(v[6], v[7]);
                reinterpret_cast<uint16_t *>(w0)[4] = pk_row_lo8(v[8], v[9]);
                reinterpret_cast<uint16_t *>(w1)[3] = pk_row_hi8(v[6], v[7]);
                reinterpret_cast<uint16_t *>(w1)[4] = pk_row_hi8(v[8], v[9]);
            }
        }
    }
}

// Row edges: a lane holds two adjacent pixel columns (one LDS dword per row for u16).
template <int WD, typename Px, int P>
__device__ __forceinline__ void lf_row_pair(Px *t, int e, int i, const uint8_t *le,
                                            const uint8_t *li, int bdm8, int bdmax) {
    constexpr int nr = WD == 16 ? 7 : WD == 8 ? 4 : WD == 6 ? 3 : 2;   // rows read each side
    constexpr int lo = WD == 16 ? 2 : WD == 8 ? 5 : 6;                 // rows [lo, 16 - lo) written
    {
        const int u = e >> 6, L = e & 63;
        const int k = u / (kLfTW / 4), col = (u % (kLfTW / 4)) * 4 + 2 * (i & 1);
        Px *w = &t[(4 * k) * P + 16 + col];
        lf_s2 v[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            v[j] = pk_splat(0);
            if (j >= 8 - nr && j < 8 + nr) {
                if constexpr (sizeof(Px) == 2)
                    v[j] = __builtin_bit_cast(lf_s2, *reinterpret_cast<const uint32_t *>(w + j * P));
                else
                    v[j] = __builtin_bit_cast(lf_s2, __builtin_amdgcn_perm(0u, (uint32_t)*reinterpret_cast<const uint16_t *>(w + j * P), 0x0c010c00u));
            }
        }
        filter_pk<WD>(v, le[L], li[L], L >> 4, bdm8, bdmax);
#pragma unroll
        for (int j = lo; j < 16 - lo; j++) {
            if constexpr (sizeof(Px) == 2)
                *reinterpret_cast<uint32_t *>(w + j * P) = __builtin_bit_cast(uint32_t, v[j]);
            else
                *reinterpret_cast<uint16_t *>(w + j * P) = (uint16_t)__builtin_amdgcn_perm(0u, __builtin_bit_cast(uint32_t, v[j]), 0x0c0c0200u);
        }
    }
}

// The four width classes of one direction as one sequence of 64-pair chunks, dealt to the
// workgroup's waves in turn: every chunk runs one filter branch (wave-uniform class), and a
// class leaves at most one partial wave instead of one partial 256-lane pass. Work lists: two
// arrays of N entries per direction, classes 0 / 2 filled upwards from the front and 1 / 3
// downwards from the back (a class pair never holds more than N units), half the LDS of four
// N-entry lists: 4 workgroups per CU instead of 3.
template <bool COLS, typename Px, int P>
__device__ __forceinline__ void lf_dir_pk(Px *t, const uint16_t (*lists)[COLS ? (kLfRows / 4) * kLfEdgesV : kLfEdgesH * (kLfTW / 4)],
                                          const int *cnt, const uint8_t *le, const uint8_t *li, int bdm8, int bdmax) {
    constexpr int N = COLS ? (kLfRows / 4) * kLfEdgesV : kLfEdgesH * (kLfTW / 4);
    const int tid = (int)threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    // chunk prefix over the classes (wave-uniform: the counts are LDS broadcasts)
    const int c0 = (cnt[0] * 2 + 63) >> 6, c1 = c0 + ((cnt[1] * 2 + 63) >> 6);
    const int c2 = c1 + ((cnt[2] * 2 + 63) >> 6), c3 = c2 + ((cnt[3] * 2 + 63) >> 6);
    // (lanes 2u / 2u + 1 take unit u; mapping lanes 0-31 and 32-63 to the two row pairs of the
    // same 32 units measured the same: 29.0-29.3 vs 29.0-30.1 us, round 5)
    for (int g = wave; g < c3; g += kLfThreads / 64) {
        const int cls = g < c0 ? 0 : g < c1 ? 1 : g < c2 ? 2 : 3;
        const int base = cls == 0 ? 0 : cls == 1 ? c0 : cls == 2 ? c1 : c2;
        const int ui = ((g - base) * 64 + lane) >> 1;
        const int i = lane;   // (the callees read i & 1)
        if (ui >= cnt[cls]) continue;
        const int e = lists[cls >> 1][cls & 1 ? N - 1 - ui : ui];
        switch (cls) {
#define LF_CASE(k, wd)                                                                     \
        case k:                                                                            \
            if constexpr (COLS) lf_col_pair<wd, Px, P>(t, e, i, le, li, bdm8, bdmax);     \
            else lf_row_pair<wd, Px, P>(t, e, i, le, li, bdm8, bdmax);                    \
            break;
        LF_CASE(0, 4) LF_CASE(1, 6) LF_CASE(2, 8) LF_CASE(3, 16)
#undef LF_CASE
        }
    }
}


// wd -> work class (lines of one class run the same filter branch)
__device__ __forceinline__ int lf_class(int wd) { return wd == 4 ? 0 : wd == 6 ? 1 : wd == 8 ? 2 : 3; }

// Staging shapes of one tile
template <typename Px>
struct LfShape {
    static constexpr int VPX = 16 / sizeof(Px);                 // pixels per 16-B vector
    // LDS pitch in pixels: the staged kLfCols (+8 px of padding cut the LDS bank conflicts
    // 3.15 -> 2.2 M cycles but ran 31 vs 29 us)
    static constexpr int P = kLfCols;
    static constexpr int NV = (kLfRows / 4) * kLfEdgesV;        // column-edge units (4 lines each)
    static constexpr int NH = kLfEdgesH * (kLfTW / 4);          // row-edge units
    static constexpr int VPR = kLfCols / VPX;                   // vectors per staged row
    static constexpr int NS = (kLfRows * VPR + kLfThreads - 1) / kLfThreads;
    static constexpr int NU = (NV + NH + kLfThreads - 1) / kLfThreads;
    static constexpr int VPT = kLfTW / VPX;                     // vectors per tile row
    static_assert(P % 8 == 0 && P >= kLfCols, "16-B aligned rows");
    static_assert((NV > NH ? NV : NH) << 6 <= 65536, "work-list entries (unit << 6 | level) must fit 16 bits");
};

// Tile b of the launch: its plane and origin. The plane's fields are read by kernarg offset
// (KARG_OF): selecting among the three copies kept every per-plane field in SGPRs.
struct LfTile {
    int p, x0, y0, pw, ph;
    int64_t st;
};
__device__ __forceinline__ LfTile lf_tile_at(const LfTileArgs &a, int b) {
    LfTile g;
    g.p = b < a.tile_start[1] ? 0 : b < a.tile_start[2] ? 1 : 2;
    const int lb = b - KARG_OF(LfTileArgs, tile_start, g.p);
    const int tx = KARG_OF(LfTileArgs, tiles_x, g.p);
    g.x0 = (lb % tx) * kLfTW; g.y0 = (lb / tx) * kLfTH;
    g.pw = KARG_OF(LfTileArgs, pw, g.p); g.ph = KARG_OF(LfTileArgs, ph, g.p);
    g.st = KARG_OF(LfTileArgs, stride, g.p);
    return g;
}

// Issue every load of tile g: rows y0-12 .. y0+TH+11, columns x0-16 .. x0+TW+15 (pixels
// outside the plane read as 0: no edge reaches them), and every edge unit's mask and level
// words. All of them are independent; none is waited for here.
template <typename Px>
__device__ __forceinline__ void lf_fetch_pixels(const LfTileArgs &a, const LfTile &g, uint4 (&sv)[LfShape<Px>::NS]) {
    using S = LfShape<Px>;
    const int tid = (int)threadIdx.x;
    const uint8_t *src = KARG_OF(LfTileArgs, src, g.p);
#pragma unroll
    for (int j = 0; j < S::NS; j++) {
        const int i = tid + kLfThreads * j;
        const int r = i / S::VPR, c = (i % S::VPR) * S::VPX;
        const int y = g.y0 - 12 + r, x = g.x0 - 16 + c;
        sv[j] = make_uint4(0, 0, 0, 0);
        if (i < kLfRows * S::VPR && y >= 0 && y < g.ph && x >= 0 && x < g.pw)
            sv[j] = *reinterpret_cast<const uint4 *>(src + (int64_t)y * g.st + (int64_t)x * sizeof(Px));
    }
}
template <typename Px>
__device__ __forceinline__ void lf_fetch_edges(const LfTileArgs &a, const LfTile &g, LfEdgeRaw (&raw)[LfShape<Px>::NU]) {
    using S = LfShape<Px>;
    const int tid = (int)threadIdx.x;
    // Edge units. The outermost edge of each direction (k = 0, 18) reaches the tile only
    // with the 16-wide filter (it writes e-6 .. e+5); narrower ones are skipped there.
    const int ux0 = (g.x0 >> 2) - 1, uy0 = (g.y0 >> 2) - 3;   // unit of the first edge / staged row
#pragma unroll
    for (int j = 0; j < S::NU; j++) {
        const int i = tid + kLfThreads * j;
        const bool v = i < S::NV;
        const int u = v ? i : i - S::NV;
        raw[j].bit = 0;
        if (i < S::NV + S::NH)
            raw[j] = v ? lf_edge_fetch(a, g.p, 0, ux0 + u % kLfEdgesV, uy0 + u / kLfEdgesV)
                       : lf_edge_fetch(a, g.p, 1, (g.x0 >> 2) + u % (kLfTW / 4), (g.y0 >> 2) - 1 + u / (kLfTW / 4));
    }
}


template <typename Px>
__device__ __forceinline__ void lf_fetch(const LfTileArgs &a, const LfTile &g, uint4 (&sv)[LfShape<Px>::NS],
                                         LfEdgeRaw (&raw)[LfShape<Px>::NU]) {
    lf_fetch_pixels<Px>(a, g, sv);
    lf_fetch_edges<Px>(a, g, raw);
}

template <typename Px>
__device__ __forceinline__ void lf_commit_pixels(Px *t, const uint4 (&sv)[LfShape<Px>::NS]) {
    using S = LfShape<Px>;
    const int tid = (int)threadIdx.x;
#pragma unroll
    for (int j = 0; j < S::NS; j++) {
        const int i = tid + kLfThreads * j;
        if (i < kLfRows * S::VPR) *reinterpret_cast<uint4 *>(&t[(i / S::VPR) * S::P + (i % S::VPR) * S::VPX]) = sv[j];
    }
}

// ---- deferred DC runs (mi_deblock_frame_dc) ----
// mi_itx_frame_runs(MI_ITX_DC_DEFER) leaves the DC-only blocks' constant out of the pixels and
// records it per 4x4 unit (tagged with the call's 16-bit tag); the tile adds it while staging,
// so the deblocked picture is the one of the undeferred residual and the DC-only blocks cost
// no pass of their own over the picture. kLfDcW x kLfDcH units cover the staged image.
constexpr int kLfDcW = kLfCols / 4, kLfDcH = kLfRows / 4;
static_assert(kLfDcW % 2 == 0 && (kLfDcW * kLfDcH) / 2 <= kLfThreads, "two map entries per lane");

// each lane's two map entries (units 2 tid, 2 tid + 1 of the staged image): one 8-B load
__device__ __forceinline__ uint2 lf_dc_fetch(const LfTileArgs &a, const LfTile &g) {
    const int e = 2 * (int)threadIdx.x;
    uint2 v = make_uint2(0, 0);
    if (e < kLfDcW * kLfDcH) {
        const int uy = (g.y0 >> 2) - 3 + e / kLfDcW, ux = (g.x0 >> 2) - 4 + e % kLfDcW;
        const int st = KARG_OF(LfTileArgs, dc_stride, g.p);
        if (uy >= 0 && uy < (g.ph >> 2) && ux >= 0 && ux + 1 < st)
            v = *reinterpret_cast<const uint2 *>(a.dc_map + KARG_OF(LfTileArgs, dc_off, g.p) + (int64_t)uy * st + ux);
    }
    return v;
}
// the entries' DC (0 for another call's tag) into the tile's LDS table
__device__ __forceinline__ void lf_dc_commit(const LfTileArgs &a, uint2 v, int *dcs) {
    const int e = 2 * (int)threadIdx.x;
    if (e < kLfDcW * kLfDcH) {
        dcs[e] = (v.x >> 16) == a.dc_tag ? (int)(int16_t)(v.x & 0xffff) : 0;
        dcs[e + 1] = (v.y >> 16) == a.dc_tag ? (int)(int16_t)(v.y & 0xffff) : 0;
    }
}
// the staged vectors plus their units' DC, clipped to [0, bdmax], into LDS
template <typename Px>
__device__ __forceinline__ void lf_commit_pixels_dc(Px *t, const uint4 (&sv)[LfShape<Px>::NS], const int *dcs, int bdmax) {
    using S = LfShape<Px>;
    const int tid = (int)threadIdx.x;
#pragma unroll
    for (int j = 0; j < S::NS; j++) {
        const int i = tid + kLfThreads * j;
        if (i < kLfRows * S::VPR) {
            const int r = i / S::VPR, c = (i % S::VPR) * S::VPX;
            const int *d = dcs + (r >> 2) * kLfDcW + (c >> 2);
            uint32_t w[4] = { sv[j].x, sv[j].y, sv[j].z, sv[j].w };
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if constexpr (sizeof(Px) == 2) {
                    // pixels 2k, 2k + 1 (one unit: (2k) / 4) in packed 16-bit arithmetic: a pixel
                    // (< 4096) plus a DC (|dc| < 2^15 - 4096 for 12-bit coefficients) fits int16
                    const lf_s2 v = __builtin_bit_cast(lf_s2, w[k]) + pk_splat(d[k >> 1]);
                    w[k] = __builtin_bit_cast(uint32_t, pk_clamp(v, pk_splat(0), pk_splat(bdmax)));
                } else {
                    const int dc = d[k];        // pixels 4k .. 4k + 3: unit k
                    uint32_t o = 0;
#pragma unroll
                    for (int b = 0; b < 4; b++) o |= (uint32_t)min(max((int)((w[k] >> (8 * b)) & 0xff) + dc, 0), bdmax) << (8 * b);
                    w[k] = o;
                }
            }
            *reinterpret_cast<uint4 *>(&t[r * S::P + c]) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

// Decode the edge units and bucket the filtered ones by width class (cnt[] zeroed and visible)
template <typename Px>
__device__ __forceinline__ void lf_build_lists(const LfTile &g, const LfEdgeRaw (&raw)[LfShape<Px>::NU],
                                               uint16_t (*listv)[LfShape<Px>::NV], uint16_t (*listh)[LfShape<Px>::NH], int *cnt) {
    using S = LfShape<Px>;
    const int tid = (int)threadIdx.x;
    const int ux0 = (g.x0 >> 2) - 1;
#pragma unroll
    for (int j = 0; j < S::NU; j++) {
        const int i = tid + kLfThreads * j;
        const bool v = i < S::NV;
        const int u = v ? i : i - S::NV;
        const int k = v ? u % kLfEdgesV : u / (kLfTW / 4);
        const int code = v ? lf_edge_decode(raw[j], 0, ux0 + k, 0)
                           : lf_edge_decode(raw[j], 1, 0, (g.y0 >> 2) - 1 + k);
        const int wd = code >> 8;
        if (!wd || ((k == 0 || k == (v ? kLfEdgesV : kLfEdgesH) - 1) && wd != 16)) continue;
        const int c = lf_class(wd);
        const int slot = atomicAdd(&cnt[(v ? 0 : 4) + c], 1);
        const int N = v ? S::NV : S::NH;
        (v ? listv[c >> 1] : listh[c >> 1])[c & 1 ? N - 1 - slot : slot] = (uint16_t)((u << 6) | (code & 63));
    }
}

template <typename Px>
__device__ __forceinline__ void lf_store_tile(const LfTile &g, const Px *t) {
    using S = LfShape<Px>;
    const int tid = (int)threadIdx.x;
    uint8_t *dst = KARG_OF(LfTileArgs, dst, g.p);
#pragma unroll
    for (int j = 0; j < (kLfTH * S::VPT + kLfThreads - 1) / kLfThreads; j++) {
        const int i = tid + kLfThreads * j;
        if ((kLfTH * S::VPT) % kLfThreads && i >= kLfTH * S::VPT) break;
        const int r = i / S::VPT, c = (i % S::VPT) * S::VPX;
        const int y = g.y0 + r, x = g.x0 + c;
        if (y < g.ph && x < g.pw)
            *reinterpret_cast<uint4 *>(dst + (int64_t)y * g.st + (int64_t)x * sizeof(Px)) =
                *reinterpret_cast<const uint4 *>(&t[(12 + r) * S::P + 16 + c]);
    }
}

template <typename Px>
__global__ __launch_bounds__(kLfThreads) void lf_tile_kernel(LfTileArgs a) {
    using S = LfShape<Px>;
    __shared__ __attribute__((aligned(16))) Px t[kLfRows * S::P];
    // work lists: active edge units bucketed by width class, so that the lanes of a wave run
    // one filter branch; entry = (unit index << 6) | L
    __shared__ uint16_t listv[2][S::NV], listh[2][S::NH];
    __shared__ int cnt[8];
    __shared__ uint8_t le[64], li[64];
    __shared__ int dcs[kLfDcW * kLfDcH];   // deferred DC per staged 4x4 unit (mi_deblock_frame_dc)
    const int tid = threadIdx.x;
    KTL(0);
    if (tid < 64) { le[tid] = a.lim_e[tid]; li[tid] = a.lim_i[tid]; }
    if (tid < 8) cnt[tid] = 0;
    const LfTile g = lf_tile_at(a, xcd_block(blockIdx.x, gridDim.x));
    __syncthreads();
    uint4 sv[S::NS];
    LfEdgeRaw raw[S::NU];
    // the DC map's entries first (after the pixels: no measurable difference)
    const uint2 dcv = a.dc_map ? lf_dc_fetch(a, g) : make_uint2(0, 0);
    lf_fetch<Px>(a, g, sv, raw);
    if (a.dc_map) {
        lf_dc_commit(a, dcv, dcs);
        __syncthreads();
        lf_commit_pixels_dc<Px>(t, sv, dcs, a.bdmax);
    } else {
        lf_commit_pixels<Px>(t, sv);
    }
    KTL(1);
    lf_build_lists<Px>(g, raw, listv, listh, cnt);
    __syncthreads();
    KTL(2);
    // column edges, then row edges, one loop per width class
    lf_dir_pk<true, Px, S::P>(t, listv, cnt, le, li, a.bdm8, a.bdmax);
    __syncthreads();
    KTL(3);
    lf_dir_pk<false, Px, S::P>(t, listh, cnt + 4, le, li, a.bdm8, a.bdmax);
    __syncthreads();
    KTL(4);
    lf_store_tile<Px>(g, t);
    KTL(5);
}

int launch_deblock_tiles(const LfTileArgs &a, int bpc, hipStream_t s) {
    const int n = a.tile_start[3];
    if (!n) return 0;
    const int grid = n;
    if (bpc == 8) hipLaunchKernelGGL(lf_tile_kernel<uint8_t>, dim3(grid), dim3(kLfThreads), 0, s, a);
    else hipLaunchKernelGGL(lf_tile_kernel<uint16_t>, dim3(grid), dim3(kLfThreads), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---- per-call loop_filter_sb[cls][dir] (loopfilter.rs:745-985) ----
// One lane per pixel line of the (up to 32) 4-px units of one edge run: bit k of the masks
// selects unit k; dst is the edge's first q0 sample. Units of one run never overlap.
template <typename Px>
__global__ __launch_bounds__(128) void lf_sb_call_kernel(LfCallArgs a) {
    const int k = threadIdx.x >> 2, line = threadIdx.x & 3;
    const unsigned bit = 1u << k;
    const unsigned vm = a.cls == 0 ? (a.vmask[0] | a.vmask[1] | a.vmask[2]) : (a.vmask[0] | a.vmask[1]);
    if (!(vm & bit)) return;
    // lvl: per unit {its level slot, the left (dir 0) / upper (dir 1) neighbour's}, gathered
    // from the caller's strided [u8;4] map by the entry point
    int L = a.lvl[2 * k] ? a.lvl[2 * k] : a.lvl[2 * k + 1];
    if (!L) return;
    const int wd = a.cls == 0 ? 4 << ((a.vmask[2] & bit) ? 2 : !!(a.vmask[1] & bit)) : 4 + 2 * !!(a.vmask[1] & bit);
    const int64_t ps = a.stride / (int64_t)sizeof(Px);
    // dir 0 (column edges): unit k is rows 4k..4k+3, filtering along the row (step 1);
    // dir 1 (row edges): unit k is columns 4k..4k+3, filtering down the column (step ps)
    Px *q0 = reinterpret_cast<Px *>(a.dst) + (a.dir == 0 ? (4 * k + line) * ps : 4 * k + line);
    filter_line<Px>(q0, a.dir == 0 ? 1 : ps, wd, a.lim_e[L], a.lim_i[L], L >> 4, a.bdm8, a.bdmax);
}

int launch_lf_sb_call(const LfCallArgs &a, int bpc, hipStream_t s) {
    if (bpc == 8) lf_sb_call_kernel<uint8_t><<<1, 128, 0, s>>>(a);
    else lf_sb_call_kernel<uint16_t><<<1, 128, 0, s>>>(a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
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
