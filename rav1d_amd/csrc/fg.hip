// fg.hip — film-grain synthesis on gfx950 (output-only path).
//
// Replaces rav1d_prep_grain / rav1d_apply_grain_row (rav1d src/fg_apply.rs:14-284) and the DSP
// generate_grain_y/uv, fgy_32x32xn, fguv_32x32xn (src/filmgrain.rs:255-830; C
// filmgrain_tmpl.c).
//
// prep (one workgroup, independent of the pixels, so it can run on a side stream at frame
// start): the 16-bit LFSR is linear over GF(2), so lane i jumps straight to its slice of the
// random sequence with a precomputed matrix power and the grain templates fill in parallel;
// the auto-regressive filter runs as a skewed wavefront (row y lags row y-1 by lag+1
// columns, one LDS barrier per step); scaling LUTs are filled from their closed form; the
// per-(32-row, 32-col) block offsets are drawn by one lane per block row.
// apply: one lane per 4 output pixels of one plane row; grain templates, scaling LUTs and
// offsets are read through L1/L2 (a few tens of KB, cache resident).
#include "common.h"

namespace mi {

__constant__ int16_t k_gauss[2048] = {
#include "tables/gaussian_sequence.inc"
};
__constant__ uint16_t k_lfsr_jump[256][16];   // M^(24*i) as 16 column vectors

constexpr int kGW = 82, kGH = 73, kDrawsPerLane = 24;

__device__ __forceinline__ unsigned lfsr_step(unsigned s) {
    const unsigned bit = (s ^ (s >> 1) ^ (s >> 3) ^ (s >> 12)) & 1;
    return ((s >> 1) | (bit << 15)) & 0xffff;
}
__device__ __forceinline__ int round2i(int x, int sh) { return (x + ((1 << sh) >> 1)) >> sh; }

// Random fill of one grain template (generate_grain_*: first loop).
__device__ void grain_fill(int16_t *buf, int gw, int gh, unsigned seed, int shift) {
    const int n = gw * gh;
    for (int lane = threadIdx.x; lane * kDrawsPerLane < n; lane += 256) {
        unsigned s = 0;
#pragma unroll
        for (int j = 0; j < 16; j++)
            if ((seed >> j) & 1) s ^= k_lfsr_jump[lane][j];
        const int d0 = lane * kDrawsPerLane;
        for (int k = 0; k < kDrawsPerLane && d0 + k < n; k++) {
            s = lfsr_step(s);
            const int d = d0 + k;
            buf[(d / gw) * kGW + d % gw] = (int16_t)round2i(k_gauss[(s >> 5) & 0x7ff], shift);
        }
    }
}

// Auto-regressive pass as a skewed wavefront. `lane_base` selects the lanes that own rows.
__device__ void grain_ar(int16_t *buf, const int16_t *buf_y, int gw, int gh, const int8_t *coef,
                         int lag, int shift, int gmin, int gmax, bool chroma, bool luma_term,
                         int subx, int suby, int lane) {
    const int skew = lag + 1;
    const int nrows = gh - 3, ncols = gw - 6;
    const int steps = ncols + skew * (nrows - 1);
    for (int t = 0; t < steps; t++) {
        const int r = lane;
        if (r >= 0 && r < nrows) {
            const int x = 3 + t - skew * r, y = 3 + r;
            if (x >= 3 && x < gw - 3) {
                int sum = 0, ci = 0;
                for (int dy = -lag; dy <= 0; dy++)
                    for (int dx = -lag; dx <= lag; dx++) {
                        if (!dx && !dy) {
                            if (chroma && luma_term) {
                                int l = 0;
                                const int lx = ((x - 3) << subx) + 3, ly = ((y - 3) << suby) + 3;
                                for (int i = 0; i <= suby; i++)
                                    for (int j = 0; j <= subx; j++) l += buf_y[(ly + i) * kGW + lx + j];
                                sum += round2i(l, subx + suby) * coef[ci];
                            }
                            dy = 1;   // leave both loops
                            break;
                        }
                        sum += coef[ci++] * buf[(y + dy) * kGW + x + dx];
                    }
                const int g = buf[y * kGW + x] + round2i(sum, shift);
                buf[y * kGW + x] = (int16_t)min(max(g, gmin), gmax);
            }
        }
        __syncthreads();
    }
}

// Closed form of generate_scaling (fg_apply.rs:14-72) for entry e.
__device__ int scaling_coarse(const uint8_t (*pts)[2], int num, int k /* coarse index */) {
    if (k < pts[0][0]) return pts[0][1];
    if (k >= pts[num - 1][0]) return pts[num - 1][1];
    int i = 0;
    while (i < num - 2 && k >= pts[i + 1][0]) i++;
    const int bx = pts[i][0], by = pts[i][1], dx = pts[i + 1][0] - bx, dy = pts[i + 1][1] - by;
    const int delta = dy * ((0x10000 + (dx >> 1)) / dx);
    return by + ((0x8000 + (k - bx) * delta) >> 16);
}
__device__ int scaling_entry(const uint8_t (*pts)[2], int num, int e, int shx) {
    if (num == 0) return 0;
    const int k = e >> shx, n = e & ((1 << shx) - 1);
    const int base = scaling_coarse(pts, num, k);
    if (!n || k < pts[0][0] || k >= pts[num - 1][0]) return base & 0xff;
    const int next = scaling_coarse(pts, num, k + 1);
    const int range = (next & 0xff) - (base & 0xff);
    const int r = ((1 << shx) >> 1) + n * range;
    return ((base & 0xff) + (r >> shx)) & 0xff;
}

__global__ __launch_bounds__(256) void fg_prep_kernel(FgArgs a) {
    __shared__ int16_t lut[3][kGH][kGW];
    const MiFilmGrainData &d = a.data;
    const int bdm8 = a.bpc - 8;
    const int shift = 4 - bdm8 + d.grain_scale_shift;
    const int gctr = 128 << bdm8;
    const bool uv0 = a.layout && (d.num_uv_points[0] || d.chroma_scaling_from_luma);
    const bool uv1 = a.layout && (d.num_uv_points[1] || d.chroma_scaling_from_luma);
    const int cw = a.ss_x ? 44 : kGW, chh = a.ss_y ? 38 : kGH;

    grain_fill(&lut[0][0][0], kGW, kGH, d.seed, shift);
    if (uv0) grain_fill(&lut[1][0][0], cw, chh, d.seed ^ 0xb524, shift);
    if (uv1) grain_fill(&lut[2][0][0], cw, chh, d.seed ^ 0x49d8, shift);
    __syncthreads();
    grain_ar(&lut[0][0][0], nullptr, kGW, kGH, d.ar_coeffs_y, d.ar_coeff_lag, (int)d.ar_coeff_shift,
             -gctr, gctr - 1, false, false, 0, 0, threadIdx.x);
    // both chroma templates advance together: lanes 0..127 own U rows, 128..255 own V rows
    {
        const int pl = threadIdx.x >> 7;
        const bool on = pl ? uv1 : uv0;
        grain_ar(&lut[1 + pl][0][0], &lut[0][0][0], cw, chh, d.ar_coeffs_uv[pl], d.ar_coeff_lag,
                 (int)d.ar_coeff_shift, -gctr, gctr - 1, true, d.num_y_points != 0, a.ss_x, a.ss_y,
                 on ? (threadIdx.x & 127) : -1);
    }
    // export templates
    for (int i = threadIdx.x; i < 3 * kGH * kGW; i += 256) a.lut[i] = (&lut[0][0][0])[i];

    // scaling LUTs
    const int size = 1 << a.bpc;
    for (int i = threadIdx.x; i < 3 * size; i += 256) {
        const int pl = i / size, e = i % size;
        int v = 0;
        if (pl == 0) { if (d.num_y_points || d.chroma_scaling_from_luma) v = scaling_entry(d.y_points, d.num_y_points, e, bdm8); }
        else if (d.num_uv_points[pl - 1]) v = scaling_entry(d.uv_points[pl - 1], d.num_uv_points[pl - 1], e, bdm8);
        a.scaling[pl * 4096 + e] = (uint8_t)v;
    }
    // per-block offsets, one lane per 32-row block row (filmgrain.rs row_seed + draws)
    for (int row = threadIdx.x; row < a.nrows; row += 256) {
        unsigned s = d.seed;
        s ^= (unsigned)(((row * 37 + 178) & 0xFF) << 8);
        s ^= (unsigned)((row * 173 + 105) & 0xFF);
        for (int b = 0; b < a.nblocks; b++) {
            s = lfsr_step(s);
            a.offsets[row * a.nblocks + b] = (uint8_t)((s >> 8) & 0xff);
        }
    }
}

__device__ __forceinline__ int lut_at(const int16_t *lut, int rv, int subx, int suby, int bx, int by, int x, int y) {
    const int ox = 3 + (2 >> subx) * (3 + (rv >> 4));
    const int oy = 3 + (2 >> suby) * (3 + (rv & 0xF));
    return lut[(oy + y + (32 >> suby) * by) * kGW + ox + x + (32 >> subx) * bx];
}

template <typename Px>
__global__ __launch_bounds__(256) void fg_apply_kernel(FgArgs a) {
    const int b = blockIdx.x;
    const int p = b < a.blk_start[1] ? 0 : b < a.blk_start[2] ? 1 : 2;
    const int lb = b - a.blk_start[p];
    const int chunks = a.chunks[p];
    const int idx = lb * 256 + threadIdx.x;
    const int y = idx / chunks, x0 = (idx % chunks) * 4;
    const int pw = a.pw[p], ph = a.ph[p];
    if (y >= ph) return;
    const MiFilmGrainData &d = a.data;
    const int sx = p ? a.ss_x : 0, sy = p ? a.ss_y : 0;
    const int64_t st = a.stride[p];
    const Px *src = reinterpret_cast<const Px *>(a.src[p] + (int64_t)y * st);
    Px *dst = reinterpret_cast<Px *>(a.dst[p] + (int64_t)y * st);
    if (!a.grain[p]) {
        for (int x = x0; x < min(x0 + 4, pw); x++) dst[x] = src[x];
        return;
    }
    const int bdm8 = a.bpc - 8, bdmax = (1 << a.bpc) - 1;
    const int gctr = 128 << bdm8, gmin = -gctr, gmax = gctr - 1;
    int minv = 0, maxv = bdmax;
    if (d.clip_to_restricted_range) {
        minv = 16 << bdm8;
        maxv = (p == 0 || a.is_id ? 235 : 240) << bdm8;
    }
    const int bsh = 32 >> sy, bsw = 32 >> sx;
    const int row = y / bsh, yy = y % bsh;
    const int bh = p ? (min(a.h - row * 32, 32) + sy) >> sy : min(a.h - row * 32, 32);
    const int16_t *lut = a.lut + p * kGH * kGW;
    const uint8_t *scl = a.scaling + (p && !d.chroma_scaling_from_luma ? p : 0) * 4096;
    const uint8_t *offr = a.offsets + row * a.nblocks;
    const uint8_t *offp = row ? a.offsets + (row - 1) * a.nblocks : offr;
    const int wl[2][2] = { { 27, 17 }, { 17, 27 } };
    const int ws[2] = { 23, 22 };
    const Px *luma = nullptr;
    int64_t lrow = 0;
    if (p) {
        lrow = (int64_t)(row * 32 + (yy << sy));
        luma = reinterpret_cast<const Px *>(a.src[0] + lrow * a.stride[0]);
    }
    for (int x = x0; x < min(x0 + 4, pw); x++) {
        const int bi = x / bsw, xx = x % bsw;
        const int bw = min(bsw, pw - bi * bsw);
        const int ystart = d.overlap_flag && row ? min(2 >> sy, bh) : 0;
        const int xstart = d.overlap_flag && bi ? min(2 >> sx, bw) : 0;
        const int rc = offr[bi];
        int grain = lut_at(lut, rc, sx, sy, 0, 0, xx, yy);
        const int wx0 = sx ? ws[0] : wl[xx & 1][0], wx1 = sx ? ws[1] : wl[xx & 1][1];
        const int wy0 = sy ? ws[0] : wl[yy & 1][0], wy1 = sy ? ws[1] : wl[yy & 1][1];
        if (xx < xstart && yy >= ystart) {
            const int old = lut_at(lut, offr[bi - 1], sx, sy, 1, 0, xx, yy);
            grain = min(max(round2i(old * wx0 + grain * wx1, 5), gmin), gmax);
        } else if (xx >= xstart && yy < ystart) {
            const int old = lut_at(lut, offp[bi], sx, sy, 0, 1, xx, yy);
            grain = min(max(round2i(old * wy0 + grain * wy1, 5), gmin), gmax);
        } else if (xx < xstart && yy < ystart) {
            int top = lut_at(lut, offp[bi], sx, sy, 0, 1, xx, yy);
            int old = lut_at(lut, offp[bi - 1], sx, sy, 1, 1, xx, yy);
            top = min(max(round2i(old * wx0 + top * wx1, 5), gmin), gmax);
            old = lut_at(lut, offr[bi - 1], sx, sy, 1, 0, xx, yy);
            grain = min(max(round2i(old * wx0 + grain * wx1, 5), gmin), gmax);
            grain = min(max(round2i(top * wy0 + grain * wy1, 5), gmin), gmax);
        }
        const int s = src[x];
        int val = s;
        if (p) {
            const int lx = x << sx;
            int avg = luma[lx];
            if (sx) avg = (avg + luma[min(lx + 1, a.w - 1)] + 1) >> 1;
            val = avg;
            if (!d.chroma_scaling_from_luma) {
                const int comb = avg * d.uv_luma_mult[p - 1] + s * d.uv_mult[p - 1];
                val = min(max((comb >> 6) + d.uv_offset[p - 1] * (1 << bdm8), 0), bdmax);
            }
        }
        const int noise = round2i(scl[val] * grain, d.scaling_shift);
        dst[x] = (Px)min(max(s + noise, minv), maxv);
    }
}

int init_fg_tables() {
    // columns of the LFSR step matrix M, then M^(24 i) by repeated multiplication
    uint16_t m[16], p[16], host[256][16];
    auto step = [](unsigned s) {
        const unsigned bit = (s ^ (s >> 1) ^ (s >> 3) ^ (s >> 12)) & 1;
        return (uint16_t)(((s >> 1) | (bit << 15)) & 0xffff);
    };
    auto apply = [](const uint16_t *mat, unsigned v) {
        unsigned r = 0;
        for (int j = 0; j < 16; j++)
            if ((v >> j) & 1) r ^= mat[j];
        return (uint16_t)r;
    };
    for (int j = 0; j < 16; j++) m[j] = step(1u << j);
    uint16_t m24[16];
    for (int j = 0; j < 16; j++) {
        unsigned v = 1u << j;
        for (int k = 0; k < kDrawsPerLane; k++) v = apply(m, v);
        m24[j] = (uint16_t)v;
    }
    for (int j = 0; j < 16; j++) p[j] = (uint16_t)(1u << j);   // identity
    for (int i = 0; i < 256; i++) {
        for (int j = 0; j < 16; j++) host[i][j] = p[j];
        uint16_t q[16];
        for (int j = 0; j < 16; j++) q[j] = apply(m24, p[j]);
        for (int j = 0; j < 16; j++) p[j] = q[j];
    }
    return hipMemcpyToSymbol(HIP_SYMBOL(k_lfsr_jump), host, sizeof(host)) == hipSuccess ? 0 : -5;
}

int launch_fg(const FgArgs &a, hipStream_t s, bool prep, bool apply) {
    if (prep) hipLaunchKernelGGL(fg_prep_kernel, dim3(1), dim3(256), 0, s, a);
    if (apply && a.blk_start[3] > 0) {
        if (a.bpc == 8) hipLaunchKernelGGL(fg_apply_kernel<uint8_t>, dim3(a.blk_start[3]), dim3(256), 0, s, a);
        else hipLaunchKernelGGL(fg_apply_kernel<uint16_t>, dim3(a.blk_start[3]), dim3(256), 0, s, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
