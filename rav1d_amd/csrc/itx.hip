// itx.hip — batched inverse transform + add for a whole frame on gfx950.
//
// Replaces the per-block itxfm_add[tx][txtp] calls made from recon (rav1d src/recon.rs:
// 1781-1788, 2674-2682, 3116, 4013) with one launch per frame. Semantics per block are
// inv_txfm_add_rust (src/itx.rs:64-188; C src/itx_tmpl.c:40-100) and the lossless WHT
// (src/itx.rs:475-526; C src/itx_tmpl.c:162-181).
//
// Mapping. Blocks arrive grouped by tx size; a 256-lane workgroup takes BPW blocks of one
// size. Within a block, lane j first runs the 1-D row transform of row j (coefficients read
// straight from the arena's column-major layout, so lanes j..j+sh-1 read consecutive
// addresses), writes the shifted/clipped row to LDS, then after one barrier runs the 1-D
// column transform of column j and adds it to the picture (lanes of a block touch
// consecutive pixels of each row). Butterflies live entirely in VGPRs; no MFMA (these are
// small fixed integer networks, not contractions).
#include "common.h"
#include "itx_1d.h"

namespace mi {

// TxfmType -> 1-D kinds (levels.rs TxfmType is VERT_HORZ; itx_tmpl.c:196-233)
__constant__ uint8_t k_col_kind[16] = { KD, KA, KD, KA, KF, KD, KF, KA, KF, KI, KD, KI, KA, KI, KF, KI };
__constant__ uint8_t k_row_kind[16] = { KD, KD, KA, KA, KD, KF, KF, KF, KA, KI, KI, KD, KI, KA, KI, KF };

// Largest per-WG LDS need: BPW * SH * (W + 1) ints over all sizes (32x32/32x64: 8*32*33).
constexpr int kItxLdsInts = 8 * 32 * 33;

template <int TX, typename Px, typename Cf, bool Wide>
__device__ __forceinline__ void itx_size(const ItxArgs &a, int lwg, int *lds) {
    constexpr TxDim D = tx_dim(TX);
    constexpr int Wd = D.w, Ht = D.h, SH = imin_c(Ht, 32), SW = imin_c(Wd, 32);
    constexpr int TPB = itx_lanes(TX), BPW = kItxThreads / TPB;
    constexpr int LS = Wd + 1;                       // padded LDS row stride (ints)
    constexpr bool Rect2 = (Wd == 2 * Ht) || (Ht == 2 * Wd);
    constexpr int Shift = D.shift, Rnd = (1 << Shift) >> 1;
    static_assert(BPW * SH * LS <= kItxLdsInts, "itx LDS budget");

    const int t = threadIdx.x;
    const int lb = t / TPB, j = t % TPB;
    const int bi = a.blk_start[TX] + lwg * BPW + lb;
    const bool valid = bi < a.blk_start[TX + 1];

    MiTxBlock b{};
    if (valid) b = a.blocks[bi];
    const int bdmax = a.bdmax;
    Cf *cf = reinterpret_cast<Cf *>(a.coef) + b.coef_off;
    const bool wht = (TX == 0) && b.txtp == 16;
    const bool dconly = b.txtp == 0 && b.eob < 1;
    int *tmp = lds + lb * SH * LS;

    int row_lo, col_lo;
    if constexpr (sizeof(Px) == 1) { row_lo = -32768; col_lo = -32768; }
    else { row_lo = (int)((unsigned)~bdmax << 7); col_lo = (int)((unsigned)~bdmax << 5); }
    const int row_hi = ~row_lo, col_hi = ~col_lo;

    // ---- row pass ----
    if (valid && !dconly && j < SH) {
        int r[Wd];
#pragma unroll
        for (int x = 0; x < Wd; x++) r[x] = 0;
#pragma unroll
        for (int x = 0; x < SW; x++) {
            const int v = (int)cf[j + x * SH];
            if constexpr (Rect2) r[x] = (v * 181 + 128) >> 8;
            else r[x] = v;
        }
        if (a.zero_coefs) {
#pragma unroll
            for (int x = 0; x < SW; x++) cf[j + x * SH] = 0;
        }
        if constexpr (TX == 0) {
            if (wht) {
#pragma unroll
                for (int x = 0; x < 4; x++) r[x] >>= 2;
                iwht4(r);
#pragma unroll
                for (int x = 0; x < 4; x++) tmp[j * LS + x] = r[x];
            }
        }
        if (!wht) {
            itx1d<Wide, Wd>(k_row_kind[b.txtp], r, row_lo, row_hi);
#pragma unroll
            for (int x = 0; x < Wd; x++)
                tmp[j * LS + x] = clampi((r[x] + Rnd) >> Shift, col_lo, col_hi);
        }
    }
    __syncthreads();

    // ---- column pass + add ----
    if (valid && j < Wd) {
        Px *dst = reinterpret_cast<Px *>(a.plane[b.plane] + (int64_t)b.y * a.stride[b.plane]) + b.x + j;
        const int64_t ps = a.stride[b.plane] / (int64_t)sizeof(Px);
        if (dconly) {
            int dc = (int)cf[0];
            if (Rect2) dc = (dc * 181 + 128) >> 8;
            dc = (dc * 181 + 128) >> 8;
            dc = (dc + Rnd) >> Shift;
            dc = (dc * 181 + 128 + 2048) >> 12;
#pragma unroll 4
            for (int y = 0; y < Ht; y++)
                dst[y * ps] = (Px)clampi((int)dst[y * ps] + dc, 0, bdmax);
        } else {
            int c[Ht];
#pragma unroll
            for (int y = 0; y < Ht; y++) c[y] = y < SH ? tmp[y * LS + j] : 0;
            if (wht) {
                if constexpr (TX == 0) {
                    iwht4(c);
#pragma unroll
                    for (int y = 0; y < 4; y++)
                        dst[y * ps] = (Px)clampi((int)dst[y * ps] + c[y], 0, bdmax);
                }
            } else {
                itx1d<Wide, Ht>(k_col_kind[b.txtp], c, col_lo, col_hi);
#pragma unroll
                for (int y = 0; y < Ht; y++)
                    dst[y * ps] = (Px)clampi((int)dst[y * ps] + ((c[y] + 8) >> 4), 0, bdmax);
            }
        }
    }
    // DC-only blocks clear their single coefficient after all lanes consumed it.
    __syncthreads();
    if (valid && dconly && j == 0 && a.zero_coefs) cf[0] = 0;
}

template <typename Px, typename Cf, bool Wide>
__global__ __launch_bounds__(kItxThreads) void itx_frame_kernel(ItxArgs a) {
    __shared__ int lds[kItxLdsInts];
    const int wg = blockIdx.x;
    int s = 0;
    while (s < 18 && wg >= a.wg_start[s + 1]) s++;
    const int lwg = wg - a.wg_start[s];
    switch (s) {
#define CASE(n) case n: itx_size<n, Px, Cf, Wide>(a, lwg, lds); break;
        CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9)
        CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16) CASE(17) CASE(18)
#undef CASE
    default: break;
    }
}

int launch_itx_frame(const ItxArgs &a, int total_wg, int bpc, hipStream_t s) {
    if (total_wg <= 0) return 0;
    if (bpc == 8)
        hipLaunchKernelGGL((itx_frame_kernel<uint8_t, int16_t, false>), dim3(total_wg), dim3(kItxThreads), 0, s, a);
    else if (bpc == 10)
        hipLaunchKernelGGL((itx_frame_kernel<uint16_t, int32_t, false>), dim3(total_wg), dim3(kItxThreads), 0, s, a);
    else
        hipLaunchKernelGGL((itx_frame_kernel<uint16_t, int32_t, true>), dim3(total_wg), dim3(kItxThreads), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
