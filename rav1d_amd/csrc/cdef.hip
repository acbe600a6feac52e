// cdef.hip — whole-frame CDEF on gfx950, out of place (deblocked D -> C).
//
// Replaces rav1d_cdef_brow (rav1d src/cdef_apply.rs:159-507) and the DSP cdef.dir/cdef.fb[3]
// (src/cdef.rs:545-1031; C src/cdef_tmpl.c). The reference filters in place and keeps line and
// column backups so every block reads deblocked (pre-CDEF) samples only; reading an immutable
// D and writing C gives the same result without backups.
//
// One 256-lane workgroup per 64x64 luma unit (the granularity of cdef_idx, so strengths are
// workgroup-uniform) plus its co-located chroma. The tile and a 2-px halo are staged in LDS as
// int16 with i16::MIN where the reference's padding marks samples unavailable (frame edges,
// cdef.rs:567-665). Phase 1: 64 lanes find the 8x8 directions; phase 2: every lane filters
// pixels straight out of LDS and streams C back with coalesced stores.
#include "cdef_dev.h"

MI_KTL_DEFINE(cdef)

namespace mi {


// One 64x64 luma unit (+ co-located chroma) per 512-lane workgroup (eight waves: one per
// direction in the search, 34 KB of LDS for four workgroups = 32 waves per CU). L = layout (0 I400,
// 1 I420, 2 I422, 3 I444), compile-time so every tile index is a shift or a constant divide.
template <typename Px, int L>
__global__ __launch_bounds__(512, 8) void cdef_kernel(CdefArgs a) {
    constexpr int NTH = 512;
    constexpr int SSH = L == 1 || L == 2, SSV = L == 1;
    constexpr int CW = 64 >> SSH, CH = 64 >> SSV, CTS = CW == 64 ? 88 : 48;   // 24-dword rows: two rows 2 apart are 16 banks apart
    constexpr int UVW = 8 >> SSH, UVH = 8 >> SSV;
    constexpr int YN = kTY * kTS, CN = L ? (CH + 4) * CTS : 2;
    constexpr int NT = 2;
    __shared__ __align__(16) int16_t ty[NT * YN];              // T, T1
    __shared__ __align__(16) int16_t tuv[2][NT * CN];          // per chroma plane: T, T1
    __shared__ int8_t bdir[64];
    __shared__ int8_t bflag[64];          // bit0 luma filtered, bit1 chroma filtered
    __shared__ unsigned dcost[8][64];     // find_dir costs per direction and block
    __shared__ int bstate[64];            // luma: filtered | dir << 8 | adjusted pri << 16
    __shared__ int4 ytaps[8][3];          // luma tap byte deltas per direction (PairTaps order)
    __shared__ int4 ctaps[8][3];          // 4:2:0 chroma tap byte deltas per direction
    KTL(0);

    const int bid = xcd_block(blockIdx.x, gridDim.x);
    const int tx = bid % a.tiles_x, tyy = bid / a.tiles_x;
    const int x0 = tx * 64, y0 = tyy * 64;
    const MiAv1Filter *lf = &a.masks[(tyy >> 1) * a.sb128w + (tx >> 1)];
    const int cdef_idx = lf->cdef_idx[(tyy & 1) * 2 + (tx & 1)];
    const int y_lvl = cdef_idx >= 0 ? a.y_strength[cdef_idx] : 0;
    const int uv_lvl = cdef_idx >= 0 && L ? a.uv_strength[cdef_idx] : 0;
    const int fwy = a.bw4 * 4, fhy = a.bh4 * 4;
    const int fwc = fwy >> SSH, fhc = fhy >> SSV;

    if (!y_lvl && !uv_lvl) {
        // untouched 64x64 unit: C = D, 8 bytes per lane
        constexpr int PX8 = 8 / sizeof(Px);
#pragma unroll
        for (int p = 0; p < (L ? 3 : 1); p++) {
            const int pw = p ? CW : 64, ph = p ? CH : 64;
            const int px0 = p ? x0 >> SSH : x0, py0 = p ? y0 >> SSV : y0;
            const int cpr = pw / PX8;   // 8-byte chunks per row
            for (int i = threadIdx.x; i < cpr * ph; i += NTH) {
                const int r = i / cpr, c = i - r * cpr;
                const int64_t off = (int64_t)(py0 + r) * a.stride[p] + (int64_t)(px0 + c * PX8) * sizeof(Px);
                *reinterpret_cast<uint2 *>(a.dst[p] + off) = *reinterpret_cast<const uint2 *>(a.src[p] + off);
            }
        }
        KTL(5);
        return;
    }

    const int bdm8 = a.bdm8;
    const int y_pri = (y_lvl >> 2) << bdm8;
    int y_sec = y_lvl & 3; y_sec += y_sec == 3; y_sec <<= bdm8;
    const int uv_pri = (uv_lvl >> 2) << bdm8;
    int uv_sec = uv_lvl & 3; uv_sec += uv_sec == 3; uv_sec <<= bdm8;

    if (threadIdx.x < 8) {
        PairTaps t;
        make_taps<kTS, YN * 2>(t, threadIdx.x);
        ytaps[threadIdx.x][0] = make_int4(t.pri[0], t.pri[1], t.pri[2], t.pri[3]);
        ytaps[threadIdx.x][1] = make_int4(t.sec[0], t.sec[1], t.sec[2], t.sec[3]);
        ytaps[threadIdx.x][2] = make_int4(t.sec[4], t.sec[5], t.sec[6], t.sec[7]);
    } else if (L == 1 && threadIdx.x < 16) {
        PairTaps t;
        make_taps<CTS, CN * 2>(t, threadIdx.x - 8);
        ctaps[threadIdx.x - 8][0] = make_int4(t.pri[0], t.pri[1], t.pri[2], t.pri[3]);
        ctaps[threadIdx.x - 8][1] = make_int4(t.sec[0], t.sec[1], t.sec[2], t.sec[3]);
        ctaps[threadIdx.x - 8][2] = make_int4(t.sec[4], t.sec[5], t.sec[6], t.sec[7]);
    }
    {
        VecTileLoad<Px, 68, 68, NTH> ly;
        VecTileLoad<Px, CH + 4, CW + 4, NTH> lu, lv;
        ly.fetch(a.src[0], a.stride[0], x0, y0, fwy, fhy);
        if (L && uv_lvl) {
            lu.fetch(a.src[1], a.stride[1], x0 >> SSH, y0 >> SSV, fwc, fhc);
            lv.fetch(a.src[2], a.stride[2], x0 >> SSH, y0 >> SSV, fwc, fhc);
        }
        ly.store(ty, ty + YN, kTS);
        if (L && uv_lvl) {
            lu.store(tuv[0], tuv[0] + CN, CTS);
            lv.store(tuv[1], tuv[1] + CN, CTS);
        }
    }
    __syncthreads();
    KTL(1);

    if (y_pri || uv_pri) {
        const int b = threadIdx.x & 63, w = threadIdx.x >> 6;   // wave-uniform direction
        const int16_t *tb = ty + ((b >> 3) * 8 + 2) * kTS + (b & 7) * 8 + 8;
        unsigned c;
        switch (w) {
        case 0: c = dir_cost1<0>(tb, kTS, bdm8); break;
        case 1: c = dir_cost1<1>(tb, kTS, bdm8); break;
        case 2: c = dir_cost1<2>(tb, kTS, bdm8); break;
        case 3: c = dir_cost1<3>(tb, kTS, bdm8); break;
        case 4: c = dir_cost1<4>(tb, kTS, bdm8); break;
        case 5: c = dir_cost1<5>(tb, kTS, bdm8); break;
        case 6: c = dir_cost1<6>(tb, kTS, bdm8); break;
        default: c = dir_cost1<7>(tb, kTS, bdm8); break;
        }
        dcost[w][b] = c;
        __syncthreads();
    }
    KTL(2);

    if (threadIdx.x < 64) {
        const int b = threadIdx.x, bxl = b & 7, byl = b >> 3;
        const int bx = (x0 >> 2) + bxl * 2, by = (y0 >> 2) + byl * 2;   // 4-px units
        int flag = 0, dir = 0, pri = 0;
        if (bx < a.bw4 && by < a.bh4) {
            const int by_idx = (by & 30) >> 1;
            const unsigned noskip = (unsigned)lf->noskip_mask[by_idx][1] << 16 | lf->noskip_mask[by_idx][0];
            if (noskip & (3u << (bx & 30))) {
                unsigned var = 0;
                if (y_pri || uv_pri) {
                    unsigned bc = dcost[0][b];
#pragma unroll
                    for (int n = 1; n < 8; n++)
                        if (dcost[n][b] > bc) { bc = dcost[n][b]; dir = n; }
                    var = (bc - dcost[dir ^ 4][b]) >> 10;
                }
                if (y_pri) {
                    pri = adjust_strength(y_pri, var);
                    if (pri || y_sec) flag |= 1;
                } else if (y_sec) {
                    flag |= 1;
                }
                if (uv_lvl) flag |= 2;
            }
        }
        bdir[b] = (int8_t)dir;
        bflag[b] = (int8_t)flag;
        bstate[b] = (flag & 1) | (y_pri ? dir : 0) << 8 | (y_pri ? pri : 0) << 16;
    }
    __syncthreads();
    KTL(3);

    // luma: 2048 pairs, one 8x8 block per 32-lane group at a time
    filter_luma<Px, kTS>(ty, ytaps, bstate, y_sec, a.damping, bdm8, a.src[0], a.dst[0], a.stride[0],
                             x0, y0, fwy, fhy);
    KTL(4);
    if (L) {
        // chroma: lanes 0..255 U, 256..511 V (damping - 1, cdef_apply.rs)
        const int p = 1 + (threadIdx.x >> 8);
        // (the chroma tile is only staged when uv_lvl != 0: unfiltered chroma copies from D)
        if constexpr (L == 1)
            filter_chroma420<Px, CTS>(tuv[p - 1], ctaps, bdir, bflag, uv_pri, uv_sec, a.damping - 1, bdm8,
                                      a.src[p], a.dst[p], a.stride[p], x0 >> SSH, y0 >> SSV);
        else
            filter_plane<Px, CW, CH, UVW, UVH, 256, CTS, CN * 2, 2, false>(
                tuv[p - 1], threadIdx.x & 255, bdir, bflag, nullptr, false, uv_pri, uv_sec, a.damping - 1, bdm8,
                L == 2, a.src[p], a.dst[p], a.stride[p], x0 >> SSH, y0 >> SSV, fwc, fhc);
    }
    KTL(5);
}

// ---- per-call cdef.fb[] / cdef.dir (cdef.rs:567-1031) ----
// One block (8x8, 4x8 or 4x4): the padded i16 tile is built in LDS as the reference's
// `padding` does (the block from dst, 2 columns from left, 2 rows above from top and below
// from bottom, i16::MIN where `edges` says the neighbour is missing), then one lane per pixel.
constexpr int kCallTs = 12;
template <typename Px>
__global__ __launch_bounds__(64) void cdef_call_kernel(CdefCallArgs a) {
    __shared__ int16_t tb[kCallTs * kCallTs];
    int16_t *t = tb + 2 * kCallTs + 2;
    const int lane = threadIdx.x, w = a.w, h = a.h;
    const int64_t ps = a.stride / (int64_t)sizeof(Px);
    const Px *dst = reinterpret_cast<const Px *>(a.dst), *top = reinterpret_cast<const Px *>(a.top);
    const Px *bot = reinterpret_cast<const Px *>(a.bottom), *left = reinterpret_cast<const Px *>(a.left);
    for (int i = lane; i < kCallTs * kCallTs; i += 64) {
        const int y = i / kCallTs - 2, x = i % kCallTs - 2;
        int v = INT16_MIN;
        if (y < h + 2 && x < w + 2) {
            const bool in_x = x >= 0 ? (x < w || (a.edges & 2)) : (a.edges & 1);   // HAVE_RIGHT 2, HAVE_LEFT 1
            const bool in_y = y >= 0 ? (y < h || (a.edges & 8)) : (a.edges & 4);   // HAVE_BOTTOM 8, HAVE_TOP 4
            if (in_x && in_y) {
                if (y < 0) v = top[(y + 2) * ps + x];
                else if (y >= h) v = bot[(y - h) * ps + x];
                else if (x < 0) v = left[y * 2 + 2 + x];
                else v = dst[y * ps + x];
            }
        }
        tb[i] = (int16_t)v;
    }
    __syncthreads();
    if (lane < w * h) {
        const int y = lane / w, x = lane % w;
        const int v = cdef_px(t, kCallTs, x, y, a.pri, a.sec, a.dir, a.damping, a.bdm8);
        reinterpret_cast<Px *>(a.out)[y * w + x] = (Px)v;
    }
}

template <typename Px>
__global__ __launch_bounds__(64) void cdef_dir_call_kernel(CdefCallArgs a) {
    __shared__ int16_t t[64];
    const int64_t ps = a.stride / (int64_t)sizeof(Px);
    const int lane = threadIdx.x;
    t[lane] = (int16_t)reinterpret_cast<const Px *>(a.dst)[(lane >> 3) * ps + (lane & 7)];
    __syncthreads();
    if (lane == 0) {
        unsigned var;
        const int d = find_dir(t, 8, a.bdm8, &var);
        reinterpret_cast<int *>(a.out)[0] = d;
        reinterpret_cast<unsigned *>(a.out)[1] = var;
    }
}

int launch_cdef_call(const CdefCallArgs &a, int bpc, bool dir, hipStream_t s) {
    if (dir) {
        if (bpc == 8) cdef_dir_call_kernel<uint8_t><<<1, 64, 0, s>>>(a);
        else cdef_dir_call_kernel<uint16_t><<<1, 64, 0, s>>>(a);
    } else {
        if (bpc == 8) cdef_call_kernel<uint8_t><<<1, 64, 0, s>>>(a);
        else cdef_call_kernel<uint16_t><<<1, 64, 0, s>>>(a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_cdef(const CdefArgs &a, int tiles, int bpc, hipStream_t s) {
    if (tiles <= 0) return 0;
#define MI_CDEF_LAUNCH(L)                                                                            \
    do {                                                                                             \
        if (bpc == 8) cdef_kernel<uint8_t, L><<<tiles, 512, 0, s>>>(a);                               \
        else cdef_kernel<uint16_t, L><<<tiles, 512, 0, s>>>(a);                                       \
    } while (0)
    switch (a.layout) {
    case 0: MI_CDEF_LAUNCH(0); break;
    case 1: MI_CDEF_LAUNCH(1); break;
    case 2: MI_CDEF_LAUNCH(2); break;
    default: MI_CDEF_LAUNCH(3); break;
    }
#undef MI_CDEF_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

} // namespace mi
