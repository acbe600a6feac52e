// masks.cpp — the blend masks of compound and inter-intra prediction (wedge.rs; C wedge.c) and
// the warped-motion solver (warpmv.rs; C warpmv.c:63-209). The masks are built once, exactly as
// dav1d_init_wedge_masks / dav1d_init_interintra_masks construct them; the descriptors of a
// frame then carry a copy of each mask a block uses.
#include <cstdlib>
#include <cstring>

#include "framedec.h"

namespace av1 {
namespace fd {

namespace {

enum { W_HOR, W_VER, W_O27, W_O63, W_O117, W_O153 };
struct WedgeCode { uint8_t dir, xo, yo; };
static const WedgeCode k_cb_hgtw[16] = {
    {W_O27, 4, 4}, {W_O63, 4, 4}, {W_O117, 4, 4}, {W_O153, 4, 4}, {W_HOR, 4, 2}, {W_HOR, 4, 4},
    {W_HOR, 4, 6}, {W_VER, 4, 4}, {W_O27, 4, 2},  {W_O27, 4, 6},  {W_O153, 4, 2}, {W_O153, 4, 6},
    {W_O63, 2, 4}, {W_O63, 6, 4}, {W_O117, 2, 4}, {W_O117, 6, 4},
};
static const WedgeCode k_cb_hltw[16] = {
    {W_O27, 4, 4}, {W_O63, 4, 4}, {W_O117, 4, 4}, {W_O153, 4, 4}, {W_VER, 2, 4}, {W_VER, 4, 4},
    {W_VER, 6, 4}, {W_HOR, 4, 4}, {W_O27, 4, 2},  {W_O27, 4, 6},  {W_O153, 4, 2}, {W_O153, 4, 6},
    {W_O63, 2, 4}, {W_O63, 6, 4}, {W_O117, 2, 4}, {W_O117, 6, 4},
};
static const WedgeCode k_cb_heqw[16] = {
    {W_O27, 4, 4}, {W_O63, 4, 4}, {W_O117, 4, 4}, {W_O153, 4, 4}, {W_HOR, 4, 2}, {W_HOR, 4, 6},
    {W_VER, 2, 4}, {W_VER, 6, 4}, {W_O27, 4, 2},  {W_O27, 4, 6},  {W_O153, 4, 2}, {W_O153, 4, 6},
    {W_O63, 2, 4}, {W_O63, 6, 4}, {W_O117, 2, 4}, {W_O117, 6, 4},
};

struct MaskTables {
    // wedge[bs][layout class][sign][idx]: w x h (class 0) or the subsampled size
    std::vector<uint8_t> store;
    const uint8_t *wedge[N_BS][3][2][16] = {};
    const uint8_t *ii[N_BS][3][4] = {};

    uint8_t *alloc(size_t n) {
        const size_t off = store.size();
        store.resize(off + n);
        return store.data() + off;
    }

    MaskTables() {
        store.reserve(1 << 20);   // pointers into store stay valid: no reallocation below
        uint8_t master[6][64 * 64];
        static const uint8_t border[3][8] = {
            {1, 2, 6, 18, 37, 53, 60, 63}, {1, 4, 11, 27, 46, 58, 62, 63}, {0, 2, 7, 21, 43, 57, 62, 64}};
        // the master templates: a soft edge (border line) through a 64x64 square
        auto line = [](uint8_t *dst, const uint8_t *src, int ctr) {
            if (ctr > 4) memset(dst, 0, ctr - 4);
            memcpy(dst + imax(ctr, 4) - 4, src + imax(4 - ctr, 0), imin(64 - ctr, 8));
            if (ctr < 64 - 4) memset(dst + ctr + 4, 64, 64 - 4 - ctr);
        };
        for (int y = 0; y < 64; y++) line(&master[W_VER][y * 64], border[2], 32);
        for (int y = 0, ctr = 48; y < 64; y += 2, ctr--) {
            line(&master[W_O63][y * 64], border[1], ctr);
            line(&master[W_O63][(y + 1) * 64], border[0], ctr - 1);
        }
        for (int y = 0; y < 64; y++)
            for (int x = 0; x < 64; x++) {
                master[W_O27][x * 64 + y] = master[W_O63][y * 64 + x];   // transpose
                master[W_HOR][x * 64 + y] = master[W_VER][y * 64 + x];
            }
        for (int y = 0; y < 64; y++)
            for (int x = 0; x < 64; x++) {
                master[W_O117][y * 64 + 63 - x] = master[W_O63][y * 64 + x];   // hflip
                master[W_O153][y * 64 + 63 - x] = master[W_O27][y * 64 + x];
            }
        struct Fill { int bs, w, h; const WedgeCode *cb; unsigned signs; };
        static const Fill fills[9] = {
            {BS_32x32, 32, 32, k_cb_heqw, 0x7bfb}, {BS_32x16, 32, 16, k_cb_hltw, 0x7beb},
            {BS_32x8, 32, 8, k_cb_hltw, 0x6beb},   {BS_16x32, 16, 32, k_cb_hgtw, 0x7beb},
            {BS_16x16, 16, 16, k_cb_heqw, 0x7bfb}, {BS_16x8, 16, 8, k_cb_hltw, 0x7beb},
            {BS_8x32, 8, 32, k_cb_hgtw, 0x7aeb},   {BS_8x16, 8, 16, k_cb_hgtw, 0x7beb},
            {BS_8x8, 8, 8, k_cb_heqw, 0x7bfb},
        };
        for (const Fill &f : fills) {
            const int w = f.w, hh = f.h, n444 = w * hh;
            // 16 masks cut from the masters, then their inversions (fill2d_16x2)
            uint8_t *m444 = alloc((size_t)2 * 16 * n444);
            for (int n = 0; n < 16; n++) {
                const uint8_t *src = master[f.cb[n].dir] + (32 - (hh * f.cb[n].yo >> 3)) * 64 + (32 - (w * f.cb[n].xo >> 3));
                for (int y = 0; y < hh; y++) memcpy(m444 + n * n444 + y * w, src + y * 64, w);
            }
            for (int i = 0; i < 16 * n444; i++) m444[16 * n444 + i] = (uint8_t)(64 - m444[i]);
            uint8_t *m422 = alloc((size_t)2 * 16 * (n444 >> 1)), *m420 = alloc((size_t)2 * 16 * (n444 >> 2));
            for (int n = 0; n < 16; n++) {
                const int sign = (f.signs >> n) & 1;
                const uint8_t *luma = m444 + sign * 16 * n444 + n * n444;
                wedge[f.bs][0][0][n] = wedge[f.bs][0][1][n] = luma;
                uint8_t *c422[2] = { m422 + sign * 16 * (n444 >> 1) + n * (n444 >> 1),
                                     m422 + !sign * 16 * (n444 >> 1) + n * (n444 >> 1) };
                uint8_t *c420[2] = { m420 + sign * 16 * (n444 >> 2) + n * (n444 >> 2),
                                     m420 + !sign * 16 * (n444 >> 2) + n * (n444 >> 2) };
                wedge[f.bs][1][0][n] = c422[0];
                wedge[f.bs][1][1][n] = c422[1];
                wedge[f.bs][2][0][n] = c420[0];
                wedge[f.bs][2][1][n] = c420[1];
                // init_chroma: averages of 2 (422) or 4 (420) luma weights, rounded toward the sign
                for (int s = 0; s < 2; s++)
                    for (int ssv = 0; ssv < 2; ssv++) {
                        uint8_t *c = ssv ? c420[s] : c422[s];
                        const uint8_t *lp = luma;
                        for (int y = 0; y < hh; y += 1 + ssv) {
                            for (int x = 0; x < w; x += 2) {
                                int sum = lp[x] + lp[x + 1] + 1;
                                if (ssv) sum += lp[w + x] + lp[w + x + 1] + 1;
                                c[x >> 1] = (uint8_t)((sum - s) >> (1 + ssv));
                            }
                            lp += w << ssv;
                            c += w >> 1;
                        }
                    }
            }
        }
        // inter-intra masks (dav1d_init_interintra_masks)
        static const uint8_t w1d[32] = {60, 52, 45, 39, 34, 30, 26, 22, 19, 17, 15, 13, 11, 10, 8, 7,
                                        6,  6,  5,  4,  4,  3,  3,  2,  2,  2,  2,  1,  1,  1,  1, 1};
        uint8_t *dc = alloc(32 * 32);
        memset(dc, 32, 32 * 32);
        struct Nd { int w, h, step; const uint8_t *m[3]; };
        Nd nd[9] = {{32, 32, 1, {}}, {16, 32, 1, {}}, {16, 16, 2, {}}, {8, 32, 1, {}}, {8, 16, 2, {}},
                    {8, 8, 4, {}},   {4, 16, 2, {}},  {4, 8, 4, {}},   {4, 4, 8, {}}};
        for (Nd &d : nd) {
            uint8_t *v = alloc((size_t)3 * d.w * d.h), *hz = v + d.w * d.h, *sm = hz + d.w * d.h;
            for (int y = 0; y < d.h; y++) {
                memset(v + y * d.w, w1d[y * d.step], d.w);
                for (int x = 0; x < d.w; x++) {
                    sm[y * d.w + x] = w1d[imin(x, y) * d.step];
                    hz[y * d.w + x] = w1d[x * d.step];
                }
            }
            d.m[0] = v;
            d.m[1] = hz;
            d.m[2] = sm;
        }
        auto find = [&](int w, int hh) -> const Nd & {
            for (const Nd &d : nd)
                if (d.w == w && d.h == hh) return d;
            return nd[0];
        };
        struct IiSet { int bs; int sz[3][2]; };
        static const IiSet sets[7] = {
            {BS_8x8, {{8, 8}, {4, 8}, {4, 4}}},        {BS_8x16, {{8, 16}, {4, 16}, {4, 8}}},
            {BS_16x8, {{16, 16}, {8, 8}, {8, 8}}},     {BS_16x16, {{16, 16}, {8, 16}, {8, 8}}},
            {BS_16x32, {{16, 32}, {8, 32}, {8, 16}}},  {BS_32x16, {{32, 32}, {16, 16}, {16, 16}}},
            {BS_32x32, {{32, 32}, {16, 32}, {16, 16}}},
        };
        for (const IiSet &st : sets)
            for (int c = 0; c < 3; c++) {
                const Nd &d = find(st.sz[c][0], st.sz[c][1]);
                ii[st.bs][c][0] = dc;
                ii[st.bs][c][1] = d.m[0];
                ii[st.bs][c][2] = d.m[1];
                ii[st.bs][c][3] = d.m[2];
            }
    }
};

const MaskTables &tables() {
    static const MaskTables t;
    return t;
}

}  // namespace

const uint8_t *wedge_mask(int bs, int cls, int sign, int idx) { return tables().wedge[bs][cls][sign][idx]; }
const uint8_t *ii_mask(int bs, int cls, int mode) { return tables().ii[bs][cls][mode]; }

// ---- warpmv.rs (C warpmv.c) ----------------------------------------------------------------

static const uint16_t k_div_lut[257] = {
    16384, 16320, 16257, 16194, 16132, 16070, 16009, 15948, 15888, 15828, 15768, 15709, 15650, 15592, 15534, 15477,
    15420, 15364, 15308, 15252, 15197, 15142, 15087, 15033, 14980, 14926, 14873, 14821, 14769, 14717, 14665, 14614,
    14564, 14513, 14463, 14413, 14364, 14315, 14266, 14218, 14170, 14122, 14075, 14028, 13981, 13935, 13888, 13843,
    13797, 13752, 13707, 13662, 13618, 13574, 13530, 13487, 13443, 13400, 13358, 13315, 13273, 13231, 13190, 13148,
    13107, 13066, 13026, 12985, 12945, 12906, 12866, 12827, 12788, 12749, 12710, 12672, 12633, 12596, 12558, 12520,
    12483, 12446, 12409, 12373, 12336, 12300, 12264, 12228, 12193, 12157, 12122, 12087, 12053, 12018, 11984, 11950,
    11916, 11882, 11848, 11815, 11782, 11749, 11716, 11683, 11651, 11619, 11586, 11555, 11523, 11491, 11460, 11429,
    11398, 11367, 11336, 11305, 11275, 11245, 11215, 11185, 11155, 11125, 11096, 11067, 11038, 11009, 10980, 10951,
    10923, 10894, 10866, 10838, 10810, 10782, 10755, 10727, 10700, 10673, 10645, 10618, 10592, 10565, 10538, 10512,
    10486, 10460, 10434, 10408, 10382, 10356, 10331, 10305, 10280, 10255, 10230, 10205, 10180, 10156, 10131, 10107,
    10082, 10058, 10034, 10010, 9986,  9963,  9939,  9916,  9892,  9869,  9846,  9823,  9800,  9777,  9754,  9732,
    9709,  9687,  9664,  9642,  9620,  9598,  9576,  9554,  9533,  9511,  9489,  9468,  9447,  9425,  9404,  9383,
    9362,  9341,  9321,  9300,  9279,  9259,  9239,  9218,  9198,  9178,  9158,  9138,  9118,  9098,  9079,  9059,
    9039,  9020,  9001,  8981,  8962,  8943,  8924,  8905,  8886,  8867,  8849,  8830,  8812,  8793,  8775,  8756,
    8738,  8720,  8702,  8684,  8666,  8648,  8630,  8613,  8595,  8577,  8560,  8542,  8525,  8508,  8490,  8473,
    8456,  8439,  8422,  8405,  8389,  8372,  8355,  8339,  8322,  8306,  8289,  8273,  8257,  8240,  8224,  8208,
    8192,
};

static inline int apply_sign(int v, int s) { return s < 0 ? -v : v; }
static inline int apply_sign64(int v, int64_t s) { return s < 0 ? -v : v; }

static int clip_wmp(int v) {
    const int cv = iclip(v, INT16_MIN, INT16_MAX);
    return apply_sign((std::abs(cv) + 32) >> 6, cv) * (1 << 6);
}

static int div32(unsigned d, int *shift) {
    *shift = ulog2(d);
    const int e = (int)(d - (1u << *shift));
    const int f = *shift > 8 ? (e + (1 << (*shift - 9))) >> (*shift - 8) : e << (8 - *shift);
    *shift += 14;
    return k_div_lut[f];
}

static int div64(uint64_t d, int *shift) {
    *shift = 63 - __builtin_clzll(d);
    const int64_t e = (int64_t)(d - (1ULL << *shift));
    const int64_t f = *shift > 8 ? (e + (1LL << (*shift - 9))) >> (*shift - 8) : e << (8 - *shift);
    *shift += 14;
    return k_div_lut[f];
}

int get_shear_params(WarpParams &wm) {
    const int32_t *mat = wm.matrix;
    if (mat[2] <= 0) return 1;
    wm.abcd[0] = (int16_t)clip_wmp(mat[2] - 0x10000);
    wm.abcd[1] = (int16_t)clip_wmp(mat[3]);
    int shift;
    const int y = apply_sign(div32((unsigned)std::abs(mat[2]), &shift), mat[2]);
    const int64_t v1 = ((int64_t)mat[4] * 0x10000) * y;
    const int rnd = (1 << shift) >> 1;
    wm.abcd[2] = (int16_t)clip_wmp(apply_sign64((int)((llabs(v1) + rnd) >> shift), v1));
    const int64_t v2 = ((int64_t)mat[3] * mat[4]) * y;
    wm.abcd[3] = (int16_t)clip_wmp(mat[5] - apply_sign64((int)((llabs(v2) + rnd) >> shift), v2) - 0x10000);
    return (4 * std::abs(wm.abcd[0]) + 7 * std::abs(wm.abcd[1]) >= 0x10000) ||
           (4 * std::abs(wm.abcd[2]) + 4 * std::abs(wm.abcd[3]) >= 0x10000);
}

static int mult_shift(int64_t px, int idet, int shift, int lo, int hi) {
    const int64_t v1 = px * idet;
    const int v2 = apply_sign64((int)((llabs(v1) + ((1LL << shift) >> 1)) >> shift), v1);
    return iclip(v2, lo, hi);
}

void set_affine_mv2d(int bw4, int bh4, Mv mv, WarpParams &wm, int bx4, int by4) {
    int32_t *mat = wm.matrix;
    const int rsuy = 2 * bh4 - 1, rsux = 2 * bw4 - 1;
    const int isuy = by4 * 4 + rsuy, isux = bx4 * 4 + rsux;
    mat[0] = iclip(mv.x * 0x2000 - (isux * (mat[2] - 0x10000) + isuy * mat[3]), -0x800000, 0x7fffff);
    mat[1] = iclip(mv.y * 0x2000 - (isux * mat[4] + isuy * (mat[5] - 0x10000)), -0x800000, 0x7fffff);
}

int find_affine_int(const int (*pts)[2][2], int np, int bw4, int bh4, Mv mv, WarpParams &wm, int bx4, int by4) {
    int32_t *mat = wm.matrix;
    int a00 = 0, a01 = 0, a11 = 0, bx0 = 0, bx1 = 0, by0 = 0, by1 = 0;
    const int rsuy = 2 * bh4 - 1, rsux = 2 * bw4 - 1;
    const int suy = rsuy * 8, sux = rsux * 8;
    const int duy = suy + mv.y, dux = sux + mv.x;
    for (int i = 0; i < np; i++) {
        const int dx = pts[i][1][0] - dux, dy = pts[i][1][1] - duy;
        const int sx = pts[i][0][0] - sux, sy = pts[i][0][1] - suy;
        if (std::abs(sx - dx) < 256 && std::abs(sy - dy) < 256) {
            a00 += ((sx * sx) >> 2) + sx * 2 + 8;
            a01 += ((sx * sy) >> 2) + sx + sy + 4;
            a11 += ((sy * sy) >> 2) + sy * 2 + 8;
            bx0 += ((sx * dx) >> 2) + sx + dx + 8;
            bx1 += ((sy * dx) >> 2) + sy + dx + 4;
            by0 += ((sx * dy) >> 2) + sx + dy + 4;
            by1 += ((sy * dy) >> 2) + sy + dy + 8;
        }
    }
    const int64_t det = (int64_t)a00 * a11 - (int64_t)a01 * a01;
    if (det == 0) return 1;
    int shift, idet = apply_sign64(div64((uint64_t)llabs(det), &shift), det);
    shift -= 16;
    if (shift < 0) {
        idet <<= -shift;
        shift = 0;
    }
    mat[2] = mult_shift((int64_t)a11 * bx0 - (int64_t)a01 * bx1, idet, shift, 0xe001, 0x11fff);
    mat[3] = mult_shift((int64_t)a00 * bx1 - (int64_t)a01 * bx0, idet, shift, -0x1fff, 0x1fff);
    mat[4] = mult_shift((int64_t)a11 * by0 - (int64_t)a01 * by1, idet, shift, -0x1fff, 0x1fff);
    mat[5] = mult_shift((int64_t)a00 * by1 - (int64_t)a01 * by0, idet, shift, 0xe001, 0x11fff);
    const int isuy = by4 * 4 + rsuy, isux = bx4 * 4 + rsux;
    mat[0] = iclip(mv.x * 0x2000 - (isux * (mat[2] - 0x10000) + isuy * mat[3]), -0x800000, 0x7fffff);
    mat[1] = iclip(mv.y * 0x2000 - (isux * mat[4] + isuy * (mat[5] - 0x10000)), -0x800000, 0x7fffff);
    return 0;
}

}  // namespace fd
}  // namespace av1
