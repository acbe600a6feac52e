// recon_inter.cpp — recon_b_inter (recon.rs:3162-4045; C recon_tmpl.c:1605-2051) of the
// front-end: instead of predicting and reconstructing one block, it emits the block's work as
// descriptors for the device (and, in tests, for the oracle's frame driver):
//  * mc() calls (recon.rs:2025-2203) -> MiMcBlock units: single puts, whole compounds (avg,
//    w_avg, mask with a wedge copy, w_mask writing the segmentation mask the chroma units read),
//    the neighbour-MV units of sub-8x8 chroma (recon.rs:3552-3694) and MI_MC_PREP sides;
//  * obmc() (recon.rs:2205-2309) -> MI_MC_OBMC_H / _V laps (a lap whose reference is scaled goes
//    through the scaled-reference path, see mi_frame_run);
//  * warp_affine() (recon.rs:2311-2400) -> MiWarpBlock per 8x8 (into the picture, or warp8x8t into
//    the tmp arena for a compound side);
//  * mc() with a scaled reference -> units of FrameWork::scaled;
//  * a compound with a warped or scaled side -> prep sides + MiMcCombine;
//  * the inter-intra blend (recon.rs:3524-3543, 3822-3833) -> an MI_INTRA_II item of the intra
//    path (its edges may read intra neighbours), whose residual follows as MI_INTRA_RESID items;
//  * read_coef_tree / the chroma loop (recon.rs:1597-1800, 3940-4045) -> MiTxBlocks.
#include <cstring>

#include "framedec.h"

namespace av1 {
namespace fd {

uint32_t FrameDec::add_mask(const uint8_t *m, int n) {
    const uint32_t off = (uint32_t)fw.masks.size();
    if (m) fw.masks.insert(fw.masks.end(), m, m + n);
    else fw.masks.resize(fw.masks.size() + n, 0);
    return off;
}

static MiMcBlock mc_unit(int plane, int x, int y, int w, int hh, int filter2d, Mv mv0, int ref0) {
    MiMcBlock u{};
    u.x = (uint16_t)x;
    u.y = (uint16_t)y;
    u.w = (uint8_t)w;
    u.h = (uint8_t)hh;
    u.plane = (uint8_t)plane;
    u.filter2d = (uint8_t)filter2d;
    u.mvx[0] = mv0.x;
    u.mvy[0] = mv0.y;
    u.ref[0] = (int8_t)ref0;
    u.ref[1] = -1;
    return u;
}

static int pow2ceil(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

// warp_affine (C recon_tmpl.c:1139-1198): the arguments of every 8x8's warp8x8 / warp8x8t call
void FrameDec::push_warp(const Block &b, int plane, const WarpParams &wm, int ref, int prep, uint32_t tmp_off) {
    const int sh = plane ? ss_hor : 0, sv = plane ? ss_ver : 0;
    const BlockDim &bd = k_bdim[b.bs];
    const int pw = bd.w4 * (4 >> sh), ph = bd.h4 * (4 >> sv);
    const int32_t *mat = wm.matrix;
    for (int y = 0; y < ph; y += 8) {
        const int src_y = by * 4 + ((y + 4) << sv);
        const int64_t mat3_y = (int64_t)mat[3] * src_y + mat[0];
        const int64_t mat5_y = (int64_t)mat[5] * src_y + mat[1];
        for (int x = 0; x < pw; x += 8) {
            const int src_x = bx * 4 + ((x + 4) << sh);
            const int64_t mvx = ((int64_t)mat[2] * src_x + mat3_y) >> sh;
            const int64_t mvy = ((int64_t)mat[4] * src_x + mat5_y) >> sv;
            MiWarpBlock w{};
            w.x = (uint16_t)(((bx * 4) >> sh) + x);
            w.y = (uint16_t)(((by * 4) >> sv) + y);
            w.plane = (uint8_t)plane;
            w.ref = (int8_t)ref;
            w.prep = (uint8_t)prep;
            w.dx = (int32_t)(mvx >> 16) - 4;
            w.mx = (((int)mvx & 0xffff) - wm.abcd[0] * 4 - wm.abcd[1] * 7) & ~0x3f;
            w.dy = (int32_t)(mvy >> 16) - 4;
            w.my = (((int)mvy & 0xffff) - wm.abcd[2] * 4 - wm.abcd[3] * 4) & ~0x3f;
            for (int k = 0; k < 4; k++) w.abcd[k] = wm.abcd[k];
            if (prep) {
                w.tmp_off = tmp_off + (uint32_t)(y * pw + x);
                w.tmp_stride = (uint16_t)pw;
            }
            fw.warp.push_back(w);
        }
    }
}

// obmc (C recon_tmpl.c:1076-1137): the laps of the above and left neighbours with their own MV,
// reference and filter, in every plane of the block
int FrameDec::push_obmc(const Block &b, int bw4, int bh4, int w4b, int h4b) {
    const BlockDim &bd = k_bdim[b.bs];
    const int has_chroma = layout != 0 && (bw4 > ss_hor || (bx & 1)) && (bh4 > ss_ver || (by & 1));
    for (int pl = 0; pl < (has_chroma ? 3 : 1); pl++) {
        const int sh = pl ? ss_hor : 0, sv = pl ? ss_ver : 0;
        const int h_mul = 4 >> sh, v_mul = 4 >> sv;
        if (by > ts->row_start && (!pl || bw4 * h_mul + bh4 * v_mul >= 16)) {
            for (int i = 0, x = 0; x < w4b && i < imin(bd.lw4, 4);) {
                const RefMvBlock &ar = rmv_at(by - 1, bx + x + 1);
                const int step4 = iclip(k_bdim[ar.bs].w4, 2, 16);
                if (ar.ref[0] > 0) {
                    const int ow4 = imin(step4, bw4), oh4 = imin(bh4, 16) >> 1;
                    const int rows = ((oh4 * 3 + 3) >> 2) * v_mul;
                    MiMcBlock u = mc_unit(pl, (bx + x) * h_mul, by * v_mul, ow4 * h_mul, imax(2, pow2ceil(rows)),
                                          f2d_at(by - 1, bx + x + 1), ar.mv[0], ar.ref[0] - 1);
                    u.comp = MI_MC_OBMC_H;
                    u.param = (uint8_t)(oh4 * v_mul);
                    fw.obmc_h.push_back(u);
                    i++;
                }
                x += step4;
            }
        }
        if (bx > ts->col_start) {
            for (int i = 0, y = 0; y < h4b && i < imin(bd.lh4, 4);) {
                const RefMvBlock &lr = rmv_at(by + y + 1, bx - 1);
                const int step4 = iclip(k_bdim[lr.bs].h4, 2, 16);
                if (lr.ref[0] > 0) {
                    const int ow4 = imin(bw4, 16) >> 1, oh4 = imin(step4, bh4);
                    MiMcBlock u = mc_unit(pl, bx * h_mul, (by + y) * v_mul, ow4 * h_mul, oh4 * v_mul,
                                          f2d_at(by + y + 1, bx - 1), lr.mv[0], lr.ref[0] - 1);
                    u.comp = MI_MC_OBMC_V;
                    fw.obmc_v.push_back(u);
                    i++;
                }
                y += step4;
            }
        }
    }
    return 0;
}

int FrameDec::emit_inter_pred(const Block &b, int has_chroma) {
    const BlockDim &bd = k_bdim[b.bs];
    const int bw4 = bd.w4, bh4 = bd.h4;
    const int w4b = imin(bw4, bw - bx), h4b = imin(bh4, bh - by);
    const int cbw4 = (bw4 + ss_hor) >> ss_hor, cbh4 = (bh4 + ss_ver) >> ss_ver;
    const int cls = layout == 0 ? 0 : 3 - layout;          // chr_layout_idx: 0 444, 1 422, 2 420
    auto scaled = [&](int r) { return svc_scale[r][0] != 0 || svc_scale[r][1] != 0; };
    // a unit of one reference: the main list, or the scaled-reference list
    auto put = [&](MiMcBlock u) {
        if (scaled(u.ref[0])) fw.scaled.push_back(u);
        else fw.mc.push_back(u);
    };

    if (b.comp_type == COMP_NONE) {
        const int r = b.ref[0];
        const bool warp = (b.inter_mode == GLOBALMV && gmv_warp_allowed[r]) ||
                          (b.motion_mode == MM_WARP && warpmv.type > WM_TRANSLATION);
        const WarpParams &wp = b.motion_mode == MM_WARP ? warpmv : gmv[r];
        // luma
        if (imin(bw4, bh4) > 1 && warp) {
            push_warp(b, 0, wp, r, 0, 0);
        } else {
            put(mc_unit(0, bx * 4, by * 4, bw4 * 4, bh4 * 4, b.filter2d, b.mv[0], r));
        }
        if (has_chroma) {
            // sub-8x8 chroma: each 4x4 luma block's chroma quadrant predicted with its own MV
            int sub8 = bw4 == ss_hor || bh4 == ss_ver;
            if (sub8) {
                if (bw4 == 1) sub8 &= rmv_at(by, bx - 1).ref[0] > 0;
                if (bh4 == ss_ver) sub8 &= rmv_at(by - 1, bx).ref[0] > 0;
                if (bw4 == 1 && bh4 == ss_ver) sub8 &= rmv_at(by - 1, bx - 1).ref[0] > 0;
            }
            const int h_mul = 4 >> ss_hor, v_mul = 4 >> ss_ver;
            if (sub8) {
                auto nb = [&](int y4, int x4) {
                    const RefMvBlock &nr = rmv_at(y4, x4);
                    for (int pl = 1; pl <= 2; pl++)
                        put(mc_unit(pl, x4 * h_mul, y4 * v_mul, bw4 * h_mul, bh4 * v_mul, f2d_at(y4, x4), nr.mv[0],
                                    nr.ref[0] - 1));
                };
                if (bw4 == 1 && bh4 == ss_ver) nb(by - 1, bx - 1);
                if (bw4 == 1) nb(by, bx - 1);
                if (bh4 == ss_ver) nb(by - 1, bx);
                for (int pl = 1; pl <= 2; pl++)
                    put(mc_unit(pl, bx * h_mul, by * v_mul, bw4 * h_mul, bh4 * v_mul, b.filter2d, b.mv[0], r));
            } else if (imin(cbw4, cbh4) > 1 && warp) {
                for (int pl = 1; pl <= 2; pl++) push_warp(b, pl, wp, r, 0, 0);
            } else {
                const int cx = (bx & ~ss_hor) * h_mul, cy = (by & ~ss_ver) * v_mul;
                const int cw = (bw4 << (bw4 == ss_hor)) * h_mul, ch = (bh4 << (bh4 == ss_ver)) * v_mul;
                for (int pl = 1; pl <= 2; pl++) put(mc_unit(pl, cx, cy, cw, ch, b.filter2d, b.mv[0], r));
            }
        }
        if (b.motion_mode == MM_OBMC) return push_obmc(b, bw4, bh4, w4b, h4b);
        return 0;
    }

    // compound: both sides predicted into intermediates and combined
    const int bdw = bw4 * 4, bdh = bh4 * 4;
    uint32_t mask_y = 0, mask_uv = 0;
    int param = 0;
    const int sign = b.mask_sign;
    switch (b.comp_type) {
    case COMP_WAVG: param = jnt_weights[b.ref[0]][b.ref[1]]; break;
    case COMP_SEG:
        param = sign << 7;
        // w_mask writes the mask at the chroma resolution of the layout (I400 / I444: full)
        mask_y = mask_uv = add_mask(nullptr, (bdw >> (layout ? ss_hor : 0)) * (bdh >> (layout ? ss_ver : 0)));
        break;
    case COMP_WEDGE:
        param = sign << 7;
        mask_y = add_mask(wedge_mask(b.bs, 0, 0, b.wedge_idx), bdw * bdh);
        if (has_chroma) mask_uv = add_mask(wedge_mask(b.bs, cls, sign, b.wedge_idx), (bdw >> ss_hor) * (bdh >> ss_ver));
        break;
    default: break;
    }
    const int comp_y = b.comp_type == COMP_AVG ? MI_MC_AVG : b.comp_type == COMP_WAVG ? MI_MC_WAVG :
                       b.comp_type == COMP_SEG ? MI_MC_SEG : MI_MC_MASK;
    const int comp_uv = b.comp_type == COMP_SEG ? MI_MC_MASK : comp_y;
    bool warp_side[2], combine = false;
    for (int i = 0; i < 2; i++) {
        warp_side[i] = b.inter_mode == GLOBALMV_GLOBALMV && gmv_warp_allowed[b.ref[i]];
        combine |= warp_side[i] || scaled(b.ref[i]);
    }
    for (int pl = 0; pl < (has_chroma ? 3 : 1); pl++) {
        const int sh = pl ? ss_hor : 0, sv = pl ? ss_ver : 0;
        const int x = (bx * 4) >> sh, y = (by * 4) >> sv, w = bdw >> sh, hh = bdh >> sv;
        const int comp = pl ? comp_uv : comp_y;
        const uint32_t moff = pl ? mask_uv : mask_y;
        if (!combine) {
            MiMcBlock u = mc_unit(pl, x, y, w, hh, b.filter2d, b.mv[0], b.ref[0]);
            u.mvx[1] = b.mv[1].x;
            u.mvy[1] = b.mv[1].y;
            u.ref[1] = (int8_t)b.ref[1];
            u.comp = (uint8_t)comp;
            u.param = (uint8_t)param;
            u.mask_off = moff;
            fw.mc.push_back(u);
            continue;
        }
        MiMcCombine c{};
        c.x = (uint16_t)x;
        c.y = (uint16_t)y;
        c.w = (uint8_t)w;
        c.h = (uint8_t)hh;
        c.plane = (uint8_t)pl;
        c.comp = (uint8_t)comp;
        c.param = (uint8_t)param;
        c.mask_off = moff;
        for (int i = 0; i < 2; i++) {
            const uint32_t toff = (uint32_t)fw.ntmp;
            fw.ntmp += (size_t)w * hh;
            c.tmp_off[i] = toff;
            if (warp_side[i] && (!pl || imin(cbw4, cbh4) > 1)) {
                push_warp(b, pl, gmv[b.ref[i]], b.ref[i], 1, toff);
            } else {
                MiMcBlock u = mc_unit(pl, x, y, w, hh, b.filter2d, b.mv[i], b.ref[i]);
                u.comp = MI_MC_PREP;
                u.mask_off = toff;
                put(u);
            }
        }
        (pl ? fw.combine_uv : fw.combine_y).push_back(c);
    }
    return 0;
}

// The inter-intra blend of a single-reference block: the intra prediction of the whole block
// from its (final) neighbours blended into the inter prediction (C recon_tmpl.c:1665-1692,
// 1790-1831), one MI_INTRA_II item per plane with the mask copied into the idx arena
void FrameDec::emit_interintra(const Block &b, int has_chroma) {
    const BlockDim &bd = k_bdim[b.bs];
    const int cls = layout == 0 ? 0 : 3 - layout;
    const int mode = b.interintra_mode == 3 ? SMOOTH_PRED : b.interintra_mode;
    for (int pl = 0; pl < (has_chroma ? 3 : 1); pl++) {
        const int sh = pl ? ss_hor : 0, sv = pl ? ss_ver : 0;
        const int w = pl ? ((bd.w4 + ss_hor) >> ss_hor) * 4 : bd.w4 * 4;
        const int hh = pl ? ((bd.h4 + ss_ver) >> ss_ver) * 4 : bd.h4 * 4;
        MiIntraBlock ib{};
        ib.x = (uint16_t)((bx >> sh) * 4);
        ib.y = (uint16_t)((by >> sv) * 4);
        ib.w = (uint8_t)w;
        ib.h = (uint8_t)hh;
        ib.plane = (uint8_t)pl;
        ib.mode = (uint8_t)mode;
        ib.tile_w = (uint16_t)((ts->col_end >> sh) * 4);
        ib.tile_h = (uint16_t)((ts->row_end >> sv) * 4);
        const int have_left = (bx >> sh) > (ts->col_start >> sh), have_top = (by >> sv) > (ts->row_start >> sv);
        ib.flags = (uint8_t)((have_left ? MI_INTRA_HAVE_LEFT : 0) | (have_top ? MI_INTRA_HAVE_TOP : 0) | MI_INTRA_II);
        const uint8_t *mk = b.interintra_type == II_BLEND ? ii_mask(b.bs, pl ? cls : 0, b.interintra_mode)
                                                          : wedge_mask(b.bs, pl ? cls : 0, 0, b.wedge_idx);
        ib.aux_off = (uint32_t)fw.idx.size();
        fw.idx.insert(fw.idx.end(), mk, mk + w * hh);
        // dependencies: the left column, the top row and the corner
        std::vector<int32_t> &deps = dep_tmp;
        deps.clear();
        const int x = ib.x, y = ib.y;
        if (have_left) add_deps(pl, x - 1, y, x, imin(y + hh, ib.tile_h), deps);
        if (have_top) add_deps(pl, x - 1, y - 1, imin(x + w, ib.tile_w), y, deps);
        const int k = (int)fw.intra.size();
        fw.intra.push_back(ib);
        fw.dep_start.push_back((int32_t)fw.deps.size());
        for (int32_t d : deps) fw.deps.push_back(d);
        MiTxBlock tb{};
        tb.x = ib.x;
        tb.y = ib.y;
        tb.plane = (uint8_t)pl;
        for (int t = 0; t < N_TX; t++)
            if (k_txdim[t].w * 4 == w && k_txdim[t].h * 4 == hh) tb.tx = (uint8_t)t;
        tb.eob = -1;
        fw.intra_tx.push_back(tb);
        Span<int32_t> &o = owner[pl];
        for (int yy = y >> 2; yy < (y + hh) >> 2; yy++)
            for (int xx = x >> 2; xx < (x + w) >> 2; xx++) {
                const size_t q = (size_t)yy * owner_stride + xx;
                if (xx < owner_stride && q < o.size()) o[q] = k;
            }
    }
}

// The residual of an inter block (read_coef_tree's leaves, then the chroma transforms): one
// MiTxBlock per coded transform block, in the reference's coefficient order. Inter-intra blocks
// put theirs on the intra path (MI_INTRA_RESID after the blend).
void FrameDec::emit_inter_residual(const Block &b, int has_chroma) {
    const BlockDim &bd = k_bdim[b.bs];
    const int bw4 = bd.w4, bh4 = bd.h4;
    const int bx4 = bx & 31, by4 = by & 31;
    const int cbw4 = (bw4 + ss_hor) >> ss_hor, cbh4 = (bh4 + ss_ver) >> ss_ver;
    const bool ii = b.interintra_type != II_NONE;
    if (ii) emit_interintra(b, has_chroma);
    if (b.skip) {
        setn(a.lcoef, bx, bw4, 0x40);
        setn(l.lcoef, by4, bh4, 0x40);
        if (has_chroma)
            for (int pl = 0; pl < 2; pl++) {
                setn(a.ccoef[pl], bx >> ss_hor, cbw4, 0x40);
                setn(l.ccoef[pl], by4 >> ss_ver, cbh4, 0x40);
            }
        return;
    }
    const int w4b = imin(bw4, bw - bx), h4b = imin(bh4, bh - by);
    const int cw4 = (w4b + ss_hor) >> ss_hor, ch4 = (h4b + ss_ver) >> ss_ver;
    const TxDim &yt = k_txdim[b.max_ytx], &ut = k_txdim[b.uvtx];
    uint8_t txtp_map[32][32];
    int32_t cf[32 * 32];

    auto emit = [&](int plane, int tx, int px, int py, int eob, int txtp) {
        if (eob < 0) return;
        MiTxBlock tb{};
        tb.x = (uint16_t)px;
        tb.y = (uint16_t)py;
        tb.plane = (uint8_t)plane;
        tb.tx = (uint8_t)tx;
        tb.txtp = (uint8_t)txtp;
        tb.eob = eob;
        tb.coef_off = store_coefs(cf, tx, txtp, eob, &tb.flags);
        if (!ii) {
            fw.inter_tx.push_back(tb);
            return;
        }
        MiIntraBlock ib{};
        ib.x = tb.x;
        ib.y = tb.y;
        ib.w = (uint8_t)(k_txdim[tx].w * 4);
        ib.h = (uint8_t)(k_txdim[tx].h * 4);
        ib.plane = (uint8_t)plane;
        ib.mode = MI_INTRA_RESID;
        std::vector<int32_t> &deps = dep_tmp;
        deps.clear();
        add_deps(plane, px, py, px + ib.w, py + ib.h, deps);
        const int k = (int)fw.intra.size();
        fw.intra.push_back(ib);
        fw.dep_start.push_back((int32_t)fw.deps.size());
        for (int32_t d : deps) fw.deps.push_back(d);
        fw.intra_tx.push_back(tb);
        Span<int32_t> &o = owner[plane];
        for (int yy = py >> 2; yy < (py + ib.h) >> 2; yy++)
            for (int xx = px >> 2; xx < (px + ib.w) >> 2; xx++) {
                const size_t q = (size_t)yy * owner_stride + xx;
                if (xx < owner_stride && q < o.size()) o[q] = k;
            }
    };
    // read_coef_tree: the var-tx leaves of one max-size transform, luma
    auto tree = [&](auto &&self, int tx, int depth, int x_off, int y_off, int tbx, int tby) -> void {
        const TxDim &t = k_txdim[tx];
        if (depth < 2 && b.tx_split[depth] && (b.tx_split[depth] & (1 << (y_off * 4 + x_off)))) {
            const int sub = t.sub, sw = k_txdim[sub].w, sh = k_txdim[sub].h;
            self(self, sub, depth + 1, x_off * 2, y_off * 2, tbx, tby);
            if (t.w >= t.h && tbx + sw < bw) self(self, sub, depth + 1, x_off * 2 + 1, y_off * 2, tbx + sw, tby);
            if (t.h >= t.w && tby + sh < bh) {
                self(self, sub, depth + 1, x_off * 2, y_off * 2 + 1, tbx, tby + sh);
                if (t.w >= t.h && tbx + sw < bw)
                    self(self, sub, depth + 1, x_off * 2 + 1, y_off * 2 + 1, tbx + sw, tby + sh);
            }
            return;
        }
        const int tby4 = tby & 31, tbx4 = tbx & 31;
        int txtp = 0;
        uint8_t res;
        memset(cf, 0, sizeof(int32_t) * imin(t.w * 4, 32) * imin(t.h * 4, 32));
        const int eob = decode_coefs(&a.lcoef[tbx], &l.lcoef[tby4], tx, b.bs, b, 0, 0, cf, &txtp, &res);
        memset(&a.lcoef[tbx], res, imin(t.w, bw - tbx));
        memset(&l.lcoef[tby4], res, imin(t.h, bh - tby));
        for (int y = 0; y < t.h && tby4 + y < 32; y++)
            for (int x = 0; x < t.w && tbx4 + x < 32; x++) txtp_map[tby4 + y][tbx4 + x] = (uint8_t)txtp;
        emit(0, tx, tbx * 4, tby * 4, eob, txtp);
    };
    for (int init_y = 0; init_y < h4b; init_y += 16) {
        for (int init_x = 0; init_x < w4b; init_x += 16) {
            int y_off = init_y != 0;
            for (int y = init_y; y < imin(h4b, init_y + 16); y += yt.h, y_off++) {
                int x_off = init_x != 0;
                for (int x = init_x; x < imin(w4b, init_x + 16); x += yt.w, x_off++)
                    tree(tree, b.max_ytx, 0, x_off, y_off, bx + x, by + y);
            }
            if (!has_chroma) continue;
            for (int pl = 0; pl < 2; pl++)
                for (int y = init_y >> ss_ver; y < imin(ch4, (init_y + 16) >> ss_ver); y += ut.h)
                    for (int x = init_x >> ss_hor; x < imin(cw4, (init_x + 16) >> ss_hor); x += ut.w) {
                        const int tby = by + (y << ss_ver), tbx = bx + (x << ss_hor);
                        int txtp = txtp_map[by4 + (y << ss_ver)][bx4 + (x << ss_hor)];
                        uint8_t res;
                        memset(cf, 0, sizeof(int32_t) * imin(ut.w * 4, 32) * imin(ut.h * 4, 32));
                        const int cx = (bx >> ss_hor) + x, cy4 = (by4 >> ss_ver) + y;
                        const int eob = decode_coefs(&a.ccoef[pl][cx], &l.ccoef[pl][cy4], b.uvtx, b.bs, b, 0, 1 + pl,
                                                     cf, &txtp, &res);
                        memset(&a.ccoef[pl][cx], res, imin(ut.w, (bw - tbx + ss_hor) >> ss_hor));
                        memset(&l.ccoef[pl][cy4], res, imin(ut.h, (bh - tby + ss_ver) >> ss_ver));
                        emit(1 + pl, b.uvtx, cx * 4, ((by >> ss_ver) + y) * 4, eob, txtp);
                    }
        }
    }
}

}  // namespace fd
}  // namespace av1
