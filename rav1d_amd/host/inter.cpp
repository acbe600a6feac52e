// inter.cpp — inter blocks of the front-end: decode_b's inter branch (decode.rs:1131-2003, C
// decode.c:1427-1981: compound / reference / mode / DRL / MV / inter-intra / motion-mode /
// filter syntax, warp derivation), the inter loop-filter masks (lf_mask.rs:486; C
// lf_mask.c:39-148, 346-406), and recon_b_inter (recon.rs:3162-4045; C recon_tmpl.c:1605-2051)
// turned into descriptors: MiMcBlock units (put, compound, OBMC laps, sub-8x8 chroma),
// MiWarpBlock 8x8s, scaled-reference units and MiMcCombine compounds for the MC kernels, the
// inter-intra blend as MI_INTRA_II work of the persistent intra kernel, and the residuals as
// MiTxBlocks. No pixels are produced here.
#include <cstdlib>
#include <cstring>

#include "framedec.h"

namespace av1 {
namespace fd {

static const unsigned kWedgeAllowed = (1u << BS_32x32) | (1u << BS_32x16) | (1u << BS_32x8) | (1u << BS_16x32) |
                                      (1u << BS_16x16) | (1u << BS_16x8) | (1u << BS_8x32) | (1u << BS_8x16) |
                                      (1u << BS_8x8);
static const unsigned kInterIntraAllowed = (1u << BS_32x32) | (1u << BS_32x16) | (1u << BS_16x32) |
                                           (1u << BS_16x16) | (1u << BS_16x8) | (1u << BS_8x16) | (1u << BS_8x8);

static int poc_diff(int nbits, int poc0, int poc1) {
    if (!nbits) return 0;
    const int mask = 1 << (nbits - 1);
    const int diff = poc0 - poc1;
    return (diff & (mask - 1)) - (diff & mask);
}

// decode.rs decode_frame_init / submit_frame (C decode.c:3102-3137, 3505-3524): scaled-reference
// steps, which global motions are warps, compound distance weights
void FrameDec::inter_frame_init() {
    for (int i = 0; i < 7; i++) {
        gmv[i] = h.gmv[i];
        const RefSlot *r = in_.refs[i];
        const int rw = r->hdr->width[1], rh = r->hdr->height;
        if (rw != h.width[0] || rh != h.height) {
            svc_scale[i][0] = ((rw << 14) + (h.width[0] >> 1)) / h.width[0];
            svc_scale[i][1] = ((rh << 14) + (h.height >> 1)) / h.height;
            svc_step[i][0] = (svc_scale[i][0] + 8) >> 4;
            svc_step[i][1] = (svc_scale[i][1] + 8) >> 4;
        } else {
            svc_scale[i][0] = svc_scale[i][1] = svc_step[i][0] = svc_step[i][1] = 0;
        }
        gmv_warp_allowed[i] =
            gmv[i].type > WM_TRANSLATION && !h.force_integer_mv && !get_shear_params(gmv[i]) && !svc_scale[i][0];
    }
    if (h.switchable_comp_refs) {
        const int nbits = s.order_hint_n_bits;
        for (int i = 0; i < 7; i++) {
            const int p0 = in_.refs[i]->hdr->frame_offset;
            for (int j = i + 1; j < 7; j++) {
                const int p1 = in_.refs[j]->hdr->frame_offset;
                const unsigned d1 = (unsigned)imin(std::abs(poc_diff(nbits, p0, h.frame_offset)), 31);
                const unsigned d0 = (unsigned)imin(std::abs(poc_diff(nbits, p1, h.frame_offset)), 31);
                const int order = d0 <= d1;
                static const uint8_t qdw[3][2] = { { 2, 3 }, { 2, 5 }, { 2, 7 } };
                static const uint8_t qdl[4][2] = { { 9, 7 }, { 11, 5 }, { 12, 4 }, { 13, 3 } };
                int k;
                for (k = 0; k < 3; k++) {
                    const int c0 = qdw[k][order], c1 = qdw[k][!order];
                    const unsigned d0c0 = d0 * c0, d1c1 = d1 * c1;
                    if ((d0 > d1 && d0c0 < d1c1) || (d0 <= d1 && d0c0 > d1c1)) break;
                }
                jnt_weights[i][j] = qdl[k][order];
            }
        }
    }
}

// ---- contexts (env.rs; C env.h:135-438) ----------------------------------------------------

namespace {

struct Ctx {
    const BlockCtx &a, &l;
    int xa, yl, have_top, have_left;
    int aref(int k) const { return a.ref[k][xa]; }
    int lref(int k) const { return l.ref[k][yl]; }
    int acomp() const { return a.comp_type[xa]; }
    int lcomp() const { return l.comp_type[yl]; }
    int aintra() const { return a.intra[xa]; }
    int lintra() const { return l.intra[yl]; }

    // counts of the neighbours' references in classes (the av1_get_*_ctx family)
    template <typename F>
    void count(F f) const {
        if (have_top && !aintra()) {
            f(aref(0));
            if (acomp()) f(aref(1));
        }
        if (have_left && !lintra()) {
            f(lref(0));
            if (lcomp()) f(lref(1));
        }
    }
    static int cmp(int c0, int c1) { return c0 == c1 ? 1 : c0 < c1 ? 0 : 2; }
    int ref_ctx() const {   // also uni_p
        int c[2] = { 0, 0 };
        count([&](int r) { c[r >= 4]++; });
        return cmp(c[0], c[1]);
    }
    int fwd_ref_ctx() const {   // also ref_3
        int c[4] = { 0, 0, 0, 0 };
        count([&](int r) { if (r < 4) c[r]++; });
        return cmp(c[0] + c[1], c[2] + c[3]);
    }
    int fwd_ref_1_ctx() const {   // also ref_4
        int c[2] = { 0, 0 };
        count([&](int r) { if (r < 2) c[r]++; });
        return cmp(c[0], c[1]);
    }
    int fwd_ref_2_ctx() const {   // also ref_5, uni_p2
        int c[2] = { 0, 0 };
        count([&](int r) { if ((unsigned)(r ^ 2) < 2) c[r - 2]++; });
        return cmp(c[0], c[1]);
    }
    int bwd_ref_ctx() const {   // also ref_2
        int c[3] = { 0, 0, 0 };
        count([&](int r) { if (r >= 4) c[r - 4]++; });
        return cmp(c[0] + c[1], c[2]);
    }
    int bwd_ref_1_ctx() const {   // also ref_6
        int c[3] = { 0, 0, 0 };
        count([&](int r) { if (r >= 4) c[r - 4]++; });
        return cmp(c[0], c[1]);
    }
    int uni_p1_ctx() const {
        int c[3] = { 0, 0, 0 };
        count([&](int r) { if ((unsigned)(r - 1) < 3) c[r - 1]++; });
        return cmp(c[0], c[1] + c[2]);
    }
    int comp_ctx() const {
        if (have_top) {
            if (have_left) {
                if (acomp()) return lcomp() ? 4 : 2 + ((unsigned)lref(0) >= 4u);
                if (lcomp()) return 2 + ((unsigned)aref(0) >= 4u);
                return (lref(0) >= 4) ^ (aref(0) >= 4);
            }
            return acomp() ? 3 : aref(0) >= 4;
        }
        if (have_left) return lcomp() ? 3 : lref(0) >= 4;
        return 1;
    }
    static int uni(int r0, int r1) { return (r0 < 4) == (r1 < 4); }
    int comp_dir_ctx() const {
        if (have_top && have_left) {
            const int ai = aintra(), li = lintra();
            if (ai && li) return 2;
            if (ai || li) {
                const bool e_is_l = ai;
                const int ct = e_is_l ? lcomp() : acomp();
                if (ct == COMP_NONE) return 2;
                return 1 + 2 * (e_is_l ? uni(lref(0), lref(1)) : uni(aref(0), aref(1)));
            }
            const int ac = acomp() != COMP_NONE, lc = lcomp() != COMP_NONE;
            const int ar0 = aref(0), lr0 = lref(0);
            if (!ac && !lc) return 1 + 2 * ((ar0 >= 4) == (lr0 >= 4));
            if (!ac || !lc) {
                const int u = ac ? uni(aref(0), aref(1)) : uni(lref(0), lref(1));
                if (!u) return 1;
                return 3 + ((ar0 >= 4) == (lr0 >= 4));
            }
            const int au = uni(aref(0), aref(1)), lu = uni(lref(0), lref(1));
            if (!au && !lu) return 0;
            if (!au || !lu) return 2;
            return 3 + ((ar0 == 4) == (lr0 == 4));
        }
        if (have_top || have_left) {
            const bool e_is_l = have_left;
            if (e_is_l ? lintra() : aintra()) return 2;
            if ((e_is_l ? lcomp() : acomp()) == COMP_NONE) return 2;
            return 4 * (e_is_l ? uni(lref(0), lref(1)) : uni(aref(0), aref(1)));
        }
        return 2;
    }
    int filter_ctx(int comp, int dir, int ref) const {
        const int af = (aref(0) == ref || aref(1) == ref) ? a.filter[dir][xa] : 3;
        const int lf = (lref(0) == ref || lref(1) == ref) ? l.filter[dir][yl] : 3;
        if (af == lf) return comp * 4 + af;
        if (af == 3) return comp * 4 + lf;
        if (lf == 3) return comp * 4 + af;
        return comp * 4 + 3;
    }
    int mask_comp_ctx() const {
        const int ac = acomp() >= COMP_SEG ? 1 : aref(0) == 6 ? 3 : 0;
        const int lc = lcomp() >= COMP_SEG ? 1 : lref(0) == 6 ? 3 : 0;
        return imin(ac + lc, 5);
    }
    int jnt_comp_ctx(int nbits, int poc, int p0, int p1) const {
        const unsigned d0 = std::abs(poc_diff(nbits, p0, poc)), d1 = std::abs(poc_diff(nbits, poc, p1));
        const int offset = d0 == d1;
        const int ac = acomp() >= COMP_AVG || aref(0) == 6;
        const int lc = lcomp() >= COMP_AVG || lref(0) == 6;
        return 3 * offset + ac + lc;
    }
};

int drl_ctx(const MvCand *st, int idx) {
    if (st[idx].weight >= 640) return st[idx + 1].weight < 640;
    return st[idx + 1].weight < 640 ? 2 : 0;
}

}  // namespace

// find_matching_ref (decode.rs; C decode.c:219-290)
void FrameDec::find_matching_ref(int edge_flags, int bw4, int bh4, int w4b, int h4b, int have_left, int have_top,
                                 int ref, uint64_t masks[2]) {
    int count = 0;
    int have_topleft = have_top && have_left;
    int have_topright = imax(bw4, bh4) < 32 && have_top && bx + bw4 < ts->col_end && (edge_flags & E444_TR);
    auto matches = [&](const RefMvBlock &r) { return r.ref[0] == ref + 1 && r.ref[1] == -1; };
    if (have_top) {
        const RefMvBlock *r2 = &rmv_at(by - 1, bx);
        if (matches(*r2)) {
            masks[0] |= 1;
            count = 1;
        }
        int aw4 = k_bdim[r2->bs].w4;
        if (aw4 >= bw4) {
            const int off = bx & (aw4 - 1);
            if (off) have_topleft = 0;
            if (aw4 - off > bw4) have_topright = 0;
        } else {
            unsigned mask = 1u << aw4;
            for (int x = aw4; x < w4b; x += aw4) {
                r2 += aw4;
                if (matches(*r2)) {
                    masks[0] |= mask;
                    if (++count >= 8) return;
                }
                aw4 = k_bdim[r2->bs].w4;
                mask <<= aw4;
            }
        }
    }
    if (have_left) {
        if (matches(rmv_at(by, bx - 1))) {
            masks[1] |= 1;
            if (++count >= 8) return;
        }
        int lh4 = k_bdim[rmv_at(by, bx - 1).bs].h4;
        if (lh4 >= bh4) {
            if (by & (lh4 - 1)) have_topleft = 0;
        } else {
            unsigned mask = 1u << lh4;
            for (int y = lh4; y < h4b; y += lh4) {
                const RefMvBlock &c = rmv_at(by + y, bx - 1);
                if (matches(c)) {
                    masks[1] |= mask;
                    if (++count >= 8) return;
                }
                lh4 = k_bdim[c.bs].h4;
                mask <<= lh4;
            }
        }
    }
    if (have_topleft && matches(rmv_at(by - 1, bx - 1))) {
        masks[1] |= 1ULL << 32;
        if (++count >= 8) return;
    }
    if (have_topright && matches(rmv_at(by - 1, bx + bw4))) masks[0] |= 1ULL << 32;
}

// derive_warpmv (decode.rs; C decode.c:292-365)
void FrameDec::derive_warpmv(int bw4, int bh4, const uint64_t masks[2], Mv mv, WarpParams &wm) {
    int pts[8][2][2], np = 0;
    auto add = [&](int dx, int dy, int sx, int sy, const RefMvBlock &r) {
        pts[np][0][0] = 16 * (2 * dx + sx * k_bdim[r.bs].w4) - 8;
        pts[np][0][1] = 16 * (2 * dy + sy * k_bdim[r.bs].h4) - 8;
        pts[np][1][0] = pts[np][0][0] + r.mv[0].x;
        pts[np][1][1] = pts[np][0][1] + r.mv[0].y;
        np++;
    };
    if ((unsigned)masks[0] == 1 && !(masks[1] >> 32)) {
        const int off = bx & (k_bdim[rmv_at(by - 1, bx).bs].w4 - 1);
        add(-off, 0, 1, -1, rmv_at(by - 1, bx));
    } else {
        for (unsigned off = 0, xmask = (uint32_t)masks[0]; np < 8 && xmask;) {
            const int tz = __builtin_ctz(xmask);
            off += tz;
            xmask >>= tz;
            add(off, 0, 1, -1, rmv_at(by - 1, bx + off));
            xmask &= ~1u;
        }
    }
    if (np < 8 && masks[1] == 1) {
        const int off = by & (k_bdim[rmv_at(by, bx - 1).bs].h4 - 1);
        add(0, -off, -1, 1, rmv_at(by - off, bx - 1));
    } else {
        for (unsigned off = 0, ymask = (uint32_t)masks[1]; np < 8 && ymask;) {
            const int tz = __builtin_ctz(ymask);
            off += tz;
            ymask >>= tz;
            add(0, off, -1, 1, rmv_at(by + off, bx - 1));
            ymask &= ~1u;
        }
    }
    if (np < 8 && (masks[1] >> 32)) add(0, 0, -1, -1, rmv_at(by - 1, bx - 1));
    if (np < 8 && (masks[0] >> 32)) add(bw4, 0, 1, -1, rmv_at(by - 1, bx + bw4));

    // keep the samples whose motion is close to the block's (the discarded ones are replaced
    // from the end of the list)
    int mvd[8], ret = 0;
    const int thresh = 4 * iclip(imax(bw4, bh4), 4, 28);
    for (int i = 0; i < np; i++) {
        mvd[i] = std::abs(pts[i][1][0] - pts[i][0][0] - mv.x) + std::abs(pts[i][1][1] - pts[i][0][1] - mv.y);
        if (mvd[i] > thresh) mvd[i] = -1;
        else ret++;
    }
    if (!ret) {
        ret = 1;
    } else {
        for (int i = 0, j = np - 1, k = 0; k < np - ret; k++, i++, j--) {
            while (mvd[i] != -1) i++;
            while (mvd[j] == -1) j--;
            if (i > j) break;
            mvd[i] = mvd[j];
            memcpy(pts[i], pts[j], sizeof(*pts));
        }
    }
    if (!find_affine_int(pts, ret, bw4, bh4, mv, wm, bx, by) && !get_shear_params(wm)) wm.type = WM_AFFINE;
    else wm.type = WM_IDENTITY;
}

// decode_b's inter branch; b.skip, seg_id and the intra flag are already read
int FrameDec::decode_inter(Block &b, int bs, int edge_flags, int has_chroma, int have_left, int have_top,
                           const SegData *seg, int seg_pred) {
    Msac &m = ts->msac;
    CdfMode &cm = ts->cdf.m;
    const BlockDim &bd = k_bdim[bs];
    const int bw4 = bd.w4, bh4 = bd.h4, by4 = by & 31;
    const int w4b = imin(bw4, bw - bx), h4b = imin(bh4, bh - by);
    const Ctx C{ a, l, bx, by4, have_top, have_left };
    int is_comp, has_subpel_filter = 0;
    MvCand st[8];
    int n_mvs = 0, ctx = 0;
    b.ref[1] = -1;
    b.interintra_type = II_NONE;
    b.motion_mode = MM_TRANSLATION;
    b.drl_idx = 0;
    if (b.skip_mode) {
        is_comp = 1;
    } else if ((!seg || (seg->ref == -1 && !seg->globalmv && !seg->skip)) && h.switchable_comp_refs &&
               imin(bw4, bh4) > 1) {
        is_comp = m.bool_adapt(cm.comp[C.comp_ctx()]);
    } else {
        is_comp = 0;
    }

    if (b.skip_mode) {
        b.ref[0] = h.skip_mode_refs[0];
        b.ref[1] = h.skip_mode_refs[1];
        b.comp_type = COMP_AVG;
        b.inter_mode = NEARESTMV_NEARESTMV;
        refmvs_find(st, &n_mvs, &ctx, b.ref[0] + 1, b.ref[1] + 1, bs, edge_flags);
        b.mv[0] = st[0].mv[0];
        b.mv[1] = st[0].mv[1];
        fix_mv(b.mv[0]);
        fix_mv(b.mv[1]);
    } else if (is_comp) {
        if (m.bool_adapt(cm.comp_dir[C.comp_dir_ctx()])) {
            // bidirectional: a forward and a backward reference
            if (m.bool_adapt(cm.comp_fwd_ref[0][C.fwd_ref_ctx()]))
                b.ref[0] = 2 + m.bool_adapt(cm.comp_fwd_ref[2][C.fwd_ref_2_ctx()]);
            else
                b.ref[0] = m.bool_adapt(cm.comp_fwd_ref[1][C.fwd_ref_1_ctx()]);
            if (m.bool_adapt(cm.comp_bwd_ref[0][C.bwd_ref_ctx()]))
                b.ref[1] = 6;
            else
                b.ref[1] = 4 + m.bool_adapt(cm.comp_bwd_ref[1][C.bwd_ref_1_ctx()]);
        } else {
            // unidirectional
            if (m.bool_adapt(cm.comp_uni_ref[0][C.ref_ctx()])) {
                b.ref[0] = 4;
                b.ref[1] = 6;
            } else {
                b.ref[0] = 0;
                b.ref[1] = 1 + m.bool_adapt(cm.comp_uni_ref[1][C.uni_p1_ctx()]);
                if (b.ref[1] == 2) b.ref[1] += m.bool_adapt(cm.comp_uni_ref[2][C.fwd_ref_2_ctx()]);
            }
        }
        refmvs_find(st, &n_mvs, &ctx, b.ref[0] + 1, b.ref[1] + 1, bs, edge_flags);
        b.inter_mode = m.symbol(cm.comp_inter_mode[ctx], 7);
        const uint8_t *im = k_comp_inter_modes[b.inter_mode];
        b.drl_idx = 0;
        if (b.inter_mode == NEWMV_NEWMV) {
            if (n_mvs > 1) {
                b.drl_idx += m.bool_adapt(cm.drl_bit[drl_ctx(st, 0)]);
                if (b.drl_idx == 1 && n_mvs > 2) b.drl_idx += m.bool_adapt(cm.drl_bit[drl_ctx(st, 1)]);
            }
        } else if (im[0] == NEARMV || im[1] == NEARMV) {
            b.drl_idx = 1;
            if (n_mvs > 2) {
                b.drl_idx += m.bool_adapt(cm.drl_bit[drl_ctx(st, 1)]);
                if (b.drl_idx == 2 && n_mvs > 3) b.drl_idx += m.bool_adapt(cm.drl_bit[drl_ctx(st, 2)]);
            }
        }
        has_subpel_filter = imin(bw4, bh4) == 1 || b.inter_mode != GLOBALMV_GLOBALMV;
        for (int i = 0; i < 2; i++) {
            switch (im[i]) {
            case NEARMV:
            case NEARESTMV:
                b.mv[i] = st[b.drl_idx].mv[i];
                fix_mv(b.mv[i]);
                break;
            case GLOBALMV:
                has_subpel_filter |= h.gmv[b.ref[i]].type == WM_TRANSLATION;
                b.mv[i] = gmv_2d(b.ref[i], bw4, bh4);
                break;
            case NEWMV:
                b.mv[i] = st[b.drl_idx].mv[i];
                read_mv_residual(b.mv[i], ts->cdf.mv, !h.force_integer_mv);
                break;
            }
        }
        // jnt_comp vs. seg vs. wedge
        int is_segwedge = 0;
        if (s.masked_compound) is_segwedge = m.bool_adapt(cm.mask_comp[C.mask_comp_ctx()]);
        if (!is_segwedge) {
            if (s.jnt_comp) {
                const int jctx = C.jnt_comp_ctx(s.order_hint_n_bits, h.frame_offset,
                                                in_.refs[b.ref[0]]->hdr->frame_offset,
                                                in_.refs[b.ref[1]]->hdr->frame_offset);
                b.comp_type = COMP_WAVG + m.bool_adapt(cm.jnt_comp[jctx]);
            } else {
                b.comp_type = COMP_AVG;
            }
        } else {
            if (kWedgeAllowed & (1u << bs)) {
                const int wctx = k_wedge_ctx[bs];
                b.comp_type = COMP_WEDGE - m.bool_adapt(cm.wedge_comp[wctx]);
                if (b.comp_type == COMP_WEDGE) b.wedge_idx = m.symbol(cm.wedge_idx[wctx], 15);
            } else {
                b.comp_type = COMP_SEG;
            }
            b.mask_sign = m.bool_equi();
        }
    } else {
        b.comp_type = COMP_NONE;
        // single reference
        if (seg && seg->ref > 0) {
            b.ref[0] = seg->ref - 1;
        } else if (seg && (seg->globalmv || seg->skip)) {
            b.ref[0] = 0;
        } else if (m.bool_adapt(cm.ref[0][C.ref_ctx()])) {
            if (m.bool_adapt(cm.ref[1][C.bwd_ref_ctx()])) b.ref[0] = 6;
            else b.ref[0] = 4 + m.bool_adapt(cm.ref[5][C.bwd_ref_1_ctx()]);
        } else {
            if (m.bool_adapt(cm.ref[2][C.fwd_ref_ctx()])) b.ref[0] = 2 + m.bool_adapt(cm.ref[4][C.fwd_ref_2_ctx()]);
            else b.ref[0] = m.bool_adapt(cm.ref[3][C.fwd_ref_1_ctx()]);
        }
        b.ref[1] = -1;
        refmvs_find(st, &n_mvs, &ctx, b.ref[0] + 1, -1, bs, edge_flags);
        if ((seg && (seg->skip || seg->globalmv)) || m.bool_adapt(cm.newmv_mode[ctx & 7])) {
            if ((seg && (seg->skip || seg->globalmv)) || !m.bool_adapt(cm.globalmv_mode[(ctx >> 3) & 1])) {
                b.inter_mode = GLOBALMV;
                b.mv[0] = gmv_2d(b.ref[0], bw4, bh4);
                has_subpel_filter = imin(bw4, bh4) == 1 || h.gmv[b.ref[0]].type == WM_TRANSLATION;
            } else {
                has_subpel_filter = 1;
                if (m.bool_adapt(cm.refmv_mode[(ctx >> 4) & 15])) {
                    b.inter_mode = NEARMV;
                    b.drl_idx = 1;
                    if (n_mvs > 2) {
                        b.drl_idx += m.bool_adapt(cm.drl_bit[drl_ctx(st, 1)]);
                        if (b.drl_idx == 2 && n_mvs > 3) b.drl_idx += m.bool_adapt(cm.drl_bit[drl_ctx(st, 2)]);
                    }
                } else {
                    b.inter_mode = NEARESTMV;
                    b.drl_idx = 0;
                }
                b.mv[0] = st[b.drl_idx].mv[0];
                if (b.drl_idx < 2) fix_mv(b.mv[0]);
            }
        } else {
            has_subpel_filter = 1;
            b.inter_mode = NEWMV;
            b.drl_idx = 0;
            if (n_mvs > 1) {
                b.drl_idx += m.bool_adapt(cm.drl_bit[drl_ctx(st, 0)]);
                if (b.drl_idx == 1 && n_mvs > 2) b.drl_idx += m.bool_adapt(cm.drl_bit[drl_ctx(st, 1)]);
            }
            if (n_mvs > 1) {
                b.mv[0] = st[b.drl_idx].mv[0];
            } else {
                b.mv[0] = st[0].mv[0];
                fix_mv(b.mv[0]);
            }
            read_mv_residual(b.mv[0], ts->cdf.mv, !h.force_integer_mv);
        }
        // inter-intra
        const int ii_grp = k_ymode_size_ctx[bs];
        if (s.inter_intra && (kInterIntraAllowed & (1u << bs)) && m.bool_adapt(cm.interintra[ii_grp])) {
            b.interintra_mode = m.symbol(cm.interintra_mode[ii_grp], 3);
            const int wctx = k_wedge_ctx[bs];
            b.interintra_type = II_BLEND + m.bool_adapt(cm.interintra_wedge[wctx]);
            if (b.interintra_type == II_WEDGE) b.wedge_idx = m.symbol(cm.wedge_idx[wctx], 15);
        }
        // motion mode (OBMC / warp)
        auto oddzero = [](const std::vector<uint8_t> &v, int off, int len) {
            for (int n = 0; n < len; n++)
                if (!v[off + n * 2]) return true;
            return false;
        };
        if (h.switchable_motion_mode && b.interintra_type == II_NONE && imin(bw4, bh4) >= 2 &&
            !(!h.force_integer_mv && b.inter_mode == GLOBALMV && h.gmv[b.ref[0]].type > WM_TRANSLATION) &&
            ((have_left && oddzero(l.intra, by4 + 1, h4b >> 1)) || (have_top && oddzero(a.intra, bx + 1, w4b >> 1)))) {
            uint64_t mask[2] = { 0, 0 };
            find_matching_ref(edge_flags, bw4, bh4, w4b, h4b, have_left, have_top, b.ref[0], mask);
            const int allow_warp = !svc_scale[b.ref[0]][0] && !h.force_integer_mv && h.warp_motion && (mask[0] | mask[1]);
            b.motion_mode = allow_warp ? m.symbol(cm.motion_mode[bs], 2) : m.bool_adapt(cm.obmc[bs]);
            if (b.motion_mode == MM_WARP) {
                has_subpel_filter = 0;
                derive_warpmv(bw4, bh4, mask, b.mv[0], warpmv);
            }
        }
    }

    // subpel filter
    int filter[2];
    if (h.subpel_filter_mode == FILTER_SWITCHABLE) {
        if (has_subpel_filter) {
            const int comp = b.comp_type != COMP_NONE;
            filter[0] = m.symbol(cm.filter[0][C.filter_ctx(comp, 0, b.ref[0])], 2);
            if (s.dual_filter) filter[1] = m.symbol(cm.filter[1][C.filter_ctx(comp, 1, b.ref[0])], 2);
            else filter[1] = filter[0];
        } else {
            filter[0] = filter[1] = FILTER_REGULAR;
        }
    } else {
        filter[0] = filter[1] = h.subpel_filter_mode;
    }
    b.filter[0] = filter[0];
    b.filter[1] = filter[1];
    b.filter2d = k_filter_2d[filter[1]][filter[0]];

    read_vartx_tree(b, bs);

    // reconstruction work: prediction descriptors, then the residual walk (coefficients)
    if (int e = emit_inter_pred(b, has_chroma)) return e;
    emit_inter_residual(b, has_chroma);

    if (h.lf.level_y[0] || h.lf.level_y[1]) create_lf_mask_inter(b, has_chroma);

    // refmvs (splat_oneref_mv / splat_tworef_mv, C decode.c:554-600) and the filter map
    RefMvBlock r{};
    r.ref[0] = (int8_t)(b.ref[0] + 1);
    r.mv[0] = b.mv[0];
    r.bs = (uint8_t)bs;
    if (is_comp) {
        r.ref[1] = (int8_t)(b.ref[1] + 1);
        r.mv[1] = b.mv[1];
        r.mf = (uint8_t)((b.inter_mode == GLOBALMV_GLOBALMV) | (!!((1 << b.inter_mode) & 0xbc) * 2));
    } else {
        r.ref[1] = b.interintra_type ? 0 : -1;
        r.mv[1] = Mv{ 0, 0 };
        r.mf = (uint8_t)((b.inter_mode == GLOBALMV && imin(bw4, bh4) >= 2) | ((b.inter_mode == NEWMV) * 2));
    }
    splat(r, bw4, bh4);
    for (int y = 0; y < bh4; y++)
        for (int x = 0; x < bw4; x++) f2d_at(by + y, bx + x) = (uint8_t)b.filter2d;

    // contexts
    setn(a.seg_pred, bx, bw4, seg_pred);
    setn(l.seg_pred, by4, bh4, seg_pred);
    setn(a.skip_mode, bx, bw4, b.skip_mode);
    setn(l.skip_mode, by4, bh4, b.skip_mode);
    setn(a.intra, bx, bw4, 0);
    setn(l.intra, by4, bh4, 0);
    setn(a.skip, bx, bw4, b.skip);
    setn(l.skip, by4, bh4, b.skip);
    setn(a.pal_sz, bx, bw4, 0);
    setn(l.pal_sz, by4, bh4, 0);
    for (int i = 0; i < bw4; i++) pal_sz_uv[0][(bx & 31) + i] = 0;
    for (int i = 0; i < bh4; i++) pal_sz_uv[1][by4 + i] = 0;
    setn(a.tx_intra, bx, bw4, bd.lw4);
    setn(l.tx_intra, by4, bh4, bd.lh4);
    setn(a.comp_type, bx, bw4, b.comp_type);
    setn(l.comp_type, by4, bh4, b.comp_type);
    setn(a.filter[0], bx, bw4, filter[0]);
    setn(l.filter[0], by4, bh4, filter[0]);
    setn(a.filter[1], bx, bw4, filter[1]);
    setn(l.filter[1], by4, bh4, filter[1]);
    setn(a.mode, bx, bw4, b.inter_mode);
    setn(l.mode, by4, bh4, b.inter_mode);
    setn(a.ref[0], bx, bw4, b.ref[0]);
    setn(l.ref[0], by4, bh4, b.ref[0]);
    setn(a.ref[1], bx, bw4, b.ref[1]);
    setn(l.ref[1], by4, bh4, b.ref[1]);
    if (has_chroma) {
        setn(a.uvmode, bx >> ss_hor, (bw4 + ss_hor) >> ss_hor, DC_PRED);
        setn(l.uvmode, by4 >> ss_ver, (bh4 + ss_ver) >> ss_ver, DC_PRED);
    }
    return 0;
}

// ---- loop-filter masks of inter blocks (lf_mask.rs; C lf_mask.c:39-148, 346-406) ------------

// decomp_tx: the transform size (log2, capped at 16 px) and step of every 4x4 of the block,
// per edge direction, from the var-tx split masks
static void decomp_tx(uint8_t (*txa)[2][32][32], int from, int depth, int y_off, int x_off, const uint16_t *tx_masks,
                      int y0, int x0) {
    const TxDim &t = k_txdim[from];
    const int is_split = (from == TX_4X4 || depth > 1) ? 0 : (tx_masks[depth] >> (y_off * 4 + x_off)) & 1;
    if (is_split) {
        const int sub = t.sub, htw4 = t.w >> 1, hth4 = t.h >> 1;
        decomp_tx(txa, sub, depth + 1, y_off * 2, x_off * 2, tx_masks, y0, x0);
        if (t.w >= t.h) decomp_tx(txa, sub, depth + 1, y_off * 2, x_off * 2 + 1, tx_masks, y0, x0 + htw4);
        if (t.h >= t.w) {
            decomp_tx(txa, sub, depth + 1, y_off * 2 + 1, x_off * 2, tx_masks, y0 + hth4, x0);
            if (t.w >= t.h) decomp_tx(txa, sub, depth + 1, y_off * 2 + 1, x_off * 2 + 1, tx_masks, y0 + hth4, x0 + htw4);
        }
    } else {
        const int lw = imin(2, t.lw), lh = imin(2, t.lh);
        for (int y = 0; y < t.h && y0 + y < 32; y++)
            for (int x = 0; x < t.w && x0 + x < 32; x++) {
                txa[0][0][y0 + y][x0 + x] = (uint8_t)lw;
                txa[1][0][y0 + y][x0 + x] = (uint8_t)lh;
                if (x == 0) txa[0][1][y0 + y][x0] = (uint8_t)t.w;
                if (y == 0) txa[1][1][y0][x0 + x] = (uint8_t)t.h;
            }
    }
}

void FrameDec::mask_edges_inter(int by4, int bx4, int w4_, int h4_, int skip, int max_tx, const uint16_t *tx_masks,
                                uint8_t *actx, uint8_t *lctx, uint16_t (*masks)[32][3][2]) {
    const TxDim &t = k_txdim[max_tx];
    static thread_local uint8_t txa[2][2][32][32];
    for (int y_off = 0, y = 0; y < h4_; y += t.h, y_off++)
        for (int x_off = 0, x = 0; x < w4_; x += t.w, x_off++) decomp_tx(txa, max_tx, 0, y_off, x_off, tx_masks, y, x);
    unsigned mask = 1u << by4;
    for (int y = 0; y < h4_; y++, mask <<= 1) {
        const int sidx = mask >= 0x10000;
        masks[0][bx4][imin(txa[0][0][y][0], lctx[y])][sidx] |= (uint16_t)(mask >> (sidx << 4));
    }
    mask = 1u << bx4;
    for (int x = 0; x < w4_; x++, mask <<= 1) {
        const int sidx = mask >= 0x10000;
        masks[1][by4][imin(txa[1][0][0][x], actx[x])][sidx] |= (uint16_t)(mask >> (sidx << 4));
    }
    if (!skip) {
        mask = 1u << by4;
        for (int y = 0; y < h4_; y++, mask <<= 1) {
            const int sidx = mask >= 0x10000;
            const uint16_t sm = (uint16_t)(mask >> (sidx << 4));
            int ltx = txa[0][0][y][0], step = txa[0][1][y][0];
            for (int x = step; x < w4_; x += step) {
                const int rtx = txa[0][0][y][x];
                masks[0][bx4 + x][imin(rtx, ltx)][sidx] |= sm;
                ltx = rtx;
                step = txa[0][1][y][x];
            }
        }
        mask = 1u << bx4;
        for (int x = 0; x < w4_; x++, mask <<= 1) {
            const int sidx = mask >= 0x10000;
            const uint16_t sm = (uint16_t)(mask >> (sidx << 4));
            int ttx = txa[1][0][0][x], step = txa[1][1][0][x];
            for (int y = step; y < h4_; y += step) {
                const int btx = txa[1][0][y][x];
                masks[1][by4 + y][imin(ttx, btx)][sidx] |= sm;
                ttx = btx;
                step = txa[1][1][y][x];
            }
        }
    }
    for (int y = 0; y < h4_; y++) lctx[y] = txa[0][0][y][w4_ - 1];
    memcpy(actx, txa[1][0][h4_ - 1], w4_);
}

void FrameDec::create_lf_mask_inter(const Block &b, int has_chroma) {
    const int is_globalmv = b.inter_mode == (b.comp_type != COMP_NONE ? (int)GLOBALMV_GLOBALMV : (int)GLOBALMV);
    // lflvl[seg][plane/dir][ref + 1][!is_globalmv]
    const uint8_t (*fl)[8][2] = ts->lflvl.v[b.seg_id];
    const int ri = b.ref[0] + 1, mi = !is_globalmv;
    int ytx = b.max_ytx, uvtx = b.uvtx;
    if (h.seg.lossless[b.seg_id]) ytx = uvtx = TX_4X4;
    const BlockDim &bd = k_bdim[b.bs];
    const int bw4 = imin(w4 - bx, bd.w4), bh4 = imin(h4 - by, bd.h4);
    const int bx4 = bx & 31, by4 = by & 31;
    if (bw4 > 0 && bh4 > 0) {
        for (int y = 0; y < bh4; y++)
            for (int x = 0; x < bw4; x++) {
                uint8_t *lv = &mw.lf_level[(((size_t)(by + y) * b4_stride) + bx + x) * 4];
                lv[0] = fl[0][ri][mi];
                lv[1] = fl[1][ri][mi];
            }
        mask_edges_inter(by4, bx4, bw4, bh4, b.skip, ytx, b.tx_split, &a.tx_lpf_y[bx], &l.tx_lpf_y[by4],
                         reinterpret_cast<uint16_t (*)[32][3][2]>(lf_mask->filter_y));
    }
    if (!has_chroma) return;
    const int cbw4 = imin(((w4 + ss_hor) >> ss_hor) - (bx >> ss_hor), (bd.w4 + ss_hor) >> ss_hor);
    const int cbh4 = imin(((h4 + ss_ver) >> ss_ver) - (by >> ss_ver), (bd.h4 + ss_ver) >> ss_ver);
    if (cbw4 <= 0 || cbh4 <= 0) return;
    for (int y = 0; y < cbh4; y++)
        for (int x = 0; x < cbw4; x++) {
            uint8_t *lv = &mw.lf_level[(((size_t)((by >> ss_ver) + y) * b4_stride) + (bx >> ss_hor) + x) * 4];
            lv[2] = fl[2][ri][mi];
            lv[3] = fl[3][ri][mi];
        }
    mask_edges_chroma(by4 >> ss_ver, bx4 >> ss_hor, cbw4, cbh4, b.skip, uvtx, &a.tx_lpf_uv[bx >> ss_hor],
                      &l.tx_lpf_uv[by4 >> ss_ver], reinterpret_cast<uint16_t (*)[32][2][2]>(lf_mask->filter_uv));
}

}  // namespace fd
}  // namespace av1
