// decode.cpp — per-frame block decoding: tiles -> superblocks -> partitions -> blocks, the
// mode info, palette, transform partition and coefficient decoding of every block, and the
// loop-filter / CDEF / restoration metadata. Emits the frame's pass-2 work (FrameWork) instead
// of reconstructing pixels.
//
// Restates decode.rs / recon.rs for the parsing side (C src/decode.c:54-3325: decode_b,
// decode_sb, setup_tile, read_restoration_info, decode_tile_sbrow, decode_frame_init; C
// src/recon_tmpl.c:49-960: get_skip_ctx, get_dc_sign_ctx, get_lo_ctx, decode_coefs,
// read_coef_tree; :2203-2376 palette), lf_mask.rs (C src/lf_mask.c) and the recon-order edge
// availability of recon_b_intra (C src/recon_tmpl.c:1200-1603), which becomes the flags of
// each MiIntraBlock.
#include <cerrno>
#include <climits>
#include <cstdio>
#include <string>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <new>
#include <thread>

#include "framedec.h"

namespace av1 {

void BlockCtx::alloc(int n) {
    for (auto *v : {&mode, &lcoef, &ccoef[0], &ccoef[1], &seg_pred, &skip, &skip_mode, &intra, &comp_type,
                    &filter[0], &filter[1], &tx_lpf_y, &tx_lpf_uv, &partition, &uvmode, &pal_sz})
        v->assign(n, 0);
    for (auto *v : {&ref[0], &ref[1], &tx_intra, &tx}) v->assign(n, 0);
}

// decode.rs reset_context (C decode.c:2440-2466), pass 0
void BlockCtx::reset(bool keyframe) {
    std::fill(intra.begin(), intra.end(), keyframe);
    std::fill(uvmode.begin(), uvmode.end(), DC_PRED);
    if (keyframe) std::fill(mode.begin(), mode.end(), DC_PRED);
    std::fill(partition.begin(), partition.end(), 0);
    std::fill(skip.begin(), skip.end(), 0);
    std::fill(skip_mode.begin(), skip_mode.end(), 0);
    std::fill(tx_lpf_y.begin(), tx_lpf_y.end(), 2);
    std::fill(tx_lpf_uv.begin(), tx_lpf_uv.end(), 1);
    std::fill(tx_intra.begin(), tx_intra.end(), -1);
    std::fill(tx.begin(), tx.end(), TX_64X64);
    if (!keyframe) {
        std::fill(ref[0].begin(), ref[0].end(), -1);
        std::fill(ref[1].begin(), ref[1].end(), -1);
        std::fill(comp_type.begin(), comp_type.end(), 0);
        std::fill(mode.begin(), mode.end(), NEARESTMV);
    }
    std::fill(lcoef.begin(), lcoef.end(), 0x40);
    std::fill(ccoef[0].begin(), ccoef[0].end(), 0x40);
    std::fill(ccoef[1].begin(), ccoef[1].end(), 0x40);
    std::fill(filter[0].begin(), filter[0].end(), 3);
    std::fill(filter[1].begin(), filter[1].end(), 3);
    std::fill(seg_pred.begin(), seg_pred.end(), 0);
    std::fill(pal_sz.begin(), pal_sz.end(), 0);
}

namespace fd {

// ------------------------------------------------------------------------------------------
// frame-level setup (decode.rs decode_frame_init; C decode.c:54-75, 2776-3155; lf_mask.c
// dav1d_calc_eih / dav1d_calc_lf_values)

void FrameDec::init_quant(int qidx, uint16_t (*dq)[3][2]) {
    for (int i = 0; i < (h.seg.enabled ? 8 : 1); i++) {
        const int yac = h.seg.enabled ? iclip(qidx + h.seg.d[i].delta_q, 0, 255) : qidx;
        const int ydc = iclip(yac + h.quant.ydc_delta, 0, 255);
        const int uac = iclip(yac + h.quant.uac_delta, 0, 255), udc = iclip(yac + h.quant.udc_delta, 0, 255);
        const int vac = iclip(yac + h.quant.vac_delta, 0, 255), vdc = iclip(yac + h.quant.vdc_delta, 0, 255);
        dq[i][0][0] = dq_value(hbd_idx, ydc, 0);
        dq[i][0][1] = dq_value(hbd_idx, yac, 1);
        dq[i][1][0] = dq_value(hbd_idx, udc, 0);
        dq[i][1][1] = dq_value(hbd_idx, uac, 1);
        dq[i][2][0] = dq_value(hbd_idx, vdc, 0);
        dq[i][2][1] = dq_value(hbd_idx, vac, 1);
    }
}

static void lf_value(uint8_t (*vals)[2], int base_lvl, int lf_delta, int seg_delta, const FrameHdr &h, bool mr) {
    const int base = iclip(iclip(base_lvl + lf_delta, 0, 63) + seg_delta, 0, 63);
    if (!mr) {
        for (int r = 0; r < 8; r++) vals[r][0] = vals[r][1] = (uint8_t)base;
        return;
    }
    const int sh = base >= 32;
    vals[0][0] = vals[0][1] = (uint8_t)iclip(base + h.lf.ref_delta[0] * (1 << sh), 0, 63);
    for (int r = 1; r < 8; r++)
        for (int m = 0; m < 2; m++)
            vals[r][m] = (uint8_t)iclip(base + (h.lf.mode_delta[m] + h.lf.ref_delta[r]) * (1 << sh), 0, 63);
}

void FrameDec::calc_lf_values(LfLvl &out, const int8_t d[4]) {
    const int n_seg = h.seg.enabled ? 8 : 1;
    if (!h.lf.level_y[0] && !h.lf.level_y[1]) {
        memset(out.v, 0, sizeof(out.v[0]) * n_seg);
        return;
    }
    const bool mr = h.lf.mode_ref_delta_enabled;
    for (int sgi = 0; sgi < n_seg; sgi++) {
        const SegData *sd = h.seg.enabled ? &h.seg.d[sgi] : nullptr;
        lf_value(out.v[sgi][0], h.lf.level_y[0], d[0], sd ? sd->delta_lf_y_v : 0, h, mr);
        lf_value(out.v[sgi][1], h.lf.level_y[1], d[h.delta.lf_multi ? 1 : 0], sd ? sd->delta_lf_y_h : 0, h, mr);
        if (!h.lf.level_u) memset(out.v[sgi][2], 0, 16);
        else lf_value(out.v[sgi][2], h.lf.level_u, d[h.delta.lf_multi ? 2 : 0], sd ? sd->delta_lf_u : 0, h, mr);
        if (!h.lf.level_v) memset(out.v[sgi][3], 0, 16);
        else lf_value(out.v[sgi][3], h.lf.level_v, d[h.delta.lf_multi ? 3 : 0], sd ? sd->delta_lf_v : 0, h, mr);
    }
}

// decode.rs setup_tile (C decode.c:2475-2556)
void FrameDec::setup_tile(TileState &t, const uint8_t *data, size_t sz, int row, int col) {
    const int col_sb_start = h.tiling.col_start_sb[col], col_sb_end = h.tiling.col_start_sb[col + 1];
    const int row_sb_start = h.tiling.row_start_sb[row], row_sb_end = h.tiling.row_start_sb[row + 1];
    if (in_cdf_) t.cdf = *in_cdf_;
    else cdf_init_default(t.cdf, h.quant.yac);
    t.last_qidx = h.quant.yac;
    memset(t.last_delta_lf, 0, 4);
    memcpy(t.dq, dq_frame, sizeof(t.dq));
    t.lflvl = lflvl_frame;
    t.msac.init(data, sz, h.disable_cdf_update);
    t.col_start = col_sb_start << sb_shift;
    t.col_end = imin(col_sb_end << sb_shift, bw);
    t.row_start = row_sb_start << sb_shift;
    t.row_end = imin(row_sb_end << sb_shift, bh);
    const int col_sb128_start = col_sb_start >> !s.sb128;
    int sb_idx, unit_idx;
    if (h.width[0] != h.width[1]) {
        sb_idx = (t.row_start >> 5) * fw.sr_sb128w;
        unit_idx = (t.row_start & 16) >> 3;
    } else {
        sb_idx = (t.row_start >> 5) * fw.sb128w + col_sb128_start;
        unit_idx = ((t.row_start & 16) >> 3) + ((t.col_start & 16) >> 4);
    }
    for (int p = 0; p < 3; p++) {
        t.lr_ref[p] = nullptr;
        if (!((fw.restore_planes >> p) & 1)) continue;
        MiAv1RestorationUnit *u;
        if (h.width[0] != h.width[1]) {
            const int sh = p && ss_hor;
            const int d = h.superres_denom, usl = h.lr.unit_size[!!p];
            const int rnd = (8 << usl) - 1, shift = usl + 3;
            const int x = ((4 * t.col_start * d >> sh) + rnd) >> shift;
            const int px_x = x << (usl + sh);
            const int u_idx = unit_idx + ((px_x & 64) >> 6);
            const int sb128x = px_x >> 7;
            if (sb128x >= fw.sr_sb128w) continue;
            u = &mw.lr_mask[sb_idx + sb128x].lr[p][u_idx];
        } else {
            u = &mw.lr_mask[sb_idx].lr[p][unit_idx];
        }
        u->filter_v[0] = 3;
        u->filter_v[1] = -7;
        u->filter_v[2] = 15;
        u->filter_h[0] = 3;
        u->filter_h[1] = -7;
        u->filter_h[2] = 15;
        u->sgr_weights[0] = -32;
        u->sgr_weights[1] = 31;
        t.lr_ref[p] = u;
    }
}

// decode.rs read_restoration_info (C decode.c:2558-2620)
void FrameDec::read_lr(MiAv1RestorationUnit *lr, int p, int frame_type) {
    Msac &m = ts->msac;
    if (frame_type == RESTORE_SWITCHABLE) {
        const int f = m.symbol(ts->cdf.m.restore_switchable, 2);
        lr->type = f + !!f;
    } else {
        const unsigned t = m.bool_adapt(frame_type == RESTORE_WIENER ? ts->cdf.m.restore_wiener : ts->cdf.m.restore_sgrproj);
        lr->type = t ? frame_type : RESTORE_NONE;
    }
    MiAv1RestorationUnit *ref = ts->lr_ref[p];
    if (lr->type == RESTORE_WIENER) {
        lr->filter_v[0] = p ? 0 : m.subexp(ref->filter_v[0] + 5, 16, 1) - 5;
        lr->filter_v[1] = m.subexp(ref->filter_v[1] + 23, 32, 2) - 23;
        lr->filter_v[2] = m.subexp(ref->filter_v[2] + 17, 64, 3) - 17;
        lr->filter_h[0] = p ? 0 : m.subexp(ref->filter_h[0] + 5, 16, 1) - 5;
        lr->filter_h[1] = m.subexp(ref->filter_h[1] + 23, 32, 2) - 23;
        lr->filter_h[2] = m.subexp(ref->filter_h[2] + 17, 64, 3) - 17;
        memcpy(lr->sgr_weights, ref->sgr_weights, 2);
        ts->lr_ref[p] = lr;
    } else if (lr->type == RESTORE_SGRPROJ) {
        const unsigned idx = m.bools(4);
        lr->type += idx;
        lr->sgr_weights[0] = k_sgr_params[idx][0] ? m.subexp(ref->sgr_weights[0] + 96, 128, 4) - 96 : 0;
        lr->sgr_weights[1] = k_sgr_params[idx][1] ? m.subexp(ref->sgr_weights[1] + 32, 128, 4) - 32 : 95;
        memcpy(lr->filter_v, ref->filter_v, 3);
        memcpy(lr->filter_h, ref->filter_h, 3);
        ts->lr_ref[p] = lr;
    }
}

// ------------------------------------------------------------------------------------------
// coefficients (recon.rs decode_coefs and its context helpers; C recon_tmpl.c:49-724)

static unsigned skip_ctx(const TxDim &t, int bs, const uint8_t *a, const uint8_t *l, int chroma, int layout) {
    const BlockDim &bd = k_bdim[bs];
    if (chroma) {
        const int ssv = layout == 1, ssh = layout != 3;
        const int not_one = bd.lw4 - (!!bd.lw4 && ssh) > t.lw || bd.lh4 - (!!bd.lh4 && ssv) > t.lh;
        int ca = 0, cl = 0;
        for (int i = 0; i < (1 << t.lw); i++) ca |= a[i] != 0x40;
        for (int i = 0; i < (1 << t.lh); i++) cl |= l[i] != 0x40;
        return 7 + not_one * 3 + ca + cl;
    }
    if (bd.lw4 == t.lw && bd.lh4 == t.lh) return 0;
    unsigned la = 0, ll = 0;
    for (int i = 0; i < (1 << t.lw); i++) la |= a[i];
    for (int i = 0; i < (1 << t.lh); i++) ll |= l[i];
    return k_skip_ctx[imin(la & 0x3f, 4)][imin(ll & 0x3f, 4)];
}

static unsigned dc_sign_ctx(const TxDim &t, const uint8_t *a, const uint8_t *l) {
    int s = 0;
    for (int i = 0; i < t.w; i++) s += (a[i] >> 6) - 1;
    for (int i = 0; i < t.h; i++) s += (l[i] >> 6) - 1;
    return (s != 0) + (s > 0);
}

static unsigned lo_ctx(const uint8_t *lv, int cls, unsigned *hi_mag, const uint8_t (*off)[5], unsigned x, unsigned y,
                       ptrdiff_t stride) {
    unsigned mag = lv[1] + lv[stride];
    unsigned o;
    if (cls == 0) {
        mag += lv[stride + 1];
        *hi_mag = mag;
        mag += lv[2] + lv[2 * stride];
        o = off[imin(y, 4)][imin(x, 4)];
    } else {
        mag += lv[2];
        *hi_mag = mag;
        mag += lv[3] + lv[4];
        o = 26 + (y > 1 ? 10 : y * 5);
    }
    return o + (mag > 512 ? 4 : (mag + 64) >> 7);
}

int FrameDec::decode_coefs(uint8_t *actx, uint8_t *lctx, int tx, int bs, const Block &b, int intra, int plane,
                           int32_t *cf, int *txtp, uint8_t *res_ctx) {
    Msac &m = ts->msac;
    CdfCoef &cc = ts->cdf.coef;
    const int chroma = !!plane;
    const int lossless = h.seg.lossless[b.seg_id];
    const TxDim &t = k_txdim[tx];

    if (m.bool_adapt(cc.skip[t.ctx][skip_ctx(t, bs, actx, lctx, chroma, layout)])) {
        *res_ctx = 0x40;
        *txtp = lossless * WHT_WHT;
        return -1;
    }
    // transform type
    if (lossless) {
        *txtp = WHT_WHT;
    } else if (t.max + intra >= TX_64X64) {
        *txtp = DCT_DCT;
    } else if (chroma) {
        if (intra) {
            *txtp = k_txtp_from_uvmode[b.uv_mode];
        } else {
            // inter chroma: derived from the co-located luma type (env.rs get_uv_inter_txtp)
            const int y = *txtp;
            if (t.max == TX_32X32) *txtp = y == IDTX ? IDTX : DCT_DCT;
            else if (t.min == TX_16X16 && ((1 << y) & ((1 << H_FLIPADST) | (1 << V_FLIPADST) | (1 << H_ADST) | (1 << V_ADST))))
                *txtp = DCT_DCT;
        }
    } else if (!h.seg.qidx[b.seg_id]) {
        *txtp = DCT_DCT;
    } else if (intra) {
        const int ym = b.y_mode == FILTER_PRED ? k_filter_mode_to_y_mode[b.y_angle] : b.y_mode;
        if (h.reduced_txtp_set || t.min == TX_16X16) {
            *txtp = k_tx_types_per_set[m.symbol(ts->cdf.m.txtp_intra2[t.min][ym], 4)];
        } else {
            *txtp = k_tx_types_per_set[m.symbol(ts->cdf.m.txtp_intra1[t.min][ym], 6) + 5];
        }
    } else {
        if (h.reduced_txtp_set || t.max == TX_32X32) {
            *txtp = m.bool_adapt(ts->cdf.m.txtp_inter3[t.min]) ? DCT_DCT : IDTX;
        } else if (t.min == TX_16X16) {
            *txtp = k_tx_types_per_set[m.symbol(ts->cdf.m.txtp_inter2, 11) + 12];
        } else {
            *txtp = k_tx_types_per_set[m.symbol(ts->cdf.m.txtp_inter1[t.min], 15) + 24];
        }
    }

    // end of block
    const int szctx = imin(t.lw, 3) + imin(t.lh, 3);
    const int cls = k_tx_class[*txtp];
    const int is_1d = cls != 0;
    int eob_bin;
    switch (szctx) {
    case 0: eob_bin = m.symbol(cc.eob_bin_16[chroma][is_1d], 4); break;
    case 1: eob_bin = m.symbol(cc.eob_bin_32[chroma][is_1d], 5); break;
    case 2: eob_bin = m.symbol(cc.eob_bin_64[chroma][is_1d], 6); break;
    case 3: eob_bin = m.symbol(cc.eob_bin_128[chroma][is_1d], 7); break;
    case 4: eob_bin = m.symbol(cc.eob_bin_256[chroma][is_1d], 8); break;
    case 5: eob_bin = m.symbol(cc.eob_bin_512[chroma], 9); break;
    default: eob_bin = m.symbol(cc.eob_bin_1024[chroma], 10); break;
    }
    int eob;
    if (eob_bin > 1) {
        const int hi = m.bool_adapt(cc.eob_hi_bit[t.ctx][chroma][eob_bin]);
        eob = ((hi | 2) << (eob_bin - 2)) | m.bools(eob_bin - 2);
    } else {
        eob = eob_bin;
    }

    uint16_t (*eob_cdf)[4] = cc.eob_base_tok[t.ctx][chroma];
    uint16_t (*hi_cdf)[4] = cc.br_tok[imin(t.ctx, 3)][chroma];
    unsigned rc, dc_tok;
    if (eob) {
        uint16_t (*lo_cdf)[4] = cc.base_tok[t.ctx][chroma];
        uint8_t levels[36 * 36];
        const int sw = imin(t.w, 8), sh = imin(t.h, 8);
        unsigned ctx = 1 + (eob > sw * sh * 2) + (eob > sw * sh * 4);
        const int eob_tok = m.symbol(eob_cdf[ctx], 2);
        int tok = eob_tok + 1;
        int level_tok = tok * 0x41;
        unsigned mag = 0;
        const uint16_t *scan = k_scan[tx];
        const uint8_t (*offs)[5] = nullptr;
        ptrdiff_t stride;
        unsigned shift, shift2 = 0, mask;
        if (cls == 0) {
            const unsigned nonsq = tx >= TX_4X8;
            offs = k_lo_ctx_offsets[nonsq + (tx & nonsq)];
            stride = 4 * sh;
            shift = t.lh < 4 ? t.lh + 2 : 5;
            mask = 4 * sh - 1;
            memset(levels, 0, stride * (4 * sw + 2));
        } else if (cls == 1) {   // horizontal class
            stride = 16;
            shift = t.lh + 2;
            mask = 4 * sh - 1;
            memset(levels, 0, stride * (4 * sh + 2));
        } else {                 // vertical class
            stride = 16;
            shift = t.lw + 2;
            shift2 = t.lh + 2;
            mask = 4 * sw - 1;
            memset(levels, 0, stride * (4 * sw + 2));
        }
        auto pos = [&](unsigned i, unsigned &x, unsigned &y) -> unsigned {
            if (cls == 0) {
                const unsigned r = scan[i];
                x = r >> shift;
                y = r & mask;
                return r;
            }
            x = i & mask;
            y = i >> shift;
            return cls == 1 ? i : ((x << shift2) | y);
        };
        unsigned x, y;
        rc = pos(eob, x, y);
        if (eob_tok == 2) {
            ctx = (cls == 0 ? (x | y) > 1 : y != 0) ? 14 : 7;
            tok = m.hi_tok(hi_cdf[ctx]);
            level_tok = tok + (3 << 6);
        }
        cf[rc] = tok << 11;
        levels[x * stride + y] = (uint8_t)level_tok;
        for (int i = eob - 1; i > 0; i--) {
            const unsigned rci = pos(i, x, y);
            uint8_t *lv = levels + x * stride + y;
            ctx = lo_ctx(lv, cls, &mag, offs, x, y, stride);
            if (cls == 0) y |= x;
            tok = m.symbol(lo_cdf[ctx], 3);
            if (tok == 3) {
                mag &= 63;
                ctx = (y > (cls == 0 ? 1u : 0u) ? 14 : 7) + (mag > 12 ? 6 : (mag + 1) >> 1);
                tok = m.hi_tok(hi_cdf[ctx]);
                *lv = (uint8_t)(tok + (3 << 6));
                cf[rci] = (tok << 11) | rc;
                rc = rci;
            } else {
                *lv = (uint8_t)(tok * 0x41);
                if (tok) {
                    cf[rci] = (tok << 11) | rc;
                    rc = rci;
                } else {
                    cf[rci] = 0;
                }
            }
        }
        // dc
        ctx = cls == 0 ? 0 : lo_ctx(levels, cls, &mag, offs, 0, 0, stride);
        dc_tok = m.symbol(lo_cdf[ctx], 3);
        if (dc_tok == 3) {
            if (cls == 0) mag = levels[1] + levels[stride] + levels[stride + 1];
            mag &= 63;
            ctx = mag > 12 ? 6 : (mag + 1) >> 1;
            dc_tok = m.hi_tok(hi_cdf[ctx]);
        }
    } else {
        const int tok_br = m.symbol(eob_cdf[0], 2);
        dc_tok = 1 + tok_br;
        if (tok_br == 2) dc_tok = m.hi_tok(hi_cdf[0]);
        rc = 0;
    }

    // signs, Golomb remainders and dequantization (forward scan order through the rc links)
    const uint16_t *dq = ts->dq[b.seg_id][plane];
    const uint8_t *qm = (h.quant.qm && *txtp < IDTX)
                            ? qm_table(plane ? (plane == 1 ? h.quant.qm_u : h.quant.qm_v) : h.quant.qm_y, !!plane, tx)
                            : nullptr;
    const int dq_shift = imax(0, t.ctx - 2);
    const unsigned cf_max = ~(~127u << (s.bpc == 8 ? 8 : s.bpc));
    unsigned cul_level, dc_sign_level;
    if (!dc_tok) {
        cul_level = 0;
        dc_sign_level = 1 << 6;
    } else {
        const int dc_sign = m.bool_adapt(cc.dc_sign[chroma][dc_sign_ctx(t, actx, lctx)]);
        unsigned dc_dq = dq[0];
        dc_sign_level = (unsigned)(dc_sign - 1) & (2 << 6);
        if (qm) dc_dq = (dc_dq * qm[0] + 16) >> 5;
        if (dc_tok == 15) {
            dc_tok = m.golomb() + 15;
            dc_tok &= 0xfffff;
            dc_dq = ((dc_dq * dc_tok) & 0xffffff) >> dq_shift;
            dc_dq = dc_dq < cf_max + dc_sign ? dc_dq : cf_max + dc_sign;
        } else {
            dc_dq = (dc_dq * dc_tok) >> dq_shift;
            if (qm) dc_dq = dc_dq < cf_max + dc_sign ? dc_dq : cf_max + dc_sign;
        }
        cul_level = dc_tok;
        cf[0] = dc_sign ? -(int32_t)dc_dq : (int32_t)dc_dq;
    }
    if (rc) {
        const unsigned ac_dq = dq[1];
        do {
            const int sign = m.bool_equi();
            const unsigned rc_tok = (unsigned)cf[rc];
            unsigned tok, dqv = qm ? (ac_dq * qm[rc] + 16) >> 5 : ac_dq;
            if (rc_tok >= (15u << 11)) {
                tok = m.golomb() + 15;
                tok &= 0xfffff;
                dqv = ((dqv * tok) & 0xffffff) >> dq_shift;
                dqv = dqv < cf_max + sign ? dqv : cf_max + sign;
            } else {
                tok = rc_tok >> 11;
                dqv = (dqv * tok) >> dq_shift;
                if (qm) dqv = dqv < cf_max + sign ? dqv : cf_max + sign;
            }
            cul_level += tok;
            cf[rc] = sign ? -(int32_t)dqv : (int32_t)dqv;
            rc = rc_tok & 0x3ff;
        } while (rc);
    }
    *res_ctx = (uint8_t)(imin(cul_level, 63) | dc_sign_level);
    return eob;
}

// copy a decoded block into the frame's coefficient arena, return its offset in coefficients.
// A DC-only block (DCT_DCT with eob 0: itxfm_add's dc-only path reads and clears coefficient 0
// alone) keeps only its DC. Any other block (a 4x4 one only as int16) keeps only the corner
// of whole 4 x 4 groups that holds its non-zero coefficients, row-major, from a 4-coefficient
// boundary, as int16 where they fit (MI_TX_PACKED, MI_TX_I16 in *flags: the layout of
// include/mi_av1dsp.h): the arena the device
// path uploads and reads shrinks, and a transform row is a few vector loads. Other 4x4 blocks
// keep itxfm_add's layout (min(w,32) x min(h,32) column-major).
uint32_t FrameDec::store_coefs(const int32_t *cf, int tx, int txtp, int eob, uint8_t *flags) {
    const TxDim &t = k_txdim[tx];
    const int sw = imin(t.w * 4, 32), sh = imin(t.h * 4, 32);
    const int cb = s.bpc == 8 ? 2 : 4;
    *flags = 0;
    // a 4x4 block stays dense unless int16 storage halves it (10/12-bit)
    bool small_dense = sw * sh <= 16 && cb == 2;
    if (sw * sh <= 16 && !small_dense)
        for (int i = 0; i < 16; i++)
            if (cf[i] < -32768 || cf[i] > 32767) small_dense = true;
    if ((txtp == 0 && eob < 1) || small_dense) {
        const int n = txtp == 0 && eob < 1 ? 1 : sw * sh;
        const uint32_t off = (uint32_t)fw.ncoef;
        fw.coef.resize((fw.ncoef + n) * cb);
        if (cb == 2) {
            int16_t *d = reinterpret_cast<int16_t *>(fw.coef.data()) + off;
            for (int i = 0; i < n; i++) d[i] = (int16_t)cf[i];
        } else {
            memcpy(fw.coef.data() + (size_t)off * 4, cf, n * 4);
        }
        fw.ncoef += n;
        return off;
    }
    // the last column and the last row group holding a non-zero coefficient
    uint32_t rows = 0;   // bit y / 4: a non-zero in rows 4 (y / 4) .. + 3
    int lastx = -1;
    for (int x = 0; x < sw; x++) {
        const int32_t *c = cf + x * sh;
        uint32_t any = 0;
        for (int y = 0; y < sh; y += 4) {
            const uint32_t g = (uint32_t)(c[y] | c[y + 1] | c[y + 2] | c[y + 3]);
            any |= g;
            rows |= (uint32_t)(g != 0) << (y >> 2);
        }
        if (any) lastx = x;
    }
    const int cw = lastx < 0 ? 4 : ((lastx >> 2) + 1) * 4;
    const int ch = rows ? (32 - __builtin_clz(rows)) * 4 : 4;
    *flags = MI_TX_PACK(cw, ch);
    // 10/12-bit: int16 storage when every coefficient of the corner fits (MI_TX_I16)
    bool i16 = cb == 2;
    if (!i16) {
        int32_t lo = 0, hi = 0;
        for (int x = 0; x < cw; x++)
            for (int y = 0; y < ch; y++) {
                lo = imin(lo, cf[y + x * sh]);
                hi = imax(hi, cf[y + x * sh]);
            }
        i16 = lo >= -32768 && hi <= 32767;
        if (i16) *flags |= MI_TX_I16;
    }
    const size_t pad = (4 - (fw.ncoef & 3)) & 3;
    const uint32_t off = (uint32_t)(fw.ncoef + pad);
    const int n = cw * ch, slots = cb == 4 && i16 ? n / 2 : n;
    fw.coef.resize((off + slots) * cb, 0);
    if (i16) {
        int16_t *d = reinterpret_cast<int16_t *>(fw.coef.data() + (size_t)off * cb);
        for (int y = 0; y < ch; y++)
            for (int x = 0; x < cw; x++) d[y * cw + x] = (int16_t)cf[y + x * sh];
        fw.ncoef = off + slots;
        return off;
    }
    {
        int32_t *d = reinterpret_cast<int32_t *>(fw.coef.data()) + off;
        for (int y = 0; y < ch; y++)
            for (int x = 0; x < cw; x++) d[y * cw + x] = cf[y + x * sh];
    }
    fw.ncoef = off + n;
    return off;
}

// ------------------------------------------------------------------------------------------
// palette (recon.rs read_pal_plane / read_pal_uv, decode.rs read_pal_indices)

void FrameDec::read_pal_plane(Block &b, int pl, int sz_ctx, int bx4, int by4, uint16_t *pal) {
    Msac &m = ts->msac;
    const int pal_sz = b.pal_sz[pl] = m.symbol(ts->cdf.m.pal_sz[pl][sz_ctx], 6) + 2;
    uint16_t cache[16], used_cache[8];
    int l_cache = pl ? pal_sz_uv[1][by4] : l.pal_sz[by4];
    int n_cache = 0;
    int a_cache = (by4 & 15) ? (pl ? pal_sz_uv[0][bx4] : a.pal_sz[bx]) : 0;
    const uint16_t *lp = al_pal[1][by4][pl], *ap = al_pal[0][bx4][pl];
    while (l_cache && a_cache) {
        if (*lp < *ap) {
            if (!n_cache || cache[n_cache - 1] != *lp) cache[n_cache++] = *lp;
            lp++;
            l_cache--;
        } else {
            if (*ap == *lp) {
                lp++;
                l_cache--;
            }
            if (!n_cache || cache[n_cache - 1] != *ap) cache[n_cache++] = *ap;
            ap++;
            a_cache--;
        }
    }
    for (; l_cache > 0; l_cache--, lp++)
        if (!n_cache || cache[n_cache - 1] != *lp) cache[n_cache++] = *lp;
    for (; a_cache > 0; a_cache--, ap++)
        if (!n_cache || cache[n_cache - 1] != *ap) cache[n_cache++] = *ap;
    int i = 0;
    for (int n = 0; n < n_cache && i < pal_sz; n++)
        if (m.bool_equi()) used_cache[i++] = cache[n];
    const int n_used = i;
    if (i < pal_sz) {
        const int bpc = s.bpc;
        int prev = pal[i++] = (uint16_t)m.bools(bpc);
        if (i < pal_sz) {
            int bits = bpc - 3 + m.bools(2);
            const int mx = (1 << bpc) - 1;
            do {
                const int delta = m.bools(bits);
                prev = pal[i++] = (uint16_t)imin(prev + delta + !pl, mx);
                if (prev + !pl >= mx) {
                    for (; i < pal_sz; i++) pal[i] = (uint16_t)mx;
                    break;
                }
                bits = imin(bits, 1 + ulog2(mx - prev - !pl));
            } while (i < pal_sz);
        }
        int n = 0, k = n_used;
        uint16_t merged[8];
        for (i = 0; i < pal_sz; i++) {
            if (n < n_used && (k >= pal_sz || used_cache[n] <= pal[k])) merged[i] = used_cache[n++];
            else merged[i] = pal[k++];
        }
        memcpy(pal, merged, pal_sz * 2);
    } else {
        memcpy(pal, used_cache, n_used * 2);
    }
}

void FrameDec::read_pal_uv(Block &b, int sz_ctx, int bx4, int by4, uint16_t (*pal)[8]) {
    read_pal_plane(b, 1, sz_ctx, bx4, by4, pal[1]);
    Msac &m = ts->msac;
    const int bpc = s.bpc;
    uint16_t *v = pal[2];
    if (m.bool_equi()) {
        const int bits = bpc - 4 + m.bools(2);
        int prev = v[0] = (uint16_t)m.bools(bpc);
        const int mx = (1 << bpc) - 1;
        for (int i = 1; i < b.pal_sz[1]; i++) {
            int delta = m.bools(bits);
            if (delta && m.bool_equi()) delta = -delta;
            prev = v[i] = (uint16_t)((prev + delta) & mx);
        }
    } else {
        for (int i = 0; i < b.pal_sz[1]; i++) v[i] = (uint16_t)m.bools(bpc);
    }
}

// decode.rs order_palette + read_pal_indices (C decode.c:381-477): anti-diagonal order with
// a colour-order context from the top, left and top-left indices
void FrameDec::read_pal_indices(uint8_t *idx, const Block &b, int pl, int w4_, int h4_, int bw4, int bh4) {
    Msac &m = ts->msac;
    const ptrdiff_t stride = bw4 * 4;
    const int n = b.pal_sz[pl];
    idx[0] = (uint8_t)m.uniform(n);
    uint16_t (*cdf)[8] = ts->cdf.m.color_map[pl][n - 2];
    for (int i = 1; i < 4 * (w4_ + h4_) - 1; i++) {
        const int first = imin(i, w4_ * 4 - 1), last = imax(0, i - h4_ * 4 + 1);
        for (int j = first; j >= last; j--) {
            const int yy = i - j, xx = j;
            uint8_t *p = idx + yy * stride + xx;
            const int have_top = yy > 0, have_left = xx > 0;
            uint8_t order[8];
            unsigned used = 0;
            int o = 0, ctx;
            auto add = [&](int v) {
                order[o++] = (uint8_t)v;
                used |= 1u << v;
            };
            if (!have_left) {
                ctx = 0;
                add(p[-stride]);
            } else if (!have_top) {
                ctx = 0;
                add(p[-1]);
            } else {
                const int lv = p[-1], tv = p[-stride], tl = p[-stride - 1];
                const int st_l = tv == lv, st_tl = tv == tl, sl_tl = lv == tl;
                if (st_l && st_tl && sl_tl) {
                    ctx = 4;
                    add(tv);
                } else if (st_l) {
                    ctx = 3;
                    add(tv);
                    add(tl);
                } else if (st_tl || sl_tl) {
                    ctx = 2;
                    add(tl);
                    add(st_tl ? lv : tv);
                } else {
                    ctx = 1;
                    add(imin(tv, lv));
                    add(imax(tv, lv));
                    add(tl);
                }
            }
            for (int c = 0; c < 8; c++)
                if (!(used & (1u << c))) order[o++] = (uint8_t)c;
            *p = order[m.symbol(cdf[ctx], n - 1)];
        }
    }
    if (bw4 > w4_)
        for (int y = 0; y < 4 * h4_; y++)
            memset(idx + y * stride + 4 * w4_, idx[y * stride + 4 * w4_ - 1], 4 * (bw4 - w4_));
    if (h4_ < bh4)
        for (int y = 4 * h4_; y < bh4 * 4; y++) memcpy(idx + y * stride, idx + (4 * h4_ - 1) * stride, bw4 * 4);
}

// ------------------------------------------------------------------------------------------
// loop-filter masks (lf_mask.rs mask_edges_intra / mask_edges_chroma / create_lf_mask_intra;
// C lf_mask.c:134-336)

void FrameDec::mask_edges_intra(int by4, int bx4, int w4_, int h4_, int tx, uint8_t *actx, uint8_t *lctx,
                                uint16_t (*masks)[32][3][2]) {
    const TxDim &t = k_txdim[tx];
    const int twl4c = imin(2, t.lw), thl4c = imin(2, t.lh);
    unsigned mask = 1u << by4;
    for (int y = 0; y < h4_; y++, mask <<= 1) {
        const int sidx = mask >= 0x10000;
        masks[0][bx4][imin(twl4c, lctx[y])][sidx] |= (uint16_t)(mask >> (sidx << 4));
    }
    mask = 1u << bx4;
    for (int x = 0; x < w4_; x++, mask <<= 1) {
        const int sidx = mask >= 0x10000;
        masks[1][by4][imin(thl4c, actx[x])][sidx] |= (uint16_t)(mask >> (sidx << 4));
    }
    unsigned tt = 1u << by4;
    unsigned inner = (unsigned)((((uint64_t)tt) << h4_) - tt);
    unsigned in1 = inner & 0xffff, in2 = inner >> 16;
    for (int x = t.w; x < w4_; x += t.w) {
        if (in1) masks[0][bx4 + x][twl4c][0] |= (uint16_t)in1;
        if (in2) masks[0][bx4 + x][twl4c][1] |= (uint16_t)in2;
    }
    tt = 1u << bx4;
    inner = (unsigned)((((uint64_t)tt) << w4_) - tt);
    in1 = inner & 0xffff;
    in2 = inner >> 16;
    for (int y = t.h; y < h4_; y += t.h) {
        if (in1) masks[1][by4 + y][thl4c][0] |= (uint16_t)in1;
        if (in2) masks[1][by4 + y][thl4c][1] |= (uint16_t)in2;
    }
    memset(actx, thl4c, w4_);
    memset(lctx, twl4c, h4_);
}

void FrameDec::mask_edges_chroma(int cby4, int cbx4, int cw4, int ch4, int skip_inter, int tx, uint8_t *actx,
                                 uint8_t *lctx, uint16_t (*masks)[32][2][2]) {
    const TxDim &t = k_txdim[tx];
    const int twl4c = !!t.lw, thl4c = !!t.lh;
    const int vbits = 4 - ss_ver, hbits = 4 - ss_hor;
    const int vmask = 16 >> ss_ver, hmask = 16 >> ss_hor;
    const unsigned vmax = 1u << vmask, hmax = 1u << hmask;
    unsigned mask = 1u << cby4;
    for (int y = 0; y < ch4; y++, mask <<= 1) {
        const int sidx = mask >= vmax;
        masks[0][cbx4][imin(twl4c, lctx[y])][sidx] |= (uint16_t)(mask >> (sidx << vbits));
    }
    mask = 1u << cbx4;
    for (int x = 0; x < cw4; x++, mask <<= 1) {
        const int sidx = mask >= hmax;
        masks[1][cby4][imin(thl4c, actx[x])][sidx] |= (uint16_t)(mask >> (sidx << hbits));
    }
    if (!skip_inter) {
        unsigned tt = 1u << cby4;
        unsigned inner = (unsigned)((((uint64_t)tt) << ch4) - tt);
        unsigned in1 = inner & ((1u << vmask) - 1), in2 = inner >> vmask;
        for (int x = t.w; x < cw4; x += t.w) {
            if (in1) masks[0][cbx4 + x][twl4c][0] |= (uint16_t)in1;
            if (in2) masks[0][cbx4 + x][twl4c][1] |= (uint16_t)in2;
        }
        tt = 1u << cbx4;
        inner = (unsigned)((((uint64_t)tt) << cw4) - tt);
        in1 = inner & ((1u << hmask) - 1);
        in2 = inner >> hmask;
        for (int y = t.h; y < ch4; y += t.h) {
            if (in1) masks[1][cby4 + y][thl4c][0] |= (uint16_t)in1;
            if (in2) masks[1][cby4 + y][thl4c][1] |= (uint16_t)in2;
        }
    }
    memset(actx, thl4c, cw4);
    memset(lctx, twl4c, ch4);
}

void FrameDec::create_lf_mask_intra(const Block &b, int has_chroma) {
    const uint8_t (*fl)[8][2] = ts->lflvl.v[b.seg_id];
    const BlockDim &bd = k_bdim[b.bs];
    const int bw4 = imin(w4 - bx, bd.w4), bh4 = imin(h4 - by, bd.h4);
    const int bx4 = bx & 31, by4 = by & 31;
    if (bw4 > 0 && bh4 > 0) {
        for (int y = 0; y < bh4; y++)
            for (int x = 0; x < bw4; x++) {
                uint8_t *lv = &mw.lf_level[(((size_t)(by + y) * b4_stride) + bx + x) * 4];
                lv[0] = fl[0][0][0];
                lv[1] = fl[1][0][0];
            }
        mask_edges_intra(by4, bx4, bw4, bh4, b.tx, &a.tx_lpf_y[bx], &l.tx_lpf_y[by4],
                         reinterpret_cast<uint16_t (*)[32][3][2]>(lf_mask->filter_y));
    }
    if (!has_chroma) return;
    const int cbw4 = imin(((w4 + ss_hor) >> ss_hor) - (bx >> ss_hor), (bd.w4 + ss_hor) >> ss_hor);
    const int cbh4 = imin(((h4 + ss_ver) >> ss_ver) - (by >> ss_ver), (bd.h4 + ss_ver) >> ss_ver);
    if (cbw4 <= 0 || cbh4 <= 0) return;
    for (int y = 0; y < cbh4; y++)
        for (int x = 0; x < cbw4; x++) {
            uint8_t *lv = &mw.lf_level[(((size_t)((by >> ss_ver) + y) * b4_stride) + (bx >> ss_hor) + x) * 4];
            lv[2] = fl[2][0][0];
            lv[3] = fl[3][0][0];
        }
    mask_edges_chroma(by4 >> ss_ver, bx4 >> ss_hor, cbw4, cbh4, 0, b.uvtx, &a.tx_lpf_uv[bx >> ss_hor],
                      &l.tx_lpf_uv[by4 >> ss_ver], reinterpret_cast<uint16_t (*)[32][2][2]>(lf_mask->filter_uv));
}

// ------------------------------------------------------------------------------------------
// intra work emission: one MiIntraBlock + MiTxBlock per transform block, in the order
// recon_b_intra predicts and adds them (C recon_tmpl.c:1200-1603), with the dependency list
// of the pixels its prediction reads

void FrameDec::add_deps(int plane, int x0, int y0, int x1, int y1, std::vector<int32_t> &out) {
    // pixel rectangle [x0, x1) x [y0, y1) of `plane`, 4x4 granular, inside the current tile:
    // prediction never reads across a tile edge (the edge flags stop at it; the top-left sample
    // is read only with both a left and a top neighbour), and the owners of other tiles' pixels
    // are indices into those tiles' lists
    const int sh = plane ? ss_hor : 0, sv = plane ? ss_ver : 0;
    x0 = imax(x0, (ts->col_start * 4) >> sh);
    y0 = imax(y0, (ts->row_start * 4) >> sv);
    const Span<int32_t> &o = owner[plane];
    // (the unit range clipped once; runs of units with one owner are checked once: an edge
    // mostly lies along few, large neighbours)
    const int ux0 = imax(x0 >> 2, 0), ux1 = imin((x1 + 3) >> 2, owner_stride);
    const int uy0 = imax(y0 >> 2, 0), uy1 = (y1 + 3) >> 2;
    // duplicates by a stamp per dependency list (a new list starts empty), not by scanning the
    // list: a CfL block's luma rectangle can hold hundreds of owners
    if (out.empty()) ++dep_stamp;
    int32_t last = -1;
    // a one-unit-wide column (a left edge) jumps over the rows its current owner covers: every
    // cell of a block's rectangle holds that block unless a later item overwrote it, which only
    // happens under an inter-intra item (MI_INTRA_II; its residual items follow it)
    const bool column = ux1 - ux0 == 1;
    for (int y = uy0; y < uy1; y++) {
        const size_t row = (size_t)y * owner_stride;
        if (row >= o.size()) break;
        const int xe = (int)std::min<size_t>((size_t)ux1, o.size() - row);
        for (int x = ux0; x < xe; x++) {
            const int32_t v = o[row + x];
            if (v < 0) continue;
            if (column && (size_t)v < fw.intra.size()) {
                const MiIntraBlock &ob = fw.intra[v];
                if (ob.plane == plane && !(ob.flags & MI_INTRA_II)) y = imax(y, ((ob.y + ob.h) >> 2) - 1);
            }
            if (v == last) continue;
            last = v;
            if ((size_t)v >= dep_seen.size()) dep_seen.resize(std::max<size_t>((size_t)v + 1, 2 * dep_seen.size()), 0);
            if (dep_seen[v] == dep_stamp) continue;
            dep_seen[v] = dep_stamp;
            out.push_back(v);
        }
    }
}

void FrameDec::emit_intra(const Block &b, int edge_flags, const uint8_t *pal_idx, const uint16_t (*pal)[8]) {
    const BlockDim &bd = k_bdim[b.bs];
    const int bw4 = bd.w4, bh4 = bd.h4;
    const int w4b = imin(bw4, bw - bx), h4b = imin(bh4, bh - by);
    const int cw4 = (w4b + ss_hor) >> ss_hor, ch4 = (h4b + ss_ver) >> ss_ver;
    const int cbw4 = (bw4 + ss_hor) >> ss_hor, cbh4 = (bh4 + ss_ver) >> ss_ver;
    const int has_chroma = layout != 0 && (bw4 > ss_hor || (bx & 1)) && (bh4 > ss_ver || (by & 1));
    const TxDim &t = k_txdim[b.tx];
    const TxDim &ut = k_txdim[b.uvtx];
    const int bx4 = bx & 31, by4 = by & 31, cbx4 = bx4 >> ss_hor, cby4 = by4 >> ss_ver;
    const int efilt = s.intra_edge_filter ? MI_INTRA_EDGE_FILTER : 0;
    auto sm = [](int m) { return m == SMOOTH_PRED || m == SMOOTH_V_PRED || m == SMOOTH_H_PRED; };
    const int sm_y = (a.intra[bx] && sm(a.mode[bx])) || (l.intra[by4] && sm(l.mode[by4]));
    const int sm_uv = has_chroma && (sm(a.uvmode[bx >> ss_hor]) || sm(l.uvmode[cby4]));
    int32_t cf[32 * 32];
    const int pb = s.bpc == 8 ? 1 : 2;

    auto push = [&](MiIntraBlock ib, int plane, int txs, int skip, uint8_t *actx, uint8_t *lctx, int nact, int nlct,
                    int intra_tx_eob_plane_bs) {
        (void)intra_tx_eob_plane_bs;
        // dependencies: every already reconstructed pixel the prediction may read
        const int k = (int)fw.intra.size();
        std::vector<int32_t> &deps = dep_tmp;
        deps.clear();
        const int x = ib.x, y = ib.y, w = ib.w, hh = ib.h;
        const int tile_w = ib.tile_w, tile_h = ib.tile_h;
        if (ib.mode == MI_IPRED_PAL) {
            // no neighbour pixels
        } else {
            if (ib.flags & MI_INTRA_HAVE_LEFT) add_deps(plane, x - 1, y, x, imin(y + 2 * hh, tile_h), deps);
            if (ib.flags & MI_INTRA_HAVE_TOP) add_deps(plane, x - 1, y - 1, imin(x + 2 * w, tile_w), y, deps);
            if ((ib.flags & MI_INTRA_HAVE_LEFT) && !(ib.flags & MI_INTRA_HAVE_TOP)) add_deps(plane, x - 1, y, x, y + 1, deps);
            if (ib.flags & MI_INTRA_CFL_AC) {
                const int ly0 = y << ss_ver, lx0 = x << ss_hor;
                add_deps(0, lx0, ly0, lx0 + (w << ss_hor), ly0 + (hh << ss_ver), deps);
            }
        }
        fw.intra.push_back(ib);
        fw.dep_start.push_back((int32_t)fw.deps.size());
        for (int32_t d : deps) fw.deps.push_back(d);
        // residual
        MiTxBlock tb{};
        tb.x = ib.x;
        tb.y = ib.y;
        tb.plane = (uint8_t)plane;
        tb.tx = (uint8_t)txs;
        tb.eob = -1;
        if (!skip) {
            int txtp = 0;
            uint8_t res;
            // decode_coefs writes scan positions of the transform's coded area only
            memset(cf, 0, sizeof(int32_t) * imin(k_txdim[txs].w * 4, 32) * imin(k_txdim[txs].h * 4, 32));
            const int eob = decode_coefs(actx, lctx, txs, b.bs, b, 1, plane, cf, &txtp, &res);
            memset(actx, res, nact);
            memset(lctx, res, nlct);
            tb.txtp = (uint8_t)txtp;
            tb.eob = eob;
            if (eob >= 0) tb.coef_off = store_coefs(cf, txs, txtp, eob, &tb.flags);
        } else {
            memset(actx, 0x40, nact);
            memset(lctx, 0x40, nlct);
        }
        fw.intra_tx.push_back(tb);
        // ownership of the written pixels
        Span<int32_t> &o = owner[plane];
        for (int yy = y >> 2; yy < (y + hh) >> 2; yy++)
            for (int xx = x >> 2; xx < (x + w) >> 2; xx++) o[(size_t)yy * owner_stride + xx] = k;
    };

    for (int init_y = 0; init_y < h4b; init_y += 16) {
        const int sub_h4 = imin(h4b, 16 + init_y);
        const int sub_ch4 = imin(ch4, (init_y + 16) >> ss_ver);
        for (int init_x = 0; init_x < w4b; init_x += 16) {
            const int sb_has_tr = init_x + 16 < w4b ? 1 : init_y ? 0 : (edge_flags & E444_TR) != 0;
            const int sb_has_bl = init_x ? 0 : init_y + 16 < h4b ? 1 : (edge_flags & E444_BL) != 0;
            const int sub_w4 = imin(w4b, init_x + 16);
            for (int y = init_y; y < sub_h4; y += t.h) {
                for (int x = init_x; x < sub_w4; x += t.w) {
                    const int tbx = bx + x, tby = by + y;
                    MiIntraBlock ib{};
                    ib.x = (uint16_t)(tbx * 4);
                    ib.y = (uint16_t)(tby * 4);
                    ib.w = (uint8_t)(t.w * 4);
                    ib.h = (uint8_t)(t.h * 4);
                    ib.plane = 0;
                    ib.tile_w = (uint16_t)(ts->col_end * 4);
                    ib.tile_h = (uint16_t)(ts->row_end * 4);
                    ib.max_w = (uint16_t)(4 * bw - 4 * tbx);
                    ib.max_h = (uint16_t)(4 * bh - 4 * tby);
                    if (b.pal_sz[0]) {
                        ib.mode = MI_IPRED_PAL;
                        ib.pal_off = (uint32_t)(fw.pal.size() / pb);
                        for (int i = 0; i < 8; i++) {
                            const uint16_t v = pal[0][i];
                            if (pb == 1) fw.pal.push_back((uint8_t)v);
                            else { fw.pal.push_back(v & 0xff); fw.pal.push_back(v >> 8); }
                        }
                        ib.aux_off = (uint32_t)fw.idx.size();
                        for (int yy = 0; yy < t.h * 4; yy++)
                            for (int xx = 0; xx < t.w * 4; xx++)
                                fw.idx.push_back(pal_idx[(y * 4 + yy) * (bw4 * 4) + x * 4 + xx]);
                    } else {
                        const int tr = ((y > init_y || !sb_has_tr) && (x + t.w >= sub_w4)) ? 0 : 1;
                        const int blf = (x > init_x || (!sb_has_bl && y + t.h >= sub_h4)) ? 0 : 1;
                        ib.flags = (uint8_t)((tbx > ts->col_start ? MI_INTRA_HAVE_LEFT : 0) |
                                             (tby > ts->row_start ? MI_INTRA_HAVE_TOP : 0) |
                                             (tr ? MI_INTRA_TOP_RIGHT : 0) | (blf ? MI_INTRA_BOTTOM_LEFT : 0) |
                                             (sm_y ? MI_INTRA_SMOOTH_NB : 0) | efilt);
                        if (b.y_mode == FILTER_PRED) {
                            ib.mode = 13;
                            ib.filt_idx = (uint8_t)b.y_angle;
                        } else {
                            ib.mode = (uint8_t)b.y_mode;
                            ib.angle = (int8_t)b.y_angle;
                        }
                    }
                    const int nact = imin(t.w, bw - tbx), nlct = imin(t.h, bh - tby);
                    push(ib, 0, b.tx, b.skip, &a.lcoef[tbx], &l.lcoef[by4 + y], nact, nlct, 0);
                }
            }
            if (!has_chroma) continue;
            const int uv_sb_has_tr = ((init_x + 16) >> ss_hor) < cw4 ? 1 : init_y ? 0 :
                                     (edge_flags & (E420_TR >> (layout - 1))) != 0;
            const int uv_sb_has_bl = init_x ? 0 : ((init_y + 16) >> ss_ver) < ch4 ? 1 :
                                     (edge_flags & (E420_BL >> (layout - 1))) != 0;
            const int sub_cw4 = imin(cw4, (init_x + 16) >> ss_hor);
            const int cfl = b.uv_mode == CFL_PRED;
            int furthest_r = 0, furthest_b = 0;
            if (cfl) {
                furthest_r = ((cw4 << ss_hor) + t.w - 1) & ~(t.w - 1);
                furthest_b = ((ch4 << ss_ver) + t.h - 1) & ~(t.h - 1);
            }
            for (int pl = 0; pl < 2; pl++) {
                for (int y = init_y >> ss_ver; y < sub_ch4; y += ut.h) {
                    for (int x = init_x >> ss_hor; x < sub_cw4; x += ut.w) {
                        // luma-unit position of this chroma transform block (as t->bx / t->by)
                        const int tbx = bx + (x << ss_hor), tby = by + (y << ss_ver);
                        const int cx = (bx >> ss_hor) + x, cy = (by >> ss_ver) + y;   // chroma 4x4 units
                        MiIntraBlock ib{};
                        ib.x = (uint16_t)(cx * 4);
                        ib.y = (uint16_t)(cy * 4);
                        ib.w = (uint8_t)(ut.w * 4);
                        ib.h = (uint8_t)(ut.h * 4);
                        ib.plane = (uint8_t)(1 + pl);
                        ib.tile_w = (uint16_t)((ts->col_end >> ss_hor) * 4);
                        ib.tile_h = (uint16_t)((ts->row_end >> ss_ver) * 4);
                        ib.max_w = (uint16_t)((4 * bw + ss_hor - 4 * (tbx & ~ss_hor)) >> ss_hor);
                        ib.max_h = (uint16_t)((4 * bh + ss_ver - 4 * (tby & ~ss_ver)) >> ss_ver);
                        const int xstart = ts->col_start >> ss_hor, ystart = ts->row_start >> ss_ver;
                        const int have = ((tbx >> ss_hor) > xstart ? MI_INTRA_HAVE_LEFT : 0) |
                                         ((tby >> ss_ver) > ystart ? MI_INTRA_HAVE_TOP : 0);
                        if (b.pal_sz[1]) {
                            ib.mode = MI_IPRED_PAL;
                            ib.pal_off = (uint32_t)(fw.pal.size() / pb);
                            for (int i = 0; i < 8; i++) {
                                const uint16_t v = pal[1 + pl][i];
                                if (pb == 1) fw.pal.push_back((uint8_t)v);
                                else { fw.pal.push_back(v & 0xff); fw.pal.push_back(v >> 8); }
                            }
                            ib.aux_off = (uint32_t)fw.idx.size();
                            const uint8_t *ci = pal_idx + bw4 * bh4 * 16;
                            for (int yy = 0; yy < ut.h * 4; yy++)
                                for (int xx = 0; xx < ut.w * 4; xx++)
                                    fw.idx.push_back(ci[(y * 4 + yy) * (cbw4 * 4) + x * 4 + xx]);
                        } else if (cfl && b.cfl_alpha[pl]) {
                            ib.mode = MI_IPRED_CFL;
                            ib.alpha = (int8_t)b.cfl_alpha[pl];
                            ib.flags = (uint8_t)(have | MI_INTRA_CFL_AC);
                            ib.reserved = (uint32_t)((cbw4 - (furthest_r >> ss_hor)) |
                                                     ((cbh4 - (furthest_b >> ss_ver)) << 8) | (ss_hor << 16) |
                                                     (ss_ver << 17));
                        } else {
                            const int tr = ((y > (init_y >> ss_ver) || !uv_sb_has_tr) && (x + ut.w >= sub_cw4)) ? 0 : 1;
                            const int blf = (x > (init_x >> ss_hor) || (!uv_sb_has_bl && y + ut.h >= sub_ch4)) ? 0 : 1;
                            ib.flags = (uint8_t)(have | (tr ? MI_INTRA_TOP_RIGHT : 0) | (blf ? MI_INTRA_BOTTOM_LEFT : 0) |
                                                 (sm_uv ? MI_INTRA_SMOOTH_NB : 0) | efilt);
                            ib.mode = (uint8_t)(cfl ? DC_PRED : b.uv_mode);
                            ib.angle = (int8_t)b.uv_angle;
                        }
                        const int nact = imin(ut.w, (bw - tbx + ss_hor) >> ss_hor);
                        const int nlct = imin(ut.h, (bh - tby + ss_ver) >> ss_ver);
                        push(ib, 1 + pl, b.uvtx, b.skip, &a.ccoef[pl][cx], &l.ccoef[pl][cby4 + y], nact, nlct, 0);
                    }
                }
            }
        }
    }
    (void)cbx4;
}

// ------------------------------------------------------------------------------------------
// blocks (decode.rs decode_b; C decode.c:723-2116), intra frames

// ---- intra block copy ----------------------------------------------------------------------

static const Mv kInvalidMv = { INT16_MIN, INT16_MIN };   // refmvs INVALID_MV: an intra block

// refmvs splat_mv (refmvs.rs; C refmvs.c:909-917): the block's entry over its bw4 x bh4 units
void FrameDec::splat(const RefMvBlock &r, int bw4, int bh4) {
    for (int y = 0; y < bh4; y++) {
        RefMvBlock *row = &rmv_at(by + y, bx);
        for (int x = 0; x < bw4; x++) row[x] = r;
    }
}

// splat_intrabc_mv / splat_intraref (decode.rs; C decode.c:570-614)
void FrameDec::splat_rmv(int bs, int bw4, int bh4, Mv mv, bool valid) {
    RefMvBlock r{};
    r.mv[0] = valid ? mv : kInvalidMv;
    r.mv[1] = Mv{ 0, 0 };
    r.ref[0] = 0;
    r.ref[1] = -1;
    r.bs = (uint8_t)bs;
    r.mf = 0;
    splat(r, bw4, bh4);
}

// rav1d_refmvs_find (refmvs.rs; C refmvs.c dav1d_refmvs_find) for ref = {INTRA_FRAME, none}:
// the spatial candidates only (intra frames carry no temporal MVs), weights, the two-stage sort
// and the clamp; stack[0..1] are the first two candidates (zero where there are fewer).
void FrameDec::find_dv(int bs, int edge_flags, Mv stack[2]) {
    struct Cand { Mv mv; int weight; } st[9];
    int cnt = 0;
    const int bw4 = k_bdim[bs].w4, bh4 = k_bdim[bs].h4;
    const int w4c = imin(imin(bw4, 16), ts->col_end - bx), h4c = imin(imin(bh4, 16), ts->row_end - by);
    auto add = [&](const RefMvBlock &c, int weight, int *have_refmv) {
        if (c.mv[0] == kInvalidMv) return;             // intra block (no block copy)
        if (c.ref[0] != 0) return;
        *have_refmv = 1;
        for (int m = 0; m < cnt; m++)
            if (st[m].mv == c.mv[0]) {
                st[m].weight += weight;
                return;
            }
        if (cnt < 8) st[cnt++] = { c.mv[0], weight };
    };
    // scan_row / scan_col: weights by the first candidate's extent, then per candidate
    auto scan_row = [&](int y4, int x4, int max_rows, int step, int *have) -> int {
        const RefMvBlock *b0 = &rmv_at(y4, x4);
        const int cbw = k_bdim[b0->bs].w4;
        int len = imax(step, imin(bw4, cbw));
        if (bw4 <= cbw) {
            const int weight = bw4 == 1 ? 2 : imax(2, imin(2 * max_rows, (int)k_bdim[b0->bs].h4));
            add(*b0, len * weight, have);
            return weight >> 1;
        }
        for (int x = 0;;) {
            add(rmv_at(y4, x4 + x), len * 2, have);
            x += len;
            if (x >= w4c) return 1;
            len = imax(step, (int)k_bdim[rmv_at(y4, x4 + x).bs].w4);
        }
    };
    auto scan_col = [&](int y4, int x4, int max_cols, int step, int *have) -> int {
        const RefMvBlock *b0 = &rmv_at(y4, x4);
        const int cbh = k_bdim[b0->bs].h4;
        int len = imax(step, imin(bh4, cbh));
        if (bh4 <= cbh) {
            const int weight = bh4 == 1 ? 2 : imax(2, imin(2 * max_cols, (int)k_bdim[b0->bs].w4));
            add(*b0, len * weight, have);
            return weight >> 1;
        }
        for (int y = 0;;) {
            add(rmv_at(y4 + y, x4), len * 2, have);
            y += len;
            if (y >= h4c) return 1;
            len = imax(step, (int)k_bdim[rmv_at(y4 + y, x4).bs].h4);
        }
    };
    int have_row = 0, have_col = 0, dummy = 0;
    unsigned max_rows = 0, n_rows = ~0u, max_cols = 0, n_cols = ~0u;
    if (by > ts->row_start) {
        max_rows = imin((by - ts->row_start + 1) >> 1, 2 + (bh4 > 1));
        n_rows = scan_row(by - 1, bx, max_rows, bw4 >= 16 ? 4 : 1, &have_row);
    }
    if (bx > ts->col_start) {
        max_cols = imin((bx - ts->col_start + 1) >> 1, 2 + (bw4 > 1));
        n_cols = scan_col(by, bx - 1, max_cols, bh4 >= 16 ? 4 : 1, &have_col);
    }
    if (n_rows != ~0u && (edge_flags & E444_TR) && imax(bw4, bh4) <= 16 && bw4 + bx < ts->col_end)
        add(rmv_at(by - 1, bx + bw4), 4, &have_row);
    const int nearest_cnt = cnt;
    for (int n = 0; n < nearest_cnt; n++) st[n].weight += 640;
    if ((n_rows | n_cols) != ~0u) add(rmv_at(by - 1, bx - 1), 4, &have_row);
    for (int n = 2; n <= 3; n++) {
        if ((unsigned)n > n_rows && (unsigned)n <= max_rows)
            n_rows += scan_row(((by - 2 * n + 1) | 1), bx | 1, 1 + max_rows - n, bw4 >= 16 ? 4 : 2, &have_row);
        if ((unsigned)n > n_cols && (unsigned)n <= max_cols)
            n_cols += scan_col(by | 1, (bx - n * 2 + 1) | 1, 1 + max_cols - n, bh4 >= 16 ? 4 : 2, &have_col);
    }
    (void)dummy;
    // bubble sorts: the nearest candidates, then the rest (stable for equal weights)
    for (int len = nearest_cnt; len;) {
        int last = 0;
        for (int n = 1; n < len; n++)
            if (st[n - 1].weight < st[n].weight) { std::swap(st[n - 1], st[n]); last = n; }
        len = last;
    }
    for (int len = cnt; len > nearest_cnt;) {
        int last = nearest_cnt;
        for (int n = nearest_cnt + 1; n < len; n++)
            if (st[n - 1].weight < st[n].weight) { std::swap(st[n - 1], st[n]); last = n; }
        len = last;
    }
    // clamp to the frame plus a 4-unit margin
    const int left = -(bx + bw4 + 4) * 4 * 8, right = (w4 - bx + 4) * 4 * 8;
    const int top = -(by + bh4 + 4) * 4 * 8, bottom = (h4 - by + 4) * 4 * 8;
    for (int n = 0; n < cnt; n++) {
        st[n].mv.x = (int16_t)iclip(st[n].mv.x, left, right);
        st[n].mv.y = (int16_t)iclip(st[n].mv.y, top, bottom);
    }
    for (int n = 0; n < 2; n++) stack[n] = n < cnt ? st[n].mv : Mv{ 0, 0 };
}

// read_mv_component_diff / read_mv_residual (decode.rs:224-311; C decode.c:76-139): have_fp = 0
// for block copies and force_integer_mv (fp = 3, hp = 1)
int FrameDec::read_mv_comp(CdfMvComp &c, int have_fp) {
    Msac &m = ts->msac;
    const int sign = m.bool_adapt(c.sign);
    const int cl = m.symbol(c.classes, 10);
    int up, fp = 3, hp = 1;
    if (!cl) {
        up = m.bool_adapt(c.class0);
        if (have_fp) {
            fp = m.symbol(c.class0_fp[up], 3);
            hp = h.hp ? m.bool_adapt(c.class0_hp) : 1;
        }
    } else {
        up = 1 << cl;
        for (int n = 0; n < cl; n++) up |= m.bool_adapt(c.classN[n]) << n;
        if (have_fp) {
            fp = m.symbol(c.classN_fp, 3);
            hp = h.hp ? m.bool_adapt(c.classN_hp) : 1;
        }
    }
    const int diff = ((up << 3) | (fp << 1) | hp) + 1;
    return sign ? -diff : diff;
}

void FrameDec::read_mv_residual(Mv &mv, CdfMv &cdf, int have_fp) {
    switch (ts->msac.symbol(ts->cdf.mv.joint, 3)) {   // the joint always comes from cdf.mv
    case 3:
        mv.y = (int16_t)(mv.y + read_mv_comp(cdf.comp[0], have_fp));
        mv.x = (int16_t)(mv.x + read_mv_comp(cdf.comp[1], have_fp));
        break;
    case 1: mv.x = (int16_t)(mv.x + read_mv_comp(cdf.comp[1], have_fp)); break;
    case 2: mv.y = (int16_t)(mv.y + read_mv_comp(cdf.comp[0], have_fp)); break;
    default: break;
    }
}

// read_tx_tree (decode.rs:313-372): split flags of the var-tx tree, contexts a.tx / l.tx
void FrameDec::read_tx_tree(int from, int depth, uint16_t *masks, int x_off, int y_off, int tbx, int tby) {
    const TxDim &t = k_txdim[from];
    const int txw = t.lw, txh = t.lh;
    const int tby4 = tby & 31;
    int is_split = 0;
    if (depth < 2 && from > TX_4X4) {
        const int cat = 2 * (TX_64X64 - t.max) - depth;
        const int ac = a.tx[tbx] < txw, lc = l.tx[tby4] < txh;
        is_split = ts->msac.bool_adapt(ts->cdf.m.txpart[cat][ac + lc]);
        if (is_split) masks[depth] |= (uint16_t)(1 << (y_off * 4 + x_off));
    }
    if (is_split && t.max > TX_8X8) {
        const int sub = t.sub;
        const int sw = k_txdim[sub].w, sh = k_txdim[sub].h;
        read_tx_tree(sub, depth + 1, masks, x_off * 2, y_off * 2, tbx, tby);
        if (txw >= txh && tbx + sw < bw) read_tx_tree(sub, depth + 1, masks, x_off * 2 + 1, y_off * 2, tbx + sw, tby);
        if (txh >= txw && tby + sh < bh) {
            read_tx_tree(sub, depth + 1, masks, x_off * 2, y_off * 2 + 1, tbx, tby + sh);
            if (txw >= txh && tbx + sw < bw)
                read_tx_tree(sub, depth + 1, masks, x_off * 2 + 1, y_off * 2 + 1, tbx + sw, tby + sh);
        }
    } else {
        setn(a.tx, tbx, t.w, is_split ? TX_4X4 : txw);
        setn(l.tx, tby4, t.h, is_split ? TX_4X4 : txh);
    }
}

// read_vartx_tree (decode.rs:770-851; C decode.c:479-532): max_ytx, uvtx and the split masks of
// an inter (or block copy) block
void FrameDec::read_vartx_tree(Block &b, int bs) {
    const BlockDim &bd = k_bdim[bs];
    const int bw4 = bd.w4, bh4 = bd.h4, by4 = by & 31;
    b.tx_split[0] = b.tx_split[1] = 0;
    b.max_ytx = k_max_tx_for_bs[bs][0];
    if (!b.skip && (h.seg.lossless[b.seg_id] || b.max_ytx == TX_4X4)) {
        b.max_ytx = b.uvtx = TX_4X4;
        if (h.txfm_mode == TXMODE_SWITCHABLE) {
            setn(a.tx, bx, bw4, TX_4X4);
            setn(l.tx, by4, bh4, TX_4X4);
        }
    } else if (h.txfm_mode != TXMODE_SWITCHABLE || b.skip) {
        if (h.txfm_mode == TXMODE_SWITCHABLE) {
            setn(a.tx, bx, bw4, bd.lw4);
            setn(l.tx, by4, bh4, bd.lh4);
        }
        b.uvtx = k_max_tx_for_bs[bs][layout];
    } else {
        const TxDim &yt = k_txdim[b.max_ytx];
        for (int yo = 0; yo < bh4 / yt.h; yo++)
            for (int xo = 0; xo < bw4 / yt.w; xo++)
                read_tx_tree(b.max_ytx, 0, b.tx_split, xo, yo, bx + xo * yt.w, by + yo * yt.h);
        b.uvtx = k_max_tx_for_bs[bs][layout];
    }
}

// One MI_INTRA_IBC work item: the block copy of one transform-sized piece (plane pixels px, py)
// and, unless the block is skipped, the residual read here (inter transform types)
void FrameDec::push_ibc(const Block &b, Mv mv, int plane, int tx, int tbx, int tby, int px, int py, int read,
                        uint8_t *actx, uint8_t *lctx, int nact, int nlct, int *txtp) {
    const TxDim &t = k_txdim[tx];
    const int sh = plane ? ss_hor : 0, sv = plane ? ss_ver : 0;
    MiIntraBlock ib{};
    ib.x = (uint16_t)px;
    ib.y = (uint16_t)py;
    ib.w = (uint8_t)(t.w * 4);
    ib.h = (uint8_t)(t.h * 4);
    ib.plane = (uint8_t)plane;
    ib.mode = MI_INTRA_IBC;
    ib.filt_idx = (uint8_t)(sh | (sv << 1));
    ib.reserved = (uint32_t)(uint16_t)mv.x | ((uint32_t)(uint16_t)mv.y << 16);
    ib.max_w = (uint16_t)((bw * 4) >> sh);
    ib.max_h = (uint16_t)((bh * 4) >> sv);
    ib.tile_w = (uint16_t)((ts->col_end >> sh) * 4);
    ib.tile_h = (uint16_t)((ts->row_end >> sv) * 4);
    // dependencies: the source rectangle (plus the second bilinear tap of a half-pel chroma
    // phase), clamped to the reference area as mc() replicates its border
    const int mx = (mv.x & (15 >> !sh)) << !sh, my = (mv.y & (15 >> !sv)) << !sv;
    const int dx = px + (mv.x >> (3 + sh)), dy = py + (mv.y >> (3 + sv));
    const int x0 = iclip(dx, 0, ib.max_w - 1), x1 = iclip(dx + ib.w + (mx != 0), 1, ib.max_w);
    const int y0 = iclip(dy, 0, ib.max_h - 1), y1 = iclip(dy + ib.h + (my != 0), 1, ib.max_h);
    std::vector<int32_t> &deps = dep_tmp;
    deps.clear();
    add_deps(plane, x0, y0, imax(x1, x0 + 1), imax(y1, y0 + 1), deps);
    const int k = (int)fw.intra.size();
    fw.intra.push_back(ib);
    fw.dep_start.push_back((int32_t)fw.deps.size());
    for (int32_t d : deps) fw.deps.push_back(d);
    MiTxBlock tb{};
    tb.x = ib.x;
    tb.y = ib.y;
    tb.plane = (uint8_t)plane;
    tb.tx = (uint8_t)tx;
    tb.eob = -1;
    if (read) {
        int32_t cf[32 * 32];
        memset(cf, 0, sizeof(int32_t) * imin(t.w * 4, 32) * imin(t.h * 4, 32));
        uint8_t res;
        const int eob = decode_coefs(actx, lctx, tx, b.bs, b, 0, plane, cf, txtp, &res);
        memset(actx, res, nact);
        memset(lctx, res, nlct);
        tb.txtp = (uint8_t)*txtp;
        tb.eob = eob;
        if (eob >= 0) tb.coef_off = store_coefs(cf, tx, *txtp, eob, &tb.flags);
    }
    fw.intra_tx.push_back(tb);
    Span<int32_t> &o = owner[plane];
    for (int yy = py >> 2; yy < (py + ib.h) >> 2; yy++)
        for (int xx = px >> 2; xx < (px + ib.w) >> 2; xx++) {
            const size_t q = (size_t)yy * owner_stride + xx;
            if (xx < owner_stride && q < o.size()) o[q] = k;
        }
    (void)tbx; (void)tby;
}

// read_coef_tree (recon.rs:1597-1800) for a block copy: the leaves of the var-tx tree
void FrameDec::ibc_residual_tree(const Block &b, Mv mv, int tx, int depth, const uint16_t *split, int x_off,
                                 int y_off, int tbx, int tby, uint8_t (*txtp_map)[32]) {
    const TxDim &t = k_txdim[tx];
    if (depth < 2 && split[depth] && (split[depth] & (1 << (y_off * 4 + x_off)))) {
        const int sub = t.sub, sw = k_txdim[sub].w, sh = k_txdim[sub].h;
        ibc_residual_tree(b, mv, sub, depth + 1, split, x_off * 2, y_off * 2, tbx, tby, txtp_map);
        if (t.w >= t.h && tbx + sw < bw)
            ibc_residual_tree(b, mv, sub, depth + 1, split, x_off * 2 + 1, y_off * 2, tbx + sw, tby, txtp_map);
        if (t.h >= t.w && tby + sh < bh) {
            ibc_residual_tree(b, mv, sub, depth + 1, split, x_off * 2, y_off * 2 + 1, tbx, tby + sh, txtp_map);
            if (t.w >= t.h && tbx + sw < bw)
                ibc_residual_tree(b, mv, sub, depth + 1, split, x_off * 2 + 1, y_off * 2 + 1, tbx + sw, tby + sh, txtp_map);
        }
        return;
    }
    const int tby4 = tby & 31, tbx4 = tbx & 31;
    int txtp = 0;
    push_ibc(b, mv, 0, tx, tbx, tby, tbx * 4, tby * 4, 1, &a.lcoef[tbx], &l.lcoef[tby4], imin(t.w, bw - tbx),
             imin(t.h, bh - tby), &txtp);
    for (int y = 0; y < t.h && tby4 + y < 32; y++)
        for (int x = 0; x < t.w && tbx4 + x < 32; x++) txtp_map[tby4 + y][tbx4 + x] = (uint8_t)txtp;
}

// decode.rs:1988-2135 (intra block copy) + rav1d_read_coef_blocks' inter walk (recon.rs:1803-2010)
int FrameDec::decode_ibc(Block &b, int bs, int edge_flags, int has_chroma) {
    const BlockDim &bd = k_bdim[bs];
    const int bw4 = bd.w4, bh4 = bd.h4;
    const int bx4 = bx & 31, by4 = by & 31;
    // DV prediction and residual
    Mv stack[2];
    find_dv(bs, edge_flags, stack);
    Mv mv;
    if (!(stack[0] == Mv{ 0, 0 })) mv = stack[0];
    else if (!(stack[1] == Mv{ 0, 0 })) mv = stack[1];
    else if (by - (16 << s.sb128) < ts->row_start) mv = Mv{ 0, (int16_t)(-(512 << s.sb128) - 2048) };
    else mv = Mv{ (int16_t)(-(512 << s.sb128)), 0 };
    read_mv_residual(mv, ts->cdf.dmv, 0);
    // keep the source inside the decoded part of the tile, outside the current superblock
    int border_left = ts->col_start * 4, border_top = ts->row_start * 4;
    if (has_chroma) {
        if (bw4 < 2 && ss_hor) border_left += 4;
        if (bh4 < 2 && ss_ver) border_top += 4;
    }
    int src_left = bx * 4 + (mv.x >> 3), src_top = by * 4 + (mv.y >> 3);
    int src_right = src_left + bw4 * 4, src_bottom = src_top + bh4 * 4;
    const int border_right = ((ts->col_end + (bw4 - 1)) & ~(bw4 - 1)) * 4;
    if (src_left < border_left) { src_right += border_left - src_left; src_left = border_left; }
    else if (src_right > border_right) { src_left -= src_right - border_right; src_right = border_right; }
    if (src_top < border_top) { src_bottom += border_top - src_top; src_top = border_top; }
    const int sbx = (bx >> (4 + s.sb128)) << (6 + s.sb128), sby = (by >> (4 + s.sb128)) << (6 + s.sb128);
    const int sb_size = 1 << (6 + s.sb128);
    if (src_bottom > sby && src_right > sbx) {
        if (src_top - border_top >= src_bottom - sby) { src_top -= src_bottom - sby; src_bottom = sby; }
        else if (src_left - border_left >= src_right - sbx) { src_left -= src_right - sbx; src_right = sbx; }
    }
    if (src_bottom > sby + sb_size) { src_top -= src_bottom - (sby + sb_size); src_bottom = sby + sb_size; }
    if (src_bottom > sby && src_right > sbx) return fail("intra block copy vector overlaps the current superblock");
    mv.x = (int16_t)((src_left - bx * 4) * 8);
    mv.y = (int16_t)((src_top - by * 4) * 8);

    read_vartx_tree(b, bs);
    const uint16_t *split = b.tx_split;
    const int max_ytx = b.max_ytx;

    // prediction + residual work in the reference's coefficient order
    const int w4b = imin(bw4, bw - bx), h4b = imin(bh4, bh - by);
    const int cw4 = (w4b + ss_hor) >> ss_hor, ch4 = (h4b + ss_ver) >> ss_ver;
    const int cbw4 = (bw4 + ss_hor) >> ss_hor, cbh4 = (bh4 + ss_ver) >> ss_ver;
    const TxDim &ut = k_txdim[b.uvtx];
    const TxDim &yt = k_txdim[max_ytx];
    uint8_t txtp_map[32][32];
    memset(txtp_map, 0, sizeof(txtp_map));
    if (b.skip) {
        for (int y = 0; y < h4b; y += yt.h)
            for (int x = 0; x < w4b; x += yt.w)
                push_ibc(b, mv, 0, max_ytx, bx + x, by + y, (bx + x) * 4, (by + y) * 4, 0, nullptr, nullptr, 0, 0, nullptr);
        if (has_chroma)
            for (int pl = 1; pl <= 2; pl++)
                for (int y = 0; y < ch4; y += ut.h)
                    for (int x = 0; x < cw4; x += ut.w)
                        push_ibc(b, mv, pl, b.uvtx, bx, by, ((bx >> ss_hor) + x) * 4, ((by >> ss_ver) + y) * 4, 0,
                                 nullptr, nullptr, 0, 0, nullptr);
        setn(a.lcoef, bx, bw4, 0x40);
        setn(l.lcoef, by4, bh4, 0x40);
        if (has_chroma)
            for (int pl = 0; pl < 2; pl++) {
                setn(a.ccoef[pl], bx >> ss_hor, cbw4, 0x40);
                setn(l.ccoef[pl], by4 >> ss_ver, cbh4, 0x40);
            }
    } else {
        for (int init_y = 0; init_y < h4b; init_y += 16) {
            const int sub_h4 = imin(h4b, 16 + init_y);
            for (int init_x = 0; init_x < w4b; init_x += 16) {
                const int sub_w4 = imin(w4b, init_x + 16);
                int y_off = init_y != 0;
                for (int y = init_y; y < sub_h4; y += yt.h, y_off++) {
                    int x_off = init_x != 0;
                    for (int x = init_x; x < sub_w4; x += yt.w, x_off++)
                        ibc_residual_tree(b, mv, max_ytx, 0, split, x_off, y_off, bx + x, by + y, txtp_map);
                }
                if (!has_chroma) continue;
                const int sub_ch4 = imin(ch4, (init_y + 16) >> ss_ver), sub_cw4 = imin(cw4, (init_x + 16) >> ss_hor);
                for (int pl = 0; pl < 2; pl++)
                    for (int y = init_y >> ss_ver; y < sub_ch4; y += ut.h)
                        for (int x = init_x >> ss_hor; x < sub_cw4; x += ut.w) {
                            int txtp = txtp_map[by4 + (y << ss_ver)][bx4 + (x << ss_hor)];
                            const int tby = by + (y << ss_ver), tbx = bx + (x << ss_hor);
                            const int cx = (bx >> ss_hor) + x;
                            push_ibc(b, mv, 1 + pl, b.uvtx, tbx, tby, cx * 4, ((by >> ss_ver) + y) * 4, 1,
                                     &a.ccoef[pl][cx], &l.ccoef[pl][(by4 >> ss_ver) + y],
                                     imin(ut.w, (bw - tbx + ss_hor) >> ss_hor), imin(ut.h, (bh - tby + ss_ver) >> ss_ver),
                                     &txtp);
                        }
            }
        }
    }
    splat_rmv(bs, bw4, bh4, mv, true);
    return 0;
}

static int neg_deinterleave(int diff, int ref, int max) {
    if (!ref) return diff;
    if (ref >= max - 1) return max - diff - 1;
    if (2 * ref < max) {
        if (diff <= 2 * ref) return (diff & 1) ? ref + ((diff + 1) >> 1) : ref - (diff >> 1);
        return diff;
    }
    if (diff <= 2 * (max - ref - 1)) return (diff & 1) ? ref + ((diff + 1) >> 1) : ref - (diff >> 1);
    return max - (diff + 1);
}

int FrameDec::decode_b(int bl, int bs, int bp, int edge_flags) {
    Msac &m = ts->msac;
    Block b{};
    const BlockDim &bd = k_bdim[bs];
    const int bx4 = bx & 31, by4 = by & 31;
    const int bw4 = bd.w4, bh4 = bd.h4;
    const int w4b = imin(bw4, bw - bx), h4b = imin(bh4, bh - by);
    const int cbw4 = (bw4 + ss_hor) >> ss_hor, cbh4 = (bh4 + ss_ver) >> ss_ver;
    const int have_left = bx > ts->col_start, have_top = by > ts->row_start;
    const int has_chroma = layout != 0 && (bw4 > ss_hor || (bx & 1)) && (bh4 > ss_ver || (by & 1));
    const int cbx = bx >> ss_hor, cby4 = by4 >> ss_ver;
    b.bl = bl;
    b.bs = bs;
    b.bp = bp;

    // segment id (preskip) -- intra frames have no temporal prediction source
    const SegData *seg = nullptr;
    int seg_pred = 0;
    auto cur_segid = [&](int *ctx) -> int {
        const uint8_t *sm = &segmap[(size_t)by * b4_stride + bx];
        if (have_left && have_top) {
            const int lv = sm[-1], av = sm[-b4_stride], alv = sm[-b4_stride - 1];
            *ctx = (lv == av && alv == lv) ? 2 : (lv == av || alv == lv || av == alv) ? 1 : 0;
            return av == alv ? av : lv;
        }
        *ctx = 0;
        return have_left ? sm[-1] : have_top ? sm[-b4_stride] : 0;
    };
    auto prev_segid = [&]() -> int {
        if (!in_.prev_segmap) return 0;
        const uint8_t *p = in_.prev_segmap->data() + (size_t)by * b4_stride + bx;
        int id = 8;
        for (int y = 0; y < h4b && id; y++, p += b4_stride)
            for (int x = 0; x < w4b; x++) id = imin(id, p[x]);
        return id;
    };
    if (h.seg.enabled) {
        if (!h.seg.update_map) {
            b.seg_id = prev_segid();
            if (b.seg_id >= 8) return fail("bad segment id");
            seg = &h.seg.d[b.seg_id];
        } else if (h.seg.preskip) {
            if (h.seg.temporal && (seg_pred = m.bool_adapt(ts->cdf.m.seg_pred[a.seg_pred[bx] + l.seg_pred[by4]]))) {
                b.seg_id = prev_segid();
                if (b.seg_id >= 8) return fail("bad segment id");
            } else {
                int ctx;
                const int pred = cur_segid(&ctx);
                const int diff = m.symbol(ts->cdf.m.seg_id[ctx], 7);
                b.seg_id = neg_deinterleave(diff, pred, h.seg.last_active_segid + 1);
                if (b.seg_id > h.seg.last_active_segid || b.seg_id >= 8) b.seg_id = 0;
            }
            seg = &h.seg.d[b.seg_id];
        }
    }
    // skip_mode (inter frames with skip_mode_present), skip
    b.skip_mode = 0;
    if ((!seg || (!seg->globalmv && seg->ref == -1 && !seg->skip)) && h.skip_mode_enabled && imin(bw4, bh4) > 1)
        b.skip_mode = m.bool_adapt(ts->cdf.m.skip_mode[a.skip_mode[bx] + l.skip_mode[by4]]);
    if (b.skip_mode || (seg && seg->skip)) b.skip = 1;
    else b.skip = m.bool_adapt(ts->cdf.m.skip[a.skip[bx] + l.skip[by4]]);
    if (h.seg.enabled && h.seg.update_map && !h.seg.preskip) {
        if (!b.skip && h.seg.temporal &&
            (seg_pred = m.bool_adapt(ts->cdf.m.seg_pred[a.seg_pred[bx] + l.seg_pred[by4]]))) {
            b.seg_id = prev_segid();
            if (b.seg_id >= 8) return fail("bad segment id");
        } else {
            int ctx;
            const int pred = cur_segid(&ctx);
            if (b.skip) {
                b.seg_id = pred;
            } else {
                const int diff = m.symbol(ts->cdf.m.seg_id[ctx], 7);
                b.seg_id = neg_deinterleave(diff, pred, h.seg.last_active_segid + 1);
                if (b.seg_id > h.seg.last_active_segid) b.seg_id = 0;
            }
            if (b.seg_id >= 8) b.seg_id = 0;
        }
        seg = &h.seg.d[b.seg_id];
    }
    // cdef index
    if (!b.skip) {
        const int idx = s.sb128 ? ((bx & 16) >> 4) + ((by & 16) >> 3) : 0;
        if (cur_cdef_idx[idx] == -1) {
            const int v = m.bools(h.cdef.n_bits);
            cur_cdef_idx[idx] = (int8_t)v;
            if (bw4 > 16) cur_cdef_idx[idx + 1] = (int8_t)v;
            if (bh4 > 16) cur_cdef_idx[idx + 2] = (int8_t)v;
            if (bw4 == 32 && bh4 == 32) cur_cdef_idx[idx + 3] = (int8_t)v;
        }
    }
    // delta q / lf at the superblock's first block
    if (!(bx & (31 >> !s.sb128)) && !(by & (31 >> !s.sb128))) {
        const int prev_qidx = ts->last_qidx;
        const int have_dq = h.delta.q_present && (bs != (s.sb128 ? BS_128x128 : BS_64x64) || !b.skip);
        int8_t prev_dlf[4];
        memcpy(prev_dlf, ts->last_delta_lf, 4);
        if (have_dq) {
            int dq = m.symbol(ts->cdf.m.delta_q, 3);
            if (dq == 3) {
                const int nb = 1 + m.bools(3);
                dq = m.bools(nb) + 1 + (1 << nb);
            }
            if (dq) {
                if (m.bool_equi()) dq = -dq;
                dq *= 1 << h.delta.q_res_log2;
            }
            ts->last_qidx = iclip(ts->last_qidx + dq, 1, 255);
            if (h.delta.lf_present) {
                const int n_lfs = h.delta.lf_multi ? (layout != 0 ? 4 : 2) : 1;
                for (int i = 0; i < n_lfs; i++) {
                    int dl = m.symbol(ts->cdf.m.delta_lf[i + h.delta.lf_multi], 3);
                    if (dl == 3) {
                        const int nb = 1 + m.bools(3);
                        dl = m.bools(nb) + 1 + (1 << nb);
                    }
                    if (dl) {
                        if (m.bool_equi()) dl = -dl;
                        dl *= 1 << h.delta.lf_res_log2;
                    }
                    ts->last_delta_lf[i] = (int8_t)iclip(ts->last_delta_lf[i] + dl, -63, 63);
                }
            }
        }
        if (ts->last_qidx == h.quant.yac) memcpy(ts->dq, dq_frame, sizeof(ts->dq));
        else if (ts->last_qidx != prev_qidx) init_quant(ts->last_qidx, ts->dq);
        static const int8_t zero4[4] = {0, 0, 0, 0};
        if (!memcmp(ts->last_delta_lf, zero4, 4)) ts->lflvl = lflvl_frame;
        else if (memcmp(ts->last_delta_lf, prev_dlf, 4)) calc_lf_values(ts->lflvl, ts->last_delta_lf);
    }

    if (b.skip_mode) {
        b.intra = 0;
    } else if (inter_frame) {
        if (seg && (seg->ref >= 0 || seg->globalmv)) {
            b.intra = !seg->ref;
        } else {
            // get_intra_ctx (env.rs; C env.h:59-73)
            int ictx = 0;
            if (have_left) {
                if (have_top) {
                    ictx = l.intra[by4] + a.intra[bx];
                    ictx += ictx == 2;
                } else {
                    ictx = l.intra[by4] * 2;
                }
            } else if (have_top) {
                ictx = a.intra[bx] * 2;
            }
            b.intra = !m.bool_adapt(ts->cdf.m.intra[ictx]);
        }
    } else if (h.allow_intrabc) {
        b.intra = !m.bool_adapt(ts->cdf.m.intrabc);
    } else {
        b.intra = 1;
    }
    if (!b.intra && inter_frame) {
        if (int e = decode_inter(b, bs, edge_flags, has_chroma, have_left, have_top, seg, seg_pred)) return e;
    } else if (!b.intra) {
        {
            if (int e = decode_ibc(b, bs, edge_flags, has_chroma)) return e;
            // contexts of a block copy (decode.rs:2104-2135)
            setn(a.tx_intra, bx, bw4, bd.lw4);
            setn(l.tx_intra, by4, bh4, bd.lh4);
            setn(a.mode, bx, bw4, DC_PRED);
            setn(l.mode, by4, bh4, DC_PRED);
            setn(a.pal_sz, bx, bw4, 0);
            setn(l.pal_sz, by4, bh4, 0);
            for (int i = 0; i < bw4; i++) pal_sz_uv[0][bx4 + i] = 0;
            for (int i = 0; i < bh4; i++) pal_sz_uv[1][by4 + i] = 0;
            setn(a.seg_pred, bx, bw4, seg_pred);
            setn(l.seg_pred, by4, bh4, seg_pred);
            setn(a.skip_mode, bx, bw4, 0);
            setn(l.skip_mode, by4, bh4, 0);
            setn(a.intra, bx, bw4, 0);
            setn(l.intra, by4, bh4, 0);
            setn(a.skip, bx, bw4, b.skip);
            setn(l.skip, by4, bh4, b.skip);
            if (has_chroma) {
                setn(a.uvmode, cbx, cbw4, DC_PRED);
                setn(l.uvmode, cby4, cbh4, DC_PRED);
            }
        }
    } else {

    // intra modes
    uint16_t *ycdf = inter_frame ? ts->cdf.m.y_mode[k_ymode_size_ctx[bs]]
                                 : ts->cdf.kfym[k_intra_mode_ctx[a.mode[bx]]][k_intra_mode_ctx[l.mode[by4]]];
    b.y_mode = m.symbol(ycdf, 12);
    if (bd.lw4 + bd.lh4 >= 2 && b.y_mode >= V_PRED && b.y_mode <= D67_PRED)
        b.y_angle = (int)m.symbol(ts->cdf.m.angle_delta[b.y_mode - V_PRED], 6) - 3;
    if (has_chroma) {
        static const unsigned cfl_mask = (1u << BS_32x32) | (1u << BS_32x16) | (1u << BS_32x8) | (1u << BS_16x32) |
                                         (1u << BS_16x16) | (1u << BS_16x8) | (1u << BS_16x4) | (1u << BS_8x32) |
                                         (1u << BS_8x16) | (1u << BS_8x8) | (1u << BS_8x4) | (1u << BS_4x16) |
                                         (1u << BS_4x8) | (1u << BS_4x4);
        const int cfl_ok = h.seg.lossless[b.seg_id] ? (cbw4 == 1 && cbh4 == 1) : !!(cfl_mask & (1u << bs));
        b.uv_mode = m.symbol(ts->cdf.m.uv_mode[cfl_ok][b.y_mode], 13 - !cfl_ok);
        if (b.uv_mode == CFL_PRED) {
            const int sign = m.symbol(ts->cdf.m.cfl_sign, 7) + 1;
            const int su = sign * 0x56 >> 8, sv = sign - su * 3;
            if (su) {
                const int ctx = (su == 2) * 3 + sv;
                b.cfl_alpha[0] = m.symbol(ts->cdf.m.cfl_alpha[ctx], 15) + 1;
                if (su == 1) b.cfl_alpha[0] = -b.cfl_alpha[0];
            }
            if (sv) {
                const int ctx = (sv == 2) * 3 + su;
                b.cfl_alpha[1] = m.symbol(ts->cdf.m.cfl_alpha[ctx], 15) + 1;
                if (sv == 1) b.cfl_alpha[1] = -b.cfl_alpha[1];
            }
        } else if (bd.lw4 + bd.lh4 >= 2 && b.uv_mode >= V_PRED && b.uv_mode <= D67_PRED) {
            b.uv_angle = (int)m.symbol(ts->cdf.m.angle_delta[b.uv_mode - V_PRED], 6) - 3;
        }
    }
    uint16_t pal[3][8] = {};
    if (h.allow_screen_content_tools && imax(bw4, bh4) <= 16 && bw4 + bh4 >= 4) {
        const int sz_ctx = bd.lw4 + bd.lh4 - 2;
        if (b.y_mode == DC_PRED) {
            const int pctx = (a.pal_sz[bx] > 0) + (l.pal_sz[by4] > 0);
            if (m.bool_adapt(ts->cdf.m.pal_y[sz_ctx][pctx])) read_pal_plane(b, 0, sz_ctx, bx4, by4, pal[0]);
        }
        if (has_chroma && b.uv_mode == DC_PRED) {
            if (m.bool_adapt(ts->cdf.m.pal_uv[b.pal_sz[0] > 0])) read_pal_uv(b, sz_ctx, bx4, by4, pal);
        }
    }
    if (b.y_mode == DC_PRED && !b.pal_sz[0] && imax(bd.lw4, bd.lh4) <= 3 && s.filter_intra) {
        if (m.bool_adapt(ts->cdf.m.use_filter_intra[bs])) {
            b.y_mode = FILTER_PRED;
            b.y_angle = m.symbol(ts->cdf.m.filter_intra, 4);
        }
    }
    std::vector<uint8_t> pal_idx;
    if (b.pal_sz[0] || (has_chroma && b.pal_sz[1])) pal_idx.assign(bw4 * bh4 * 16 * 2, 0);
    if (b.pal_sz[0]) read_pal_indices(pal_idx.data(), b, 0, w4b, h4b, bw4, bh4);
    if (has_chroma && b.pal_sz[1]) {
        const int cw4 = (w4b + ss_hor) >> ss_hor, ch4 = (h4b + ss_ver) >> ss_ver;
        read_pal_indices(pal_idx.data() + bw4 * bh4 * 16, b, 1, cw4, ch4, cbw4, cbh4);
    }
    // transform size
    const TxDim *td;
    if (h.seg.lossless[b.seg_id]) {
        b.tx = b.uvtx = TX_4X4;
        td = &k_txdim[TX_4X4];
    } else {
        b.tx = k_max_tx_for_bs[bs][0];
        b.uvtx = k_max_tx_for_bs[bs][layout];
        td = &k_txdim[b.tx];
        if (h.txfm_mode == TXMODE_SWITCHABLE && td->max > TX_4X4) {
            const int tctx = (l.tx_intra[by4] >= td->lh) + (a.tx_intra[bx] >= td->lw);
            int depth = m.symbol(ts->cdf.m.txsz[td->max - 1][tctx], imin(td->max, 2));
            while (depth--) {
                b.tx = td->sub;
                td = &k_txdim[b.tx];
            }
        }
    }

    // pass-2 work (prediction + residual per transform block) and coefficients
    emit_intra(b, edge_flags, pal_idx.empty() ? nullptr : pal_idx.data(), pal);

    if (h.lf.level_y[0] || h.lf.level_y[1]) create_lf_mask_intra(b, has_chroma);

    // contexts
    const int ymnf = b.y_mode == FILTER_PRED ? DC_PRED : b.y_mode;
    setn(a.tx_intra, bx, bw4, td->lw);
    setn(l.tx_intra, by4, bh4, td->lh);
    setn(a.tx, bx, bw4, td->lw);
    setn(l.tx, by4, bh4, td->lh);
    setn(a.mode, bx, bw4, ymnf);
    setn(l.mode, by4, bh4, ymnf);
    setn(a.pal_sz, bx, bw4, b.pal_sz[0]);
    setn(l.pal_sz, by4, bh4, b.pal_sz[0]);
    setn(a.seg_pred, bx, bw4, seg_pred);
    setn(l.seg_pred, by4, bh4, seg_pred);
    setn(a.skip_mode, bx, bw4, 0);
    setn(l.skip_mode, by4, bh4, 0);
    setn(a.intra, bx, bw4, 1);
    setn(l.intra, by4, bh4, 1);
    setn(a.skip, bx, bw4, b.skip);
    setn(l.skip, by4, bh4, b.skip);
    for (int i = 0; i < bw4; i++) pal_sz_uv[0][bx4 + i] = (uint8_t)(has_chroma ? b.pal_sz[1] : 0);
    for (int i = 0; i < bh4; i++) pal_sz_uv[1][by4 + i] = (uint8_t)(has_chroma ? b.pal_sz[1] : 0);
    if (b.pal_sz[0]) {
        for (int x = 0; x < bw4; x++) memcpy(al_pal[0][bx4 + x][0], pal[0], 16);
        for (int y = 0; y < bh4; y++) memcpy(al_pal[1][by4 + y][0], pal[0], 16);
    }
    if (has_chroma) {
        setn(a.uvmode, cbx, cbw4, b.uv_mode);
        setn(l.uvmode, cby4, cbh4, b.uv_mode);
        if (b.pal_sz[1])
            for (int pl = 1; pl <= 2; pl++) {
                for (int x = 0; x < bw4; x++) memcpy(al_pal[0][bx4 + x][pl], pal[pl], 16);
                for (int y = 0; y < bh4; y++) memcpy(al_pal[1][by4 + y][pl], pal[pl], 16);
            }
    }
    if (inter_frame) {
        setn(a.comp_type, bx, bw4, COMP_NONE);
        setn(l.comp_type, by4, bh4, COMP_NONE);
        setn(a.ref[0], bx, bw4, -1);
        setn(l.ref[0], by4, bh4, -1);
        setn(a.ref[1], bx, bw4, -1);
        setn(l.ref[1], by4, bh4, -1);
        setn(a.filter[0], bx, bw4, 3);
        setn(l.filter[0], by4, bh4, 3);
        setn(a.filter[1], bx, bw4, 3);
        setn(l.filter[1], by4, bh4, 3);
    }
    if (h.allow_intrabc || inter_frame) splat_rmv(bs, bw4, bh4, Mv{ 0, 0 }, false);
    }   // intra

    // segmentation map, CDEF skip mask
    if (h.seg.enabled && h.seg.update_map)
        for (int y = 0; y < bh4; y++)
            if (by + y < (int)(segmap.size() / b4_stride))
                memset(&segmap[(size_t)(by + y) * b4_stride + bx], b.seg_id, bw4);
    if (!b.skip) {
        uint16_t (*ns)[2] = &lf_mask->noskip_mask[by4 >> 1];
        const unsigned mask = (~0u >> (32 - bw4)) << (bx4 & 15);
        const int bx_idx = (bx4 & 16) >> 4;
        for (int y = 0; y < bh4; y += 2, ns++) {
            (*ns)[bx_idx] |= (uint16_t)mask;
            if (bw4 == 32) (*ns)[1] |= (uint16_t)mask;
        }
    }
    return 0;
}

// ------------------------------------------------------------------------------------------
// partition tree (decode.rs decode_sb; C decode.c:2167-2438) with the edge-availability flags
// of intra_edge.rs computed on the fly: a node is described by (top_has_right,
// left_has_bottom), and its split children n = 0..3 by
//   top_has_right' = !(n == 3 || (n == 1 && !top_has_right)), left_has_bottom' = n == 0 || (n == 2 && left_has_bottom)

struct EdgeNode { int o, h[2], v[2], h4, v4, split[3]; };

static EdgeNode edge_node(int bl, bool tr, bool lb) {
    const int f = (tr ? E_ALL_TR : 0) | (lb ? E_ALL_BL : 0);
    EdgeNode n{};
    n.o = f;
    n.h[0] = f | E_ALL_BL;
    n.v[0] = f | E_ALL_TR;
    if (bl == BL_8) {
        n.h[1] = f & (E_ALL_BL | E420_TR);
        n.v[1] = f & (E_ALL_TR | E420_BL | E422_BL);
        n.split[0] = (f & E_ALL_TR) | E422_BL;
        n.split[1] = f | E444_TR;
        n.split[2] = f & (E420_TR | E420_BL | E422_BL);
    } else {
        n.h[1] = f & E_ALL_BL;
        n.v[1] = f & E_ALL_TR;
        n.h4 = E_ALL_BL;
        n.v4 = E_ALL_TR;
        if (bl == BL_16) {
            n.h4 |= f & E420_TR;
            n.v4 |= f & (E420_BL | E422_BL);
        }
    }
    return n;
}
static bool child_tr(int n, bool tr) { return !(n == 3 || (n == 1 && !tr)); }
static bool child_lb(int n, bool lb) { return n == 0 || (n == 2 && lb); }

int FrameDec::decode_sb(int bl, bool tr, bool lb) {
    const int hsz = 16 >> bl;
    const int have_h_split = bw > bx + hsz, have_v_split = bh > by + hsz;
    if (!have_h_split && !have_v_split) return decode_sb(bl + 1, child_tr(0, tr), child_lb(0, lb));
    Msac &m = ts->msac;
    const EdgeNode node = edge_node(bl, tr, lb);
    const int bx8 = bx >> 1, by8 = (by & 31) >> 1;
    const int ctx = ((a.partition[bx8] >> (4 - bl)) & 1) + (((l.partition[by8] >> (4 - bl)) & 1) << 1);
    uint16_t *pc = ts->cdf.m.partition[bl][ctx];
    int bp;
    int r = 0;
    if (have_h_split && have_v_split) {
        bp = m.symbol(pc, k_part_count[bl]);
        if (layout == 2 && (bp == P_V || bp == P_V4 || bp == P_T_LEFT || bp == P_T_RIGHT)) return fail("4:2:2 vertical split");
        const uint8_t *b = k_block_sizes[bl][bp];
        switch (bp) {
        case P_NONE: r = decode_b(bl, b[0], bp, node.o); break;
        case P_H:
            r = decode_b(bl, b[0], bp, node.h[0]);
            by += hsz;
            if (!r) r = decode_b(bl, b[0], bp, node.h[1]);
            by -= hsz;
            break;
        case P_V:
            r = decode_b(bl, b[0], bp, node.v[0]);
            bx += hsz;
            if (!r) r = decode_b(bl, b[0], bp, node.v[1]);
            bx -= hsz;
            break;
        case P_SPLIT:
            if (bl == BL_8) {
                r = decode_b(bl, BS_4x4, bp, E_ALL_TR | E_ALL_BL);
                bx++;
                if (!r) r = decode_b(bl, BS_4x4, bp, node.split[0]);
                bx--;
                by++;
                if (!r) r = decode_b(bl, BS_4x4, bp, node.split[1]);
                bx++;
                if (!r) r = decode_b(bl, BS_4x4, bp, node.split[2]);
                bx--;
                by--;
            } else {
                r = decode_sb(bl + 1, child_tr(0, tr), child_lb(0, lb));
                bx += hsz;
                if (!r) r = decode_sb(bl + 1, child_tr(1, tr), child_lb(1, lb));
                bx -= hsz;
                by += hsz;
                if (!r) r = decode_sb(bl + 1, child_tr(2, tr), child_lb(2, lb));
                bx += hsz;
                if (!r) r = decode_sb(bl + 1, child_tr(3, tr), child_lb(3, lb));
                bx -= hsz;
                by -= hsz;
            }
            break;
        case P_T_TOP:
            r = decode_b(bl, b[0], bp, E_ALL_TR | E_ALL_BL);
            bx += hsz;
            if (!r) r = decode_b(bl, b[0], bp, node.v[1]);
            bx -= hsz;
            by += hsz;
            if (!r) r = decode_b(bl, b[1], bp, node.h[1]);
            by -= hsz;
            break;
        case P_T_BOTTOM:
            r = decode_b(bl, b[0], bp, node.h[0]);
            by += hsz;
            if (!r) r = decode_b(bl, b[1], bp, node.v[0]);
            bx += hsz;
            if (!r) r = decode_b(bl, b[1], bp, 0);
            bx -= hsz;
            by -= hsz;
            break;
        case P_T_LEFT:
            r = decode_b(bl, b[0], bp, E_ALL_TR | E_ALL_BL);
            by += hsz;
            if (!r) r = decode_b(bl, b[0], bp, node.h[1]);
            by -= hsz;
            bx += hsz;
            if (!r) r = decode_b(bl, b[1], bp, node.v[1]);
            bx -= hsz;
            break;
        case P_T_RIGHT:
            r = decode_b(bl, b[0], bp, node.v[0]);
            bx += hsz;
            if (!r) r = decode_b(bl, b[1], bp, node.h[0]);
            by += hsz;
            if (!r) r = decode_b(bl, b[1], bp, 0);
            by -= hsz;
            bx -= hsz;
            break;
        case P_H4:
            r = decode_b(bl, b[0], bp, node.h[0]);
            by += hsz >> 1;
            if (!r) r = decode_b(bl, b[0], bp, node.h4);
            by += hsz >> 1;
            if (!r) r = decode_b(bl, b[0], bp, E_ALL_BL);
            by += hsz >> 1;
            if (!r && by < bh) r = decode_b(bl, b[0], bp, node.h[1]);
            by -= hsz * 3 >> 1;
            break;
        case P_V4:
            r = decode_b(bl, b[0], bp, node.v[0]);
            bx += hsz >> 1;
            if (!r) r = decode_b(bl, b[0], bp, node.v4);
            bx += hsz >> 1;
            if (!r) r = decode_b(bl, b[0], bp, E_ALL_TR);
            bx += hsz >> 1;
            if (!r && bx < bw) r = decode_b(bl, b[0], bp, node.v[1]);
            bx -= hsz * 3 >> 1;
            break;
        default: return fail("bad partition");
        }
    } else if (have_h_split) {
        // gather_top_partition_prob (env.rs)
        int p = pc[P_V - 1] - pc[P_T_TOP] + pc[P_T_LEFT - 1];
        if (bl != BL_128) p += pc[P_V4 - 1] - pc[P_T_RIGHT];
        const int is_split = m.bool_prob((unsigned)p);
        if (is_split) {
            bp = P_SPLIT;
            r = decode_sb(bl + 1, child_tr(0, tr), child_lb(0, lb));
            bx += hsz;
            if (!r) r = decode_sb(bl + 1, child_tr(1, tr), child_lb(1, lb));
            bx -= hsz;
        } else {
            bp = P_H;
            r = decode_b(bl, k_block_sizes[bl][P_H][0], P_H, node.h[0]);
        }
    } else {
        // gather_left_partition_prob (env.rs)
        int p = pc[P_H - 1] - pc[P_H] + pc[P_SPLIT - 1] - pc[P_T_LEFT];
        if (bl != BL_128) p += pc[P_H4 - 1] - pc[P_H4];
        const int is_split = m.bool_prob((unsigned)p);
        if (layout == 2 && !is_split) return fail("4:2:2 vertical split");
        if (is_split) {
            bp = P_SPLIT;
            r = decode_sb(bl + 1, child_tr(0, tr), child_lb(0, lb));
            by += hsz;
            if (!r) r = decode_sb(bl + 1, child_tr(2, tr), child_lb(2, lb));
            by -= hsz;
        } else {
            bp = P_V;
            r = decode_b(bl, k_block_sizes[bl][P_V][0], P_V, node.v[0]);
        }
    }
    if (r) return r;
    if (bp != P_SPLIT || bl == BL_8) {
        setn(a.partition, bx8, hsz, k_part_ctx_val[0][bl][bp]);
        setn(l.partition, by8, hsz, k_part_ctx_val[1][bl][bp]);
    }
    return 0;
}

// ------------------------------------------------------------------------------------------
// one superblock row of one tile (decode.rs decode_tile_sbrow; C decode.c:2622-2774)

int FrameDec::decode_tile_sbrow(int tile_row, int tile_col) {
    (void)tile_row;
    l.reset(is_intra_frame(h));
    memset(pal_sz_uv[1], 0, sizeof(pal_sz_uv[1]));
    const int sb128y = by >> 5;
    const int root = s.sb128 ? BL_128 : BL_64;
    for (bx = ts->col_start; bx < ts->col_end; bx += sb_step) {
        lf_mask = &mw.lf_masks[(size_t)sb128y * sb128w + (bx >> 5)];
        if (root == BL_128) {
            cur_cdef_idx = lf_mask->cdef_idx;
            for (int i = 0; i < 4; i++) cur_cdef_idx[i] = -1;
        } else {
            cur_cdef_idx = &lf_mask->cdef_idx[((bx & 16) >> 4) + ((by & 16) >> 3)];
            cur_cdef_idx[0] = -1;
        }
        for (int p = 0; p < 3; p++) {
            if (!((fw.restore_planes >> p) & 1)) continue;
            const int sv = p && ss_ver, sh = p && ss_hor;
            const int usl = h.lr.unit_size[!!p];
            const int y = by * 4 >> sv;
            const int ph = (h.height + sv) >> sv;
            const int unit = 1 << usl;
            const unsigned umask = unit - 1;
            if (y & umask) continue;
            const int half = unit >> 1;
            if (y && y + half > ph) continue;
            const int ftype = h.lr.type[p];
            if (h.width[0] != h.width[1]) {
                const int w = (h.width[1] + sh) >> sh;
                const int n_units = imax(1, (w + half) >> usl);
                const int d = h.superres_denom;
                const int rnd = unit * 8 - 1, shift = usl + 3;
                const int x0 = ((4 * bx * d >> sh) + rnd) >> shift;
                const int x1 = ((4 * (bx + sb_step) * d >> sh) + rnd) >> shift;
                for (int x = x0; x < imin(x1, n_units); x++) {
                    const int px_x = x << (usl + sh);
                    const int sb_idx = (by >> 5) * fw.sr_sb128w + (px_x >> 7);
                    const int unit_idx = ((by & 16) >> 3) + ((px_x & 64) >> 6);
                    read_lr(&mw.lr_mask[sb_idx].lr[p][unit_idx], p, ftype);
                }
            } else {
                const int x = 4 * bx >> sh;
                if (x & umask) continue;
                const int w = (h.width[0] + sh) >> sh;
                if (x && x + half > w) continue;
                const int sb_idx = (by >> 5) * fw.sr_sb128w + (bx >> 5);
                const int unit_idx = ((by & 16) >> 3) + ((bx & 16) >> 4);
                read_lr(&mw.lr_mask[sb_idx].lr[p][unit_idx], p, ftype);
            }
        }
        const int r = decode_sb(root, true, false);
        if (r) return r;
    }
    // left context at the tile's right edge, for the loop filter's tile-column fixup
    const int align_h = (bh + 31) & ~31;
    for (int i = 0; i < sb_step; i++)
        if ((size_t)(align_h * tile_col + by + i) < tx_lpf_right[0].size())
            tx_lpf_right[0][align_h * tile_col + by + i] = l.tx_lpf_y[(by & 16) + i];
    const int ah = align_h >> ss_ver;
    for (int i = 0; i < (sb_step >> ss_ver); i++)
        if ((size_t)(ah * tile_col + (by >> ss_ver) + i) < tx_lpf_right[1].size())
            tx_lpf_right[1][ah * tile_col + (by >> ss_ver) + i] = l.tx_lpf_uv[((by & 16) >> ss_ver) + i];
    return 0;
}

// rav1d_loopfilter_sbrow_cols' tile-boundary fixups (lf_apply.rs:625-705; C lf_apply_tmpl.c:
// 331-401), applied once to the whole frame's masks: at every tile column's first 4x4 column
// and every tile row's first 4x4 row, the edge filter size is capped by the transform size the
// neighbouring tile left in its context
void FrameDec::tile_fixups() {
    const int is_sb64 = !s.sb128, sbsz = 32 >> is_sb64, sbl2 = 5 - is_sb64;
    const int halign = (bh + 31) & ~31;
    const int vmask = 16 >> ss_ver, hmask = 16 >> ss_hor;
    const unsigned vmax = 1u << vmask, hmax = 1u << hmask;
    for (int sby = 0; sby < sbh; sby++) {
        const int starty4 = (sby & is_sb64) << 4;
        const unsigned endy4 = starty4 + imin(h4 - sby * sbsz, sbsz);
        const unsigned uv_endy4 = (endy4 + ss_ver) >> ss_ver;
        MiAv1Filter *lflvl = &mw.lf_masks[(size_t)(sby >> is_sb64) * sb128w];
        const uint8_t *lpf_y = &tx_lpf_right[0][sby << sbl2];
        const uint8_t *lpf_uv = &tx_lpf_right[1][sby << (sbl2 - ss_ver)];
        for (int tc = 1;; tc++) {
            int x = h.tiling.col_start_sb[tc];
            if ((x << sbl2) >= bw) break;
            const int bx4 = x & is_sb64 ? 16 : 0, cbx4 = bx4 >> ss_hor;
            x >>= is_sb64;
            uint16_t (*yh)[2] = lflvl[x].filter_y[0][bx4];
            for (unsigned y = starty4, mk = 1u << y; y < endy4; y++, mk <<= 1) {
                const int sidx = mk >= 0x10000u;
                const uint16_t sm = (uint16_t)(mk >> (sidx << 4));
                const int idx = 2 * !!(yh[2][sidx] & sm) + !!(yh[1][sidx] & sm);
                yh[2][sidx] &= ~sm;
                yh[1][sidx] &= ~sm;
                yh[0][sidx] &= ~sm;
                yh[imin(idx, lpf_y[y - starty4])][sidx] |= sm;
            }
            if (layout != 0) {
                uint16_t (*uh)[2] = lflvl[x].filter_uv[0][cbx4];
                for (unsigned y = starty4 >> ss_ver, mk = 1u << y; y < uv_endy4; y++, mk <<= 1) {
                    const int sidx = mk >= vmax;
                    const uint16_t sm = (uint16_t)(mk >> (sidx << (4 - ss_ver)));
                    const int idx = !!(uh[1][sidx] & sm);
                    uh[1][sidx] &= ~sm;
                    uh[0][sidx] &= ~sm;
                    uh[imin(idx, lpf_uv[y - (starty4 >> ss_ver)])][sidx] |= sm;
                }
            }
            lpf_y += halign;
            lpf_uv += halign >> ss_ver;
        }
        // first superblock row of a tile row (other than the first)
        int tile_row = -1;
        for (int tr = 1; tr < h.tiling.rows; tr++)
            if (h.tiling.row_start_sb[tr] == sby) tile_row = tr;
        if (tile_row > 0) {
            const std::vector<uint8_t> &ay = S->a_tx_lpf_end[0][tile_row - 1], &auv = S->a_tx_lpf_end[1][tile_row - 1];
            for (int x = 0; x < sb128w; x++) {
                uint16_t (*yv)[2] = lflvl[x].filter_y[1][starty4];
                const unsigned w = imin(32, w4 - (x << 5));
                for (unsigned mk = 1, i = 0; i < w; mk <<= 1, i++) {
                    const int sidx = mk >= 0x10000u;
                    const uint16_t sm = (uint16_t)(mk >> (sidx << 4));
                    const int idx = 2 * !!(yv[2][sidx] & sm) + !!(yv[1][sidx] & sm);
                    yv[2][sidx] &= ~sm;
                    yv[1][sidx] &= ~sm;
                    yv[0][sidx] &= ~sm;
                    yv[imin(idx, ay[(x << 5) + i])][sidx] |= sm;
                }
                if (layout != 0) {
                    const unsigned cw = (w + ss_hor) >> ss_hor;
                    uint16_t (*uv)[2] = lflvl[x].filter_uv[1][starty4 >> ss_ver];
                    for (unsigned mk = 1, i = 0; i < cw; mk <<= 1, i++) {
                        const int sidx = mk >= hmax;
                        const uint16_t sm = (uint16_t)(mk >> (sidx << (4 - ss_hor)));
                        const int idx = !!(uv[1][sidx] & sm);
                        uv[1][sidx] &= ~sm;
                        uv[0][sidx] &= ~sm;
                        uv[imin(idx, auv[((x << 5) >> ss_hor) + i])][sidx] |= sm;
                    }
                }
            }
        }
    }
}

int FrameDec::init_frame() {
    inter_frame = !is_intra_frame(h);
    layout = s.layout;
    ss_hor = layout == 1 || layout == 2;
    ss_ver = layout == 1;
    hbd_idx = s.hbd;
    bw = ((h.width[0] + 7) >> 3) << 1;
    bh = ((h.height + 7) >> 3) << 1;
    w4 = (h.width[0] + 3) >> 2;
    h4 = (h.height + 3) >> 2;
    sb128w = (bw + 31) >> 5;
    sb128h = (bh + 31) >> 5;
    sb_shift = 4 + s.sb128;
    sb_step = 16 << s.sb128;
    sbh = (bh + sb_step - 1) >> sb_shift;
    b4_stride = (bw + 31) & ~31;

    fw.w = h.width[0];
    fw.h = h.height;
    fw.up_w = h.width[1];
    fw.render_w = h.render_width;
    fw.render_h = h.render_height;
    fw.bpc = s.bpc;
    fw.layout = layout;
    fw.ss_hor = ss_hor;
    fw.ss_ver = ss_ver;
    fw.sb128 = s.sb128;
    fw.intra_only = !inter_frame;
    // arena entries 0..15: the reserved zero block that residual-free records point at
    fw.ncoef = 16;
    fw.coef.assign((size_t)16 * (s.bpc == 8 ? 2 : 4), 0);
    fw.b4_stride = b4_stride;
    fw.sb128w = sb128w;
    fw.sb128h = sb128h;
    fw.filter_y = h.lf.level_y[0] || h.lf.level_y[1];
    fw.filter_uv = h.lf.level_u || h.lf.level_v;
    // E / I limits (lf_mask.rs calc_eih)
    for (int lvl = 0; lvl < 64; lvl++) {
        int lim = lvl;
        const int sh = h.lf.sharpness;
        if (sh > 0) {
            lim >>= (sh + 3) >> 2;
            lim = imin(lim, 9 - sh);
        }
        lim = imax(lim, 1);
        fw.lim_i[lvl] = (uint8_t)lim;
        fw.lim_e[lvl] = (uint8_t)(2 * (lvl + 2) + lim);
    }
    fw.cdef_on = s.cdef;
    fw.cdef_damping = h.cdef.damping;
    for (int i = 0; i < 8; i++) {
        fw.cdef_y[i] = (uint8_t)h.cdef.y_strength[i];
        fw.cdef_uv[i] = (uint8_t)h.cdef.uv_strength[i];
    }
    fw.sr_sb128w = (h.width[1] + 127) >> 7;
    fw.restore_planes = (h.lr.type[0] != RESTORE_NONE) | ((h.lr.type[1] != RESTORE_NONE) << 1) |
                        ((h.lr.type[2] != RESTORE_NONE) << 2);
    fw.lr_unit_size[0] = h.lr.unit_size[0];
    fw.lr_unit_size[1] = h.lr.unit_size[1];
    fw.fg_present = h.fg.present;
    fw.fg = h.fg.data;

    init_quant(h.quant.yac, dq_frame);
    static const int8_t zero4[4] = {0, 0, 0, 0};
    calc_lf_values(lflvl_frame, zero4);
    const int align_h = (bh + 31) & ~31;
    owner_stride = (b4_stride + 32);
    if (h.allow_intrabc || inter_frame) rmv_stride = b4_stride + 16;
    if (master_) {
        // the frame's maps: allocated once, shared with the tile decoders
        fw.lf_level.assign((size_t)b4_stride * sb128h * 32 * 4, 0);
        fw.lf_masks.assign((size_t)sb128w * sb128h, MiAv1Filter{});
        fw.lr_mask.assign((size_t)fw.sr_sb128w * sb128h, MiAv1Restoration{});
        if (in_.segmap_buf && in_.segmap_buf->size() == (size_t)b4_stride * sb128h * 32) S->segmap = in_.segmap_buf;
        else S->segmap = std::make_shared<std::vector<uint8_t>>((size_t)b4_stride * sb128h * 32, 0);
        S->tx_lpf_right[0].assign((size_t)align_h * h.tiling.cols, 0);
        S->tx_lpf_right[1].assign((size_t)(align_h >> ss_ver) * h.tiling.cols, 0);
        S->a_tx_lpf_end[0].assign(h.tiling.rows, std::vector<uint8_t>());
        S->a_tx_lpf_end[1].assign(h.tiling.rows, std::vector<uint8_t>());
        for (int p = 0; p < 3; p++) S->owner[p].assign((size_t)owner_stride * (sb128h * 32 + 32), -1);
        if (h.allow_intrabc || inter_frame) {
            // the refmvs blocks and their filter map are read only where this frame wrote them
            // (above / left neighbours inside the tile, as refmvs.rs reads its rows), so they are
            // not reset: decoding every reference vector with both filled with garbage instead
            // is MD5-exact
            S->rmv.reset((size_t)rmv_stride * (sb128h * 32 + 16));
            S->f2d_map.reset(S->rmv.size());
        }
    }
    segmap.bind(*S->segmap);
    for (int k = 0; k < 2; k++) tx_lpf_right[k].bind(S->tx_lpf_right[k]);
    for (int p = 0; p < 3; p++) owner[p].bind(S->owner[p]);
    rmv.bind(S->rmv);
    f2d_map.bind(S->f2d_map);
    if (inter_frame) {
        refmvs_init_frame();
        inter_frame_init();
    }
    a.alloc(b4_stride + 64);
    l.alloc(64);
    memset(al_pal, 0, sizeof(al_pal));
    memset(pal_sz_uv, 0, sizeof(pal_sz_uv));
    return 0;
}

// All superblock rows of tile k (decode.rs decode_tile_sbrow over the tile). tile_tmvs: the
// temporal MVs projected (load_tmvs) and saved (save_tmvs) over the tile's columns per sbrow,
// as rav1d's tile threads do (thread_task.rs); the result equals the frame-wide passes of the
// single-threaded decode (decode.rs decode_frame_main), which run() uses without threads.
int FrameDec::decode_tile(int k, bool tile_tmvs) {
    const int tr = k / h.tiling.cols, tc = k % h.tiling.cols;
    ts = &ts_[k];
    a.reset(is_intra_frame(h));
    const int sb_end = imin(h.tiling.row_start_sb[tr + 1], sbh);
    const int c8s = ts->col_start >> 1, c8e = ts->col_end >> 1;
    for (int sby = h.tiling.row_start_sb[tr]; sby < sb_end; sby++) {
        by = sby << sb_shift;
        if (int r = wait_refs(by)) return r;
        if (tile_tmvs && inter_frame && h.use_ref_frame_mvs) load_tmvs(by >> 1, (by + sb_step) >> 1, c8s, c8e);
        if (ts->msac.cnt < -15) return fail("symbol decoder overread");
        const int r = decode_tile_sbrow(tr, tc);
        if (r) return r;
        if (tile_tmvs && inter_frame) save_tmvs(by >> 1, (by + sb_step) >> 1, c8s, c8e);
        if (in_.progress) in_.progress->tile_row_done(sby);
    }
    if (k == h.tiling.update && h.refresh_context && in_.progress) in_.progress->publish_cdf(out_cdf());
    // the above context at the tile row's end (loop-filter fixups at the next tile row), the
    // tile's columns
    if (tr + 1 < h.tiling.rows) {
        for (int pl = 0; pl < 2; pl++) {
            const std::vector<uint8_t> &src = pl ? a.tx_lpf_uv : a.tx_lpf_y;
            std::vector<uint8_t> &dst = S->a_tx_lpf_end[pl][tr];
            const int sh = pl ? ss_hor : 0;
            const int x0 = ts->col_start >> sh, x1 = imin((ts->col_end + sh) >> sh, (int)src.size());
            for (int x = x0; x < x1; x++) dst[x] = src[x];
        }
    }
    return 0;
}

// Append tile decoder t's work lists, rebasing every index into the lists and arenas it
// points at (intra blocks of dependencies, coefficient / idx / palette / mask / tmp arenas)
void FrameDec::merge_tile(const FrameWork &t) {
    // packed blocks start on 4-coefficient boundaries of their tile's arena: keep them there
    if (fw.ncoef & 3) {
        const size_t pad = 4 - (fw.ncoef & 3);
        fw.coef.resize((fw.ncoef + pad) * (s.bpc == 8 ? 2 : 4), 0);
        fw.ncoef += pad;
    }
    const uint32_t intra_base = (uint32_t)fw.intra.size(), deps_base = (uint32_t)fw.deps.size();
    const uint32_t coef_base = (uint32_t)fw.ncoef, idx_base = (uint32_t)fw.idx.size();
    const uint32_t pal_base = (uint32_t)(fw.pal.size() / (s.bpc == 8 ? 1 : 2));
    const uint32_t masks_base = (uint32_t)fw.masks.size(), tmp_base = (uint32_t)fw.ntmp;
    for (MiIntraBlock b : t.intra) {
        if (b.mode == MI_IPRED_PAL) {
            b.aux_off += idx_base;
            b.pal_off += pal_base;
        } else if (b.flags & MI_INTRA_II) {
            b.aux_off += idx_base;
        }
        fw.intra.push_back(b);
    }
    for (MiTxBlock b : t.intra_tx) {
        b.coef_off += coef_base;
        fw.intra_tx.push_back(b);
    }
    for (int32_t d : t.dep_start) fw.dep_start.push_back(d + (int32_t)deps_base);
    for (int32_t d : t.deps) fw.deps.push_back(d + (int32_t)intra_base);
    for (MiTxBlock b : t.inter_tx) {
        b.coef_off += coef_base;
        fw.inter_tx.push_back(b);
    }
    auto mc_list = [&](const std::vector<MiMcBlock> &src, std::vector<MiMcBlock> &dst) {
        for (MiMcBlock u : src) {
            if (u.comp == MI_MC_MASK || u.comp == MI_MC_SEG) u.mask_off += masks_base;
            else if (u.comp == MI_MC_PREP) u.mask_off += tmp_base;
            dst.push_back(u);
        }
    };
    mc_list(t.mc, fw.mc);
    mc_list(t.obmc_h, fw.obmc_h);
    mc_list(t.obmc_v, fw.obmc_v);
    mc_list(t.scaled, fw.scaled);
    for (MiWarpBlock w : t.warp) {
        if (w.prep) w.tmp_off += tmp_base;
        fw.warp.push_back(w);
    }
    auto combine_list = [&](const std::vector<MiMcCombine> &src, std::vector<MiMcCombine> &dst) {
        for (MiMcCombine c : src) {
            c.tmp_off[0] += tmp_base;
            c.tmp_off[1] += tmp_base;
            if (c.comp == MI_MC_MASK || c.comp == MI_MC_SEG) c.mask_off += masks_base;
            dst.push_back(c);
        }
    };
    combine_list(t.combine_y, fw.combine_y);
    combine_list(t.combine_uv, fw.combine_uv);
    fw.masks.insert(fw.masks.end(), t.masks.begin(), t.masks.end());
    fw.ntmp += t.ntmp;
    fw.coef.insert(fw.coef.end(), t.coef.begin(), t.coef.end());
    fw.ncoef += t.ncoef;
    fw.idx.insert(fw.idx.end(), t.idx.begin(), t.idx.end());
    fw.pal.insert(fw.pal.end(), t.pal.begin(), t.pal.end());
}

}  // namespace fd

void frame_buffers(const FrameHdr &h, std::shared_ptr<std::vector<TmvBlock>> &rp,
                   std::shared_ptr<std::vector<uint8_t>> &segmap) {
    // (init_frame's and refmvs_init_frame's geometry)
    const int bw = ((h.width[0] + 7) >> 3) << 1, bh = ((h.height + 7) >> 3) << 1;
    const int b4_stride = (bw + 31) & ~31, sb128h = (bh + 31) >> 5;
    segmap = std::make_shared<std::vector<uint8_t>>((size_t)b4_stride * sb128h * 32, 0);
    rp.reset();
    if (!is_intra_frame(h)) rp = std::make_shared<std::vector<TmvBlock>>((size_t)(b4_stride >> 1) * sb128h * 16, TmvBlock{});
}

namespace fd {

int FrameDec::wait_refs(int by) {
    const int rows = by + sb_step;
    for (int i = 0; i < 7; i++)
        if (in_.ref_prog[i] && inter_frame && rp_ref[i] && !in_.ref_prog[i]->wait_rows(rows))
            return fail("reference frame failed");
    if (in_.prev_segmap_prog && h.seg.enabled && !in_.prev_segmap_prog->wait_rows(rows))
        return fail("reference frame failed");
    return 0;
}

// the entropy state later frames start from (refresh_context): the frame's initial CDFs with
// the context-update tile's adapted ones (cdf.rs update)
std::shared_ptr<const Cdf> FrameDec::out_cdf() {
    auto c = std::make_shared<Cdf>();
    if (in_cdf_) *c = *in_cdf_;
    else cdf_init_default(*c, h.quant.yac);
    cdf_update_frame(*c, ts_[h.tiling.update].cdf, is_intra_frame(h));
    return c;
}

int FrameDec::run(FrameResult &res, std::string &err) {
    err_ = &err;
    static const bool rtrace = getenv("MI_DEC_TRACE") != nullptr;   // (diagnostics)
    const auto r0 = std::chrono::steady_clock::now();
    auto rms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r0).count(); };
    if (int r = init_frame()) return r;
    if (rtrace) fprintf(stderr, "  init %.2f ms\n", rms());
    const int n_tiles = h.tiling.cols * h.tiling.rows;
    if ((int)in_.tiles.size() != n_tiles) return fail("tile count mismatch");
    // the frame's maps are published before its entropy state is waited for: frames whose
    // primary reference is still adapting it are set up meanwhile
    // (its own segment map also when it is all zeros: no update and no primary reference's)
    std::shared_ptr<const std::vector<uint8_t>> seg_out;
    if (h.seg.enabled) seg_out = h.seg.update_map || !in_.prev_segmap ? S->segmap : in_.prev_segmap;
    if (in_.progress) {
        in_.progress->set_tiling(h.tiling.cols, sb_shift, sbh);
        in_.progress->publish(inter_frame ? rp : nullptr, seg_out);
    }
    in_cdf_ = in_.in_cdf;
    if (in_.in_cdf_prog) {
        if (!in_.in_cdf_prog->wait_cdf()) return fail("reference frame failed");
        in_cdf_hold_ = in_.in_cdf_prog->cdf;
        in_cdf_ = in_cdf_hold_.get();
    }
    ts_.resize(n_tiles);
    for (int tr = 0; tr < h.tiling.rows; tr++)
        for (int tc = 0; tc < h.tiling.cols; tc++) {
            const int k = tr * h.tiling.cols + tc;
            setup_tile(ts_[k], in_.tiles[k].data, in_.tiles[k].size, tr, tc);
        }
    for (int tr = 0; tr + 1 < h.tiling.rows; tr++)
        for (int pl = 0; pl < 2; pl++) S->a_tx_lpf_end[pl][tr].assign(a.tx_lpf_y.size(), 0);
    std::shared_ptr<const Cdf> cdf_done;
    if (!in_.pool || n_tiles <= 1) {
        // decode.rs decode_frame_main (C decode.c:3225-3244): per sbrow, temporal MVs projected
        // over the frame before its tiles and this frame's MVs saved after them
        for (int tr = 0; tr < h.tiling.rows; tr++) {
            a.reset(is_intra_frame(h));
            const int sb_end = imin(h.tiling.row_start_sb[tr + 1], sbh);
            for (int sby = h.tiling.row_start_sb[tr]; sby < sb_end; sby++) {
                by = sby << sb_shift;
                if (int r = wait_refs(by)) return r;
                if (inter_frame && h.use_ref_frame_mvs) load_tmvs(by >> 1, (by + sb_step) >> 1, 0, iw8);
                for (int tc = 0; tc < h.tiling.cols; tc++) {
                    ts = &ts_[tr * h.tiling.cols + tc];
                    if (ts->msac.cnt < -15) return fail("symbol decoder overread");
                    const int r = decode_tile_sbrow(tr, tc);
                    if (r) return r;
                }
                if (inter_frame) save_tmvs(by >> 1, (by + sb_step) >> 1, 0, iw8);
                if (in_.progress) in_.progress->rows_done((sby + 1) << sb_shift);
            }
            if (tr + 1 < h.tiling.rows) {
                S->a_tx_lpf_end[0][tr] = a.tx_lpf_y;
                S->a_tx_lpf_end[1][tr] = a.tx_lpf_uv;
            }
            if (h.refresh_context && tr == h.tiling.update / h.tiling.cols) {
                cdf_done = out_cdf();
                if (in_.progress) in_.progress->publish_cdf(cdf_done);
            }
        }
    } else {
        // rav1d's tile threads: tiles are independent in entropy, contexts and prediction; each
        // runs on its own decoder (own above / left contexts and work lists), tiles dealt to
        // nt threads in turn, then the lists are appended in tile order
        std::vector<FrameWork> tw(n_tiles);
        std::vector<std::string> terr(n_tiles);
        std::vector<int> trc(n_tiles, 0);
        std::vector<double> tdur(n_tiles, 0.0), tstart(n_tiles, 0.0);   // (MI_DEC_TRACE)
        static const bool trace = getenv("MI_DEC_TRACE") != nullptr;   // (diagnostics)
        const auto t0 = std::chrono::steady_clock::now();
        // (the context-update tile first: later frames start from its entropy state)
        in_.pool->run(n_tiles, [&](int i) {
            const int k = (i + h.tiling.update) % n_tiles;
            FrameDec td(*this, tw[k]);
            td.err_ = &terr[k];
            try {
                const auto a0 = std::chrono::steady_clock::now();
                trc[k] = td.init_frame();
                tstart[k] = std::chrono::duration<double, std::milli>(a0 - t0).count();
                if (!trc[k]) trc[k] = td.decode_tile(k, true);
                tdur[k] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a0).count();
            } catch (const std::bad_alloc &) {
                trc[k] = -ENOMEM;
                terr[k] = "out of memory";
            }
        });
        const auto t1 = std::chrono::steady_clock::now();
        if (trace) {
            fprintf(stderr, "  tiles %.2f ms, each ms (started at):", std::chrono::duration<double, std::milli>(t1 - t0).count());
            for (int k = 0; k < n_tiles; k++) fprintf(stderr, " %.2f(%.2f)", tdur[k], tstart[k]);
            fprintf(stderr, "\n");
        }
        const auto t2 = std::chrono::steady_clock::now();
        for (int k = 0; k < n_tiles; k++)
            if (trc[k]) {
                err = terr[k];
                return trc[k];
            }
        for (int k = 0; k < n_tiles; k++) merge_tile(tw[k]);
        if (trace)
            fprintf(stderr, "  merge %.2f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count());
    }
    if (rtrace) fprintf(stderr, "  tiles done %.2f ms\n", rms());
    if (h.tiling.cols > 1 || h.tiling.rows > 1) tile_fixups();
    fw.dep_start.push_back((int32_t)fw.deps.size());
    if (rtrace) fprintf(stderr, "  fixups done %.2f ms\n", rms());

    if (h.refresh_context) res.out_cdf = cdf_done ? cdf_done : out_cdf();
    if (inter_frame) res.mvs = rp;
    res.segmap = seg_out;
    if (in_.progress) {
        in_.progress->rows_done(INT_MAX);
        if (h.refresh_context && !cdf_done) in_.progress->publish_cdf(res.out_cdf);
    }
    if (rtrace) fprintf(stderr, "  result %.2f ms\n", rms());
    return 0;
}

}  // namespace fd

int decode_frame(const FrameInputs &in, FrameWork &work, FrameResult &res, std::string &err) {
    fd::FrameDec d(in, work);
    return d.run(res, err);
}

}  // namespace av1
