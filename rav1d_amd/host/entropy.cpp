// entropy.cpp — the header bit reader, the msac range decoder and the CDF context.
//
// Bit reader: getbits.rs (C src/getbits.c). Range decoder: msac.rs (C src/msac.c:28-248),
// with a 64-bit window, 15-bit range, EC_PROB_SHIFT 6, EC_MIN_PROB 4, and the adaptation
// rate 4 + (count >> 4) + (n_symbols > 2) with counter saturation at 32. CDF defaults:
// cdf.rs (C src/cdf.c: av1_default_cdf, default_kf_y_mode_cdf, av1_default_coef_cdf[4] by
// quantizer category, default_mv_component_cdf / default_mv_joint_cdf), data generated into
// tables/cdf_default.inc by tools/gen_dec_tables.py. End-of-frame CDF propagation follows
// dav1d_cdf_thread_update (C cdf.c:3948-4067).
#include "av1.h"

namespace av1 {

// ---------------------------------------------------------------------- header bits
unsigned Bits::uleb128() {
    uint64_t v = 0;
    unsigned i = 0, more;
    do {
        const unsigned b = bits(8);
        more = b & 0x80;
        v |= (uint64_t)(b & 0x7f) << i;
        i += 7;
    } while (more && i < 56);
    if (v > 0xffffffffu || more) {
        error = true;
        return 0;
    }
    return (unsigned)v;
}

unsigned Bits::uniform(unsigned max) {   // value in [0, max), max > 1
    const int l = ulog2(max) + 1;
    const unsigned m = (1u << l) - max;
    const unsigned v = bits(l - 1);
    return v < m ? v : (v << 1) - m + bit();
}

unsigned Bits::vlc() {
    int n = 0;
    while (!bit()) {
        if (++n == 32) return 0xffffffffu;
    }
    return n ? ((1u << n) - 1) + bits(n) : 0;
}

static unsigned inv_recenter(unsigned r, unsigned v) {
    if (v > (r << 1)) return v;
    return (v & 1) ? r - ((v + 1) >> 1) : r + (v >> 1);
}

// decode_signed_subexp_with_ref (spec 5.9.26 / getbits.rs get_bits_subexp), n = log2 range
int Bits::subexp(int ref, int n) {
    const unsigned mx = 2u << n, r = (unsigned)(ref + (1 << n));
    unsigned v = 0;
    for (int i = 0;; i++) {
        const int b = i ? 3 + i - 1 : 3;
        if (mx < v + 3 * (1u << b)) {
            v += uniform(mx - v + 1);
            break;
        }
        if (!bit()) {
            v += bits(b);
            break;
        }
        v += 1u << b;
    }
    const unsigned u = r * 2 <= mx ? inv_recenter(r, v) : mx - inv_recenter(mx - r, v);
    return (int)u - (1 << n);
}

// ---------------------------------------------------------------------- msac

void Msac::init(const uint8_t *data, size_t sz, bool disable_update) {
    pos = data;
    end = data + sz;
    dif = ((uint64_t)1 << (kWin - 1)) - 1;
    rng = 0x8000;
    cnt = -15;
    adapt = !disable_update;
    refill();
}

void Msac::refill() {
    int c = kWin - cnt - 24;
    uint64_t d = dif;
    while (c >= 0 && pos < end) {
        d ^= (uint64_t)*pos++ << c;
        c -= 8;
    }
    dif = d;
    cnt = kWin - c - 24;
}

int Msac::uniform(unsigned n) {
    const int l = ulog2(n) + 1;
    const unsigned m = (1u << l) - n;
    const unsigned v = bools(l - 1);
    return (int)(v < m ? v : (v << 1) - m + bool_equi());
}

int Msac::subexp(int ref, int n, unsigned k) {
    unsigned a = 0;
    if (bool_equi()) {
        if (bool_equi()) k += bool_equi() + 1;
        a = 1u << k;
    }
    const unsigned v = bools(k) + a;
    return ref * 2 <= n ? (int)inv_recenter(ref, v) : n - 1 - (int)inv_recenter(n - 1 - ref, v);
}

unsigned Msac::golomb() {
    int len = 0;
    unsigned val = 1;
    while (!bool_equi() && len < 32) len++;
    while (len--) val = (val << 1) + bool_equi();
    return val - 1;
}

// ---------------------------------------------------------------------- CDF defaults
#include "tables/cdf_default.inc"

template <typename T, typename S>
static void load(T &dst, const S &src) {
    static_assert(sizeof(T) == sizeof(src), "CDF table shape mismatch");
    memcpy(&dst, src, sizeof(T));
}

static int qcat(int qidx) { return qidx <= 20 ? 0 : qidx <= 60 ? 1 : qidx <= 120 ? 2 : 3; }

void cdf_init_default(Cdf &c, int base_qidx) {
    CdfMode &m = c.m;
#define M(f) load(m.f, k_cdf_mode_##f)
    M(y_mode); M(uv_mode); M(wedge_idx); M(partition); M(cfl_alpha); M(txtp_inter1); M(txtp_inter2);
    M(txtp_intra1); M(txtp_intra2); M(cfl_sign); M(angle_delta); M(filter_intra); M(comp_inter_mode);
    M(seg_id); M(pal_sz); M(color_map); M(filter); M(txsz); M(motion_mode); M(delta_q); M(delta_lf);
    M(interintra_mode); M(restore_switchable); M(restore_wiener); M(restore_sgrproj); M(interintra);
    M(interintra_wedge); M(txtp_inter3); M(use_filter_intra); M(newmv_mode); M(globalmv_mode);
    M(refmv_mode); M(drl_bit); M(intra); M(comp); M(comp_dir); M(jnt_comp); M(mask_comp); M(wedge_comp);
    M(ref); M(comp_fwd_ref); M(comp_bwd_ref); M(comp_uni_ref); M(txpart); M(skip); M(skip_mode);
    M(seg_pred); M(obmc); M(pal_y); M(pal_uv); M(intrabc);
#undef M
    load(c.kfym, k_cdf_kf_y_mode);
    CdfCoef &k = c.coef;
    switch (qcat(base_qidx)) {
#define C(q, f) load(k.f, k_cdf_coef##q##_##f)
#define Q(q) \
    case q: \
        C(q, eob_bin_16); C(q, eob_bin_32); C(q, eob_bin_64); C(q, eob_bin_128); C(q, eob_bin_256); \
        C(q, eob_bin_512); C(q, eob_bin_1024); C(q, eob_base_tok); C(q, base_tok); C(q, br_tok); \
        C(q, eob_hi_bit); C(q, skip); C(q, dc_sign); break;
        Q(0) Q(1) Q(2) Q(3)
#undef Q
#undef C
    }
    CdfMvComp mc;
    load(mc.classes, k_cdf_mv_classes);
    load(mc.class0_fp, k_cdf_mv_class0_fp);
    load(mc.classN_fp, k_cdf_mv_classN_fp);
    load(mc.class0_hp, k_cdf_mv_class0_hp);
    load(mc.classN_hp, k_cdf_mv_classN_hp);
    load(mc.class0, k_cdf_mv_class0);
    load(mc.classN, k_cdf_mv_classN);
    load(mc.sign, k_cdf_mv_sign);
    c.mv.comp[0] = c.mv.comp[1] = c.dmv.comp[0] = c.dmv.comp[1] = mc;
    load(c.mv.joint, k_cdf_mv_joint);
    load(c.dmv.joint, k_cdf_mv_joint);
}

// ---------------------------------------------------------------------- end-of-frame update
// Copy an adapted table and clear its counter (slot n). `n` may depend on the outer index.
static void upd(uint16_t *dst, const uint16_t *src, int len, int n) {
    memcpy(dst, src, len * sizeof(uint16_t));
    dst[n] = 0;
}
static void upd_bit(uint16_t *dst, const uint16_t *src) {
    dst[0] = src[0];
    dst[1] = 0;
}
template <size_t N, size_t L>
static void upd_rows(uint16_t (&d)[N][L], const uint16_t (&s)[N][L], int n) {
    for (size_t i = 0; i < N; i++) upd(d[i], s[i], L, n);
}
template <size_t N>
static void upd_bits(uint16_t (&d)[N][2], const uint16_t (&s)[N][2]) {
    for (size_t i = 0; i < N; i++) upd_bit(d[i], s[i]);
}

void cdf_update_frame(Cdf &dst, const Cdf &src, bool intra_frame) {
    CdfMode &d = dst.m;
    const CdfMode &s = src.m;
    upd_bits(d.use_filter_intra, s.use_filter_intra);
    upd(d.filter_intra, s.filter_intra, 8, 4);
    for (int k = 0; k < 2; k++)
        for (int j = 0; j < 13; j++) upd(d.uv_mode[k][j], s.uv_mode[k][j], 16, 13 - !k);
    upd_rows(d.angle_delta, s.angle_delta, 6);
    for (int k = 0; k < 4; k++)
        for (int j = 0; j < 3; j++) upd(d.txsz[k][j], s.txsz[k][j], 4, imin(k + 1, 2));
    for (int k = 0; k < 2; k++)
        for (int j = 0; j < 13; j++) upd(d.txtp_intra1[k][j], s.txtp_intra1[k][j], 8, 6);
    for (int k = 0; k < 3; k++)
        for (int j = 0; j < 13; j++) upd(d.txtp_intra2[k][j], s.txtp_intra2[k][j], 8, 4);
    upd_bits(d.skip, s.skip);
    for (int k = 0; k < N_BL; k++)
        for (int j = 0; j < 4; j++) upd(d.partition[k][j], s.partition[k][j], 16, k_part_count[k]);
    CdfCoef &dc = dst.coef;
    const CdfCoef &sc = src.coef;
    for (int k = 0; k < 5; k++) upd_bits(dc.skip[k], sc.skip[k]);
    for (int k = 0; k < 2; k++)
        for (int j = 0; j < 2; j++) {
            upd(dc.eob_bin_16[k][j], sc.eob_bin_16[k][j], 8, 4);
            upd(dc.eob_bin_32[k][j], sc.eob_bin_32[k][j], 8, 5);
            upd(dc.eob_bin_64[k][j], sc.eob_bin_64[k][j], 8, 6);
            upd(dc.eob_bin_128[k][j], sc.eob_bin_128[k][j], 8, 7);
            upd(dc.eob_bin_256[k][j], sc.eob_bin_256[k][j], 16, 8);
        }
    upd_rows(dc.eob_bin_512, sc.eob_bin_512, 9);
    upd_rows(dc.eob_bin_1024, sc.eob_bin_1024, 10);
    for (int k = 0; k < 5; k++)
        for (int j = 0; j < 2; j++) {
            upd_bits(dc.eob_hi_bit[k][j], sc.eob_hi_bit[k][j]);
            upd_rows(dc.eob_base_tok[k][j], sc.eob_base_tok[k][j], 2);
            upd_rows(dc.base_tok[k][j], sc.base_tok[k][j], 3);
        }
    for (int k = 0; k < 2; k++) upd_bits(dc.dc_sign[k], sc.dc_sign[k]);
    for (int k = 0; k < 4; k++)
        for (int j = 0; j < 2; j++) upd_rows(dc.br_tok[k][j], sc.br_tok[k][j], 3);
    upd_rows(d.seg_id, s.seg_id, 7);
    upd(d.cfl_sign, s.cfl_sign, 8, 7);
    upd_rows(d.cfl_alpha, s.cfl_alpha, 15);
    upd_bit(d.restore_wiener, s.restore_wiener);
    upd_bit(d.restore_sgrproj, s.restore_sgrproj);
    upd(d.restore_switchable, s.restore_switchable, 4, 2);
    upd(d.delta_q, s.delta_q, 4, 3);
    upd_rows(d.delta_lf, s.delta_lf, 3);
    for (int k = 0; k < 7; k++) upd_bits(d.pal_y[k], s.pal_y[k]);
    upd_bits(d.pal_uv, s.pal_uv);
    for (int k = 0; k < 2; k++) upd_rows(d.pal_sz[k], s.pal_sz[k], 6);
    for (int k = 0; k < 2; k++)
        for (int j = 0; j < 7; j++)
            for (int i = 0; i < 5; i++) upd(d.color_map[k][j][i], s.color_map[k][j][i], 8, j + 1);
    for (int k = 0; k < 7; k++) upd_bits(d.txpart[k], s.txpart[k]);
    upd_rows(d.txtp_inter1, s.txtp_inter1, 15);
    upd(d.txtp_inter2, s.txtp_inter2, 16, 11);
    upd_bits(d.txtp_inter3, s.txtp_inter3);

    auto upd_mv_common = [&](CdfMv &dm, const CdfMv &sm) {
        upd(dm.joint, sm.joint, 4, 3);
        for (int k = 0; k < 2; k++) {
            upd(dm.comp[k].classes, sm.comp[k].classes, 16, 10);
            upd_bit(dm.comp[k].class0, sm.comp[k].class0);
            upd_bits(dm.comp[k].classN, sm.comp[k].classN);
            upd_bit(dm.comp[k].sign, sm.comp[k].sign);
        }
    };
    if (intra_frame) {
        upd_bit(d.intrabc, s.intrabc);
        upd_mv_common(dst.dmv, src.dmv);
        return;
    }
    upd_bits(d.skip_mode, s.skip_mode);
    upd_rows(d.y_mode, s.y_mode, 12);
    for (int k = 0; k < 2; k++) upd_rows(d.filter[k], s.filter[k], 2);
    upd_bits(d.newmv_mode, s.newmv_mode);
    upd_bits(d.globalmv_mode, s.globalmv_mode);
    upd_bits(d.refmv_mode, s.refmv_mode);
    upd_bits(d.drl_bit, s.drl_bit);
    upd_rows(d.comp_inter_mode, s.comp_inter_mode, 7);
    upd_bits(d.intra, s.intra);
    upd_bits(d.comp, s.comp);
    upd_bits(d.comp_dir, s.comp_dir);
    upd_bits(d.jnt_comp, s.jnt_comp);
    upd_bits(d.mask_comp, s.mask_comp);
    upd_bits(d.wedge_comp, s.wedge_comp);
    upd_rows(d.wedge_idx, s.wedge_idx, 15);
    for (int k = 0; k < 6; k++) upd_bits(d.ref[k], s.ref[k]);
    for (int k = 0; k < 3; k++) upd_bits(d.comp_fwd_ref[k], s.comp_fwd_ref[k]);
    for (int k = 0; k < 2; k++) upd_bits(d.comp_bwd_ref[k], s.comp_bwd_ref[k]);
    for (int k = 0; k < 3; k++) upd_bits(d.comp_uni_ref[k], s.comp_uni_ref[k]);
    upd_bits(d.seg_pred, s.seg_pred);
    upd_bits(d.interintra, s.interintra);
    upd_bits(d.interintra_wedge, s.interintra_wedge);
    upd_rows(d.interintra_mode, s.interintra_mode, 3);
    upd_rows(d.motion_mode, s.motion_mode, 2);
    upd_bits(d.obmc, s.obmc);
    upd_mv_common(dst.mv, src.mv);
    for (int k = 0; k < 2; k++) {
        upd_rows(dst.mv.comp[k].class0_fp, src.mv.comp[k].class0_fp, 3);
        upd(dst.mv.comp[k].classN_fp, src.mv.comp[k].classN_fp, 4, 3);
        upd_bit(dst.mv.comp[k].class0_hp, src.mv.comp[k].class0_hp);
        upd_bit(dst.mv.comp[k].classN_hp, src.mv.comp[k].classN_hp);
    }
}

}  // namespace av1
