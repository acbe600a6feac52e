// av1.h — host front-end of the MI355X AV1 decode path: shared types of the bitstream side.
//
// This is the CPU half that rav1d keeps on the host (north_star): OBU/header parsing
// (src/obu.rs:2662; C src/obu.c), the msac range decoder (src/msac.rs; C src/msac.c), block
// mode and coefficient decoding (src/decode.rs:1131-4067, src/recon.rs:478-2023; C
// src/decode.c, src/recon_tmpl.c:49-960), loop-filter level / mask creation (src/lf_mask.rs;
// C src/lf_mask.c). Its output is not pixels but the descriptor lists of include/mi_av1dsp.h
// that the gfx950 kernels (or the CPU oracle, in tests) turn into pixels.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "mi_av1dsp.h"

namespace av1 {

// ---- enums (values as the AV1 spec / the reference's levels.rs) ---------------------------
enum BlockLevel { BL_128, BL_64, BL_32, BL_16, BL_8, N_BL };
enum Partition { P_NONE, P_H, P_V, P_SPLIT, P_T_TOP, P_T_BOTTOM, P_T_LEFT, P_T_RIGHT, P_H4, P_V4, N_PART };
// block sizes, largest first (levels.rs BlockSize)
enum BlockSize {
    BS_128x128, BS_128x64, BS_64x128, BS_64x64, BS_64x32, BS_64x16, BS_32x64, BS_32x32, BS_32x16,
    BS_32x8, BS_16x64, BS_16x32, BS_16x16, BS_16x8, BS_16x4, BS_8x32, BS_8x16, BS_8x8, BS_8x4,
    BS_4x16, BS_4x8, BS_4x4, N_BS
};
enum TxSize {
    TX_4X4, TX_8X8, TX_16X16, TX_32X32, TX_64X64, TX_4X8, TX_8X4, TX_8X16, TX_16X8, TX_16X32,
    TX_32X16, TX_32X64, TX_64X32, TX_4X16, TX_16X4, TX_8X32, TX_32X8, TX_16X64, TX_64X16, N_TX
};
enum TxType {
    DCT_DCT, ADST_DCT, DCT_ADST, ADST_ADST, FLIPADST_DCT, DCT_FLIPADST, FLIPADST_FLIPADST,
    ADST_FLIPADST, FLIPADST_ADST, IDTX, V_DCT, H_DCT, V_ADST, H_ADST, V_FLIPADST, H_FLIPADST, WHT_WHT
};
enum IntraMode {
    DC_PRED, V_PRED, H_PRED, D45_PRED, D135_PRED, D113_PRED, D157_PRED, D203_PRED, D67_PRED,
    SMOOTH_PRED, SMOOTH_V_PRED, SMOOTH_H_PRED, PAETH_PRED, N_INTRA_MODES,
    CFL_PRED = N_INTRA_MODES, FILTER_PRED = N_INTRA_MODES
};
enum FrameType { FRAME_KEY, FRAME_INTER, FRAME_INTRA, FRAME_SWITCH };
enum RestorationType { RESTORE_NONE, RESTORE_SWITCHABLE, RESTORE_WIENER, RESTORE_SGRPROJ };
enum TxMode { TXMODE_4X4_ONLY, TXMODE_LARGEST, TXMODE_SWITCHABLE };
enum WarpType { WM_IDENTITY, WM_TRANSLATION, WM_ROT_ZOOM, WM_AFFINE };
enum FilterMode { FILTER_REGULAR, FILTER_SMOOTH, FILTER_SHARP, FILTER_BILINEAR, FILTER_SWITCHABLE };
enum InterMode { NEARESTMV, NEARMV, GLOBALMV, NEWMV };
enum CompInterMode {
    NEARESTMV_NEARESTMV, NEARMV_NEARMV, NEARESTMV_NEWMV, NEWMV_NEARESTMV, NEARMV_NEWMV,
    NEWMV_NEARMV, GLOBALMV_GLOBALMV, NEWMV_NEWMV
};
enum CompType { COMP_NONE, COMP_WAVG, COMP_AVG, COMP_SEG, COMP_WEDGE };
enum MotionMode { MM_TRANSLATION, MM_OBMC, MM_WARP };

// edge availability bits of the partition tree (intra_edge.rs EdgeFlags)
enum EdgeFlag {
    E444_TR = 1, E422_TR = 2, E420_TR = 4, E444_BL = 8, E422_BL = 16, E420_BL = 32,
    E_ALL_TR = 7, E_ALL_BL = 56
};

// ---- static tables ------------------------------------------------------------------------
struct BlockDim { uint8_t w4, h4, lw4, lh4; };   // size in 4-px units and log2 of it
struct TxDim { uint8_t w, h, lw, lh, min, max, sub, ctx; };
extern const BlockDim k_bdim[N_BS];
extern const TxDim k_txdim[N_TX];
extern const uint8_t k_max_tx_for_bs[N_BS][4];       // [bs][0 luma, layout 1..3 chroma]
extern const uint8_t k_block_sizes[N_BL][N_PART][2];
extern const uint8_t k_part_ctx_val[2][N_BL][N_PART];   // above / left partition context bits
extern const uint8_t k_part_count[N_BL];
extern const uint8_t k_txtp_from_uvmode[14];
extern const uint8_t k_tx_types_per_set[40];
extern const uint8_t k_ymode_size_ctx[N_BS];
extern const uint8_t k_lo_ctx_offsets[3][5][5];
extern const uint8_t k_skip_ctx[5][5];
extern const uint8_t k_tx_class[17];                  // 0 2-D, 1 horizontal, 2 vertical
extern const uint8_t k_intra_mode_ctx[N_INTRA_MODES];
extern const uint8_t k_filter_mode_to_y_mode[5];
extern const uint16_t k_sgr_params[16][2];
extern const uint16_t *k_scan[N_TX];
int dq_value(int hbd_idx, int qidx, int ac);   // dav1d_dq_tbl[hbd_idx][qidx][ac]
const uint8_t *qm_table(int level, int chroma, int tx);   // nullptr for level 15
extern const uint8_t k_filter_2d[4][4];               // [h filter][v filter] -> Filter2d
extern const uint8_t k_filter_dir[10][2];
extern const uint8_t k_wedge_ctx[N_BS];
extern const uint8_t k_comp_inter_modes[8][2];

inline int imin(int a, int b) { return a < b ? a : b; }
inline int imax(int a, int b) { return a > b ? a : b; }
inline int iclip(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
inline int ulog2(unsigned v) { return 31 - __builtin_clz(v); }

// ---- CDF context (the reference's CdfContext, src/cdf.rs; stored as 32768 - cdf with the
// adaptation counter in slot n_symbols) ----------------------------------------------------
struct CdfMode {
    uint16_t y_mode[4][16];
    uint16_t uv_mode[2][13][16];
    uint16_t wedge_idx[9][16];
    uint16_t partition[N_BL][4][16];
    uint16_t cfl_alpha[6][16];
    uint16_t txtp_inter1[2][16];
    uint16_t txtp_inter2[16];
    uint16_t txtp_intra1[2][13][8];
    uint16_t txtp_intra2[3][13][8];
    uint16_t cfl_sign[8];
    uint16_t angle_delta[8][8];
    uint16_t filter_intra[8];
    uint16_t comp_inter_mode[8][8];
    uint16_t seg_id[3][8];
    uint16_t pal_sz[2][7][8];
    uint16_t color_map[2][7][5][8];
    uint16_t filter[2][8][4];
    uint16_t txsz[4][3][4];
    uint16_t motion_mode[N_BS][4];
    uint16_t delta_q[4];
    uint16_t delta_lf[5][4];
    uint16_t interintra_mode[4][4];
    uint16_t restore_switchable[4];
    uint16_t restore_wiener[2];
    uint16_t restore_sgrproj[2];
    uint16_t interintra[7][2];
    uint16_t interintra_wedge[7][2];
    uint16_t txtp_inter3[4][2];
    uint16_t use_filter_intra[N_BS][2];
    uint16_t newmv_mode[6][2];
    uint16_t globalmv_mode[2][2];
    uint16_t refmv_mode[6][2];
    uint16_t drl_bit[3][2];
    uint16_t intra[4][2];
    uint16_t comp[5][2];
    uint16_t comp_dir[5][2];
    uint16_t jnt_comp[6][2];
    uint16_t mask_comp[6][2];
    uint16_t wedge_comp[9][2];
    uint16_t ref[6][3][2];
    uint16_t comp_fwd_ref[3][3][2];
    uint16_t comp_bwd_ref[2][3][2];
    uint16_t comp_uni_ref[3][3][2];
    uint16_t txpart[7][3][2];
    uint16_t skip[3][2];
    uint16_t skip_mode[3][2];
    uint16_t seg_pred[3][2];
    uint16_t obmc[N_BS][2];
    uint16_t pal_y[7][3][2];
    uint16_t pal_uv[2][2];
    uint16_t intrabc[2];
};
struct CdfCoef {
    uint16_t eob_bin_16[2][2][8];
    uint16_t eob_bin_32[2][2][8];
    uint16_t eob_bin_64[2][2][8];
    uint16_t eob_bin_128[2][2][8];
    uint16_t eob_bin_256[2][2][16];
    uint16_t eob_bin_512[2][16];
    uint16_t eob_bin_1024[2][16];
    uint16_t eob_base_tok[5][2][4][4];
    uint16_t base_tok[5][2][41][4];
    uint16_t br_tok[4][2][21][4];
    uint16_t eob_hi_bit[5][2][11][2];
    uint16_t skip[5][13][2];
    uint16_t dc_sign[2][3][2];
};
struct CdfMvComp {
    uint16_t classes[16];
    uint16_t class0_fp[2][4];
    uint16_t classN_fp[4];
    uint16_t class0_hp[2];
    uint16_t classN_hp[2];
    uint16_t class0[2];
    uint16_t classN[10][2];
    uint16_t sign[2];
};
struct CdfMv { CdfMvComp comp[2]; uint16_t joint[4]; };
struct Cdf {
    CdfMode m;
    uint16_t kfym[5][5][16];
    CdfCoef coef;
    CdfMv mv, dmv;
};
void cdf_init_default(Cdf &c, int base_qidx);
// End-of-frame CDF propagation (cdf.rs / C cdf.c dav1d_cdf_thread_update): dst := src for the
// adapted tables (counters cleared); dst keeps its other tables.
void cdf_update_frame(Cdf &dst, const Cdf &src, bool intra_frame);

// ---- msac (src/msac.rs) -------------------------------------------------------------------
struct Msac {
    const uint8_t *pos, *end;
    uint64_t dif;
    unsigned rng;
    int cnt;
    bool adapt;
    void init(const uint8_t *data, size_t sz, bool disable_update);
    void refill();
    void norm(uint64_t d, unsigned r);
    unsigned bool_equi();
    unsigned bool_prob(unsigned f);
    unsigned bools(unsigned n) {
        unsigned v = 0;
        while (n--) v = (v << 1) | bool_equi();
        return v;
    }
    unsigned symbol(uint16_t *cdf, unsigned n_symbols);   // n_symbols = count - 1
    unsigned bool_adapt(uint16_t *cdf);
    unsigned hi_tok(uint16_t *cdf);
    int uniform(unsigned n);
    int subexp(int ref, int n, unsigned k);
    unsigned golomb();
};

// the per-symbol paths, inline in every caller (the front-end's hottest code)
static constexpr int kWin = 64;
inline void Msac::norm(uint64_t d, unsigned r) {
    const int s = 15 ^ (31 ^ __builtin_clz(r));
    cnt -= s;
    dif = ((d + 1) << s) - 1;   // ones shifted into the low bits
    rng = r << s;
    if (cnt < 0) refill();
}

inline unsigned Msac::bool_equi() {
    unsigned v = ((rng >> 8) << 7) + 4;
    const uint64_t vw = (uint64_t)v << (kWin - 16);
    const unsigned ret = dif >= vw;
    uint64_t d = dif - ret * vw;
    v += ret * (rng - 2 * v);
    norm(d, v);
    return !ret;
}

inline unsigned Msac::bool_prob(unsigned f) {
    unsigned v = ((rng >> 8) * (f >> 6) >> 1) + 4;
    const uint64_t vw = (uint64_t)v << (kWin - 16);
    const unsigned ret = dif >= vw;
    uint64_t d = dif - ret * vw;
    v += ret * (rng - 2 * v);
    norm(d, v);
    return !ret;
}

inline unsigned Msac::symbol(uint16_t *cdf, unsigned n) {
    const unsigned c = (unsigned)(dif >> (kWin - 16)), r = rng >> 8;
    unsigned u, v = rng, val = (unsigned)-1;
    do {
        val++;
        u = v;
        v = (r * (cdf[val] >> 6) >> 1) + 4 * (n - val);
    } while (c < v);
    norm(dif - ((uint64_t)v << (kWin - 16)), u - v);
    if (adapt) {
        const unsigned count = cdf[n];
        const unsigned rate = 4 + (count >> 4) + (n > 2);
        unsigned i = 0;
        for (; i < val; i++) cdf[i] += (32768 - cdf[i]) >> rate;
        for (; i < n; i++) cdf[i] -= cdf[i] >> rate;
        cdf[n] = count + (count < 32);
    }
    return val;
}

inline unsigned Msac::bool_adapt(uint16_t *cdf) {
    const unsigned b = bool_prob(cdf[0]);
    if (adapt) {
        const unsigned count = cdf[1];
        const int rate = 4 + (count >> 4);
        if (b) cdf[0] += (32768 - cdf[0]) >> rate;
        else cdf[0] -= cdf[0] >> rate;
        cdf[1] = count + (count < 32);
    }
    return b;
}

inline unsigned Msac::hi_tok(uint16_t *cdf) {
    unsigned tok = 3, br;
    do {
        br = symbol(cdf, 3);
        tok += br;
    } while (br == 3 && tok < 15);
    return tok;
}


// ---- headers ------------------------------------------------------------------------------
struct SeqHdr {
    int profile, still_picture, reduced_still;
    int timing_info_present, decoder_model_info_present, equal_picture_interval;
    int buffer_delay_len, buffer_removal_delay_len, frame_presentation_delay_len;
    int num_op, op_idc[32], op_decoder_model_present[32];
    int width_n_bits, height_n_bits, max_width, max_height;
    int frame_id_numbers_present, delta_frame_id_n_bits, frame_id_n_bits;
    int sb128, filter_intra, intra_edge_filter, inter_intra, masked_compound, warped_motion;
    int dual_filter, order_hint, jnt_comp, ref_frame_mvs, screen_content_tools, force_integer_mv;
    int order_hint_n_bits, super_res, cdef, restoration;
    int hbd, bpc, monochrome, color_description_present, pri, trc, mtrx, color_range;
    int layout, ss_hor, ss_ver, chr, separate_uv_delta_q, film_grain_present;
};

struct WarpParams {
    int type;
    int32_t matrix[6];
    int16_t abcd[4];   // alpha, beta, gamma, delta (after shear derivation)
};

struct SegData {
    int delta_q, delta_lf_y_v, delta_lf_y_h, delta_lf_u, delta_lf_v, ref, skip, globalmv;
};

struct FrameHdr {
    int show_existing_frame, existing_frame_idx;
    int frame_type, show_frame, showable_frame, error_resilient, disable_cdf_update;
    int allow_screen_content_tools, force_integer_mv, frame_id, frame_size_override;
    int frame_offset, primary_ref_frame, refresh_frame_flags;
    int width[2], height, render_width, render_height, superres_enabled, superres_denom;
    int allow_intrabc, refidx[7], hp, subpel_filter_mode, switchable_motion_mode, use_ref_frame_mvs;
    int refresh_context;
    struct {
        int uniform, cols, rows, log2_cols, log2_rows, min_log2_cols, max_log2_cols, max_log2_rows;
        int min_log2_rows, col_start_sb[65], row_start_sb[65], update, n_bytes;
    } tiling;
    struct { int yac, ydc_delta, udc_delta, uac_delta, vdc_delta, vac_delta, qm, qm_y, qm_u, qm_v; } quant;
    struct {
        int enabled, update_map, temporal, update_data;
        SegData d[8];
        int preskip, last_active_segid;
        int qidx[8], lossless[8];
    } seg;
    struct { int q_present, q_res_log2, lf_present, lf_res_log2, lf_multi; } delta;
    int all_lossless;
    struct {
        int level_y[2], level_u, level_v, sharpness, mode_ref_delta_enabled, mode_ref_delta_update;
        int mode_delta[2], ref_delta[8];
    } lf;
    struct { int damping, n_bits, y_strength[8], uv_strength[8]; } cdef;
    struct { int type[3], unit_size[2]; } lr;
    int txfm_mode, switchable_comp_refs, skip_mode_allowed, skip_mode_enabled, skip_mode_refs[2];
    int warp_motion, reduced_txtp_set;
    WarpParams gmv[7];
    struct { int present, update; MiFilmGrainData data; } fg;
    int temporal_id, spatial_id;
};

inline bool is_intra_frame(const FrameHdr &h) { return h.frame_type == FRAME_KEY || h.frame_type == FRAME_INTRA; }

// bit reader for the uncompressed headers (getbits.rs)
struct Bits {
    const uint8_t *data;
    size_t size, pos;   // pos in bits
    bool error;
    void init(const uint8_t *d, size_t n) { data = d; size = n; pos = 0; error = false; }
    unsigned bit() {
        if (pos >= size * 8) { error = true; pos++; return 0; }
        const unsigned b = (data[pos >> 3] >> (7 - (pos & 7))) & 1;
        pos++;
        return b;
    }
    unsigned bits(int n) {
        unsigned v = 0;
        while (n--) v = (v << 1) | bit();
        return v;
    }
    int sbits(int n) {   // n-bit two's complement
        const unsigned v = bits(n);
        return (int)(v << (32 - n)) >> (32 - n);
    }
    unsigned uleb128();
    unsigned uniform(unsigned max);
    unsigned vlc();
    int subexp(int ref, int n);
    void byte_align() { pos = (pos + 7) & ~(size_t)7; }
    size_t byte_pos() const { return pos >> 3; }
};

}  // namespace av1
