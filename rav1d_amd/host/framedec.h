// framedec.h — the per-frame block decoder shared by decode.cpp (partition tree, intra blocks,
// coefficients, loop-filter metadata), refmvs.cpp (motion-vector candidate lists and temporal
// MVs) and inter.cpp (inter modes, recon_b_inter's prediction descriptors). Internal to the
// front-end library.
#pragma once
#include <cerrno>
#include <string>
#include <vector>

#include "decoder.h"

namespace av1 {
namespace fd {

template <typename T>
inline void setn(std::vector<T> &v, int off, int n, int val) {
    for (int i = 0; i < n; i++) v[off + i] = (T)val;
}

// Av1Block (levels.rs:285-360; C src/levels.h): what decode_b reads for one block
struct Block {
    int bl, bs, bp, intra, seg_id, skip_mode, skip;
    int y_mode, uv_mode, tx, uvtx, pal_sz[2], y_angle, uv_angle, cfl_alpha[2];
    // inter
    int ref[2], comp_type, inter_mode, drl_idx, motion_mode, interintra_type, interintra_mode;
    int wedge_idx, mask_sign, filter2d, max_ytx, filter[2];
    uint16_t tx_split[2];
    Mv mv[2];
};

enum { II_NONE, II_BLEND, II_WEDGE };

// A view of a frame-wide array owned by FrameShared: the tile decoders of one frame write
// disjoint parts of it (their tiles' 4x4 units, superblocks' mask words, 8x8 MV rows)
template <typename T>
struct Span {
    T *p = nullptr;
    size_t n = 0;
    T &operator[](size_t i) const { return p[i]; }
    T *data() const { return p; }
    size_t size() const { return n; }
    void bind(std::vector<T> &v) {
        p = v.data();
        n = v.size();
    }
    template <typename B>
    void bind(B &v) {
        p = v.data();
        n = v.size();
    }
};

// An array of a plain type left uninitialised: for maps whose entries are only read where the
// frame has written them
template <typename T>
class RawBuf {
public:
    void reset(size_t n) {
        if (n != n_) p_.reset(n ? new T[n] : nullptr);
        n_ = n;
    }
    void clear() { reset(0); }
    T *data() { return p_.get(); }
    size_t size() const { return n_; }

private:
    std::unique_ptr<T[]> p_;
    size_t n_ = 0;
};

// The per-4x4 / per-8x8 maps of a frame that every tile decoder of it reads and writes (within
// its own tile): segment ids, the loop filter's tile-edge contexts, intra owners, refmvs blocks,
// projected and saved temporal MVs
struct FrameShared {
    std::shared_ptr<std::vector<uint8_t>> segmap;   // (published to later frames as it fills)
    std::vector<uint8_t> tx_lpf_right[2];
    std::vector<std::vector<uint8_t>> a_tx_lpf_end[2];
    std::vector<int32_t> owner[3];
    RawBuf<RefMvBlock> rmv;       // (read only where written: no reset value)
    RawBuf<uint8_t> f2d_map;
    std::vector<TmvBlock> rp_proj;
    std::shared_ptr<std::vector<TmvBlock>> rp;
};

struct TileState {
    Cdf cdf;
    Msac msac;
    int col_start, col_end, row_start, row_end;   // 4x4 units
    int last_qidx;
    int8_t last_delta_lf[4];
    uint16_t dq[8][3][2];
    LfLvl lflvl;
    MiAv1RestorationUnit *lr_ref[3];
};

// refmvs_candidate (refmvs.rs; C refmvs.h)
struct MvCand {
    Mv mv[2];
    int weight;
};

class FrameDec {
public:
    // the frame's decoder: its work lists and maps in fw
    FrameDec(const FrameInputs &in, FrameWork &fw)
        : in_(in), s(*in.seq), h(*in.hdr), fw(fw), mw(fw), own_sh_(new FrameShared), S(own_sh_.get()), master_(true) {}
    // a tile decoder of `m`'s frame: its blocks' work lists in `own` (merged by the frame's
    // decoder afterwards), the frame's maps in m's FrameWork and FrameShared
    FrameDec(const FrameDec &m, FrameWork &own)
        : in_(m.in_), s(m.s), h(m.h), fw(own), mw(m.fw), S(m.S), master_(false), in_cdf_(m.in_cdf_), ts_(m.ts_) {}
    // with in.pool: the frame's tiles decoded on its workers (rav1d's tile threads)
    int run(FrameResult &res, std::string &err);

private:
    const FrameInputs &in_;
    const SeqHdr &s;
    const FrameHdr &h;
    FrameWork &fw;        // work lists of the blocks this decoder decodes
    FrameWork &mw;        // the frame's loop-filter / CDEF / LR maps (== fw for the frame's decoder)
    std::unique_ptr<FrameShared> own_sh_;
    FrameShared *S;
    const bool master_;
    const Cdf *in_cdf_ = nullptr;   // in.in_cdf, or once ready the cdf of in.in_cdf_prog
    std::shared_ptr<const Cdf> in_cdf_hold_;
    int init_frame();
    int decode_tile(int k, bool tile_tmvs);
    // before superblock row `by`: the references still decoding have finished the saved MVs and
    // segment ids this row reads (frame threads; -EINVAL when one failed)
    int wait_refs(int by);
    std::shared_ptr<const Cdf> out_cdf();
    void merge_tile(const FrameWork &t);

    int bw, bh, w4, h4, sb128w, sb128h, sb_shift, sb_step, sbh, b4_stride, layout, ss_hor, ss_ver, hbd_idx;
    uint16_t dq_frame[8][3][2];
    LfLvl lflvl_frame;
    std::vector<TileState> ts_stor_;
    std::vector<TileState> &ts_ = ts_stor_;   // (a tile decoder's refers to the frame decoder's)
    TileState *ts = nullptr;
    BlockCtx a, l;
    int bx = 0, by = 0;
    int8_t *cur_cdef_idx = nullptr;
    MiAv1Filter *lf_mask = nullptr;
    uint16_t al_pal[2][32][3][8];            // [above / left][pos][plane][entry]
    uint8_t pal_sz_uv[2][32];
    Span<uint8_t> segmap;
    Span<uint8_t> tx_lpf_right[2];           // per tile column: left context at the tile's right edge
    Span<int32_t> owner[3];                  // per plane, per 4x4: index (in its tile's list) of the intra block there
    int owner_stride;
    std::string *err_ = nullptr;
    bool inter_frame = false;

    int fail(const char *m) {
        if (err_) *err_ = m;
        return -EINVAL;
    }
    int unsupported(const char *m) {
        if (err_) *err_ = m;
        return -ENOTSUP;
    }
    void init_quant(int qidx, uint16_t (*dq)[3][2]);
    void calc_lf_values(LfLvl &out, const int8_t delta[4]);
    void setup_tile(TileState &t, const uint8_t *data, size_t sz, int row, int col);
    int decode_tile_sbrow(int tile_row, int tile_col);
    void read_lr(MiAv1RestorationUnit *lr, int p, int frame_type);
    int decode_sb(int bl, bool tr, bool lb);
    int decode_b(int bl, int bs, int bp, int edge_flags);
    void read_pal_plane(Block &b, int pl, int sz_ctx, int bx4, int by4, uint16_t *pal);
    void read_pal_uv(Block &b, int sz_ctx, int bx4, int by4, uint16_t (*pal)[8]);
    void read_pal_indices(uint8_t *idx, const Block &b, int pl, int w4, int h4, int bw4, int bh4);
    int decode_coefs(uint8_t *actx, uint8_t *lctx, int tx, int bs, const Block &b, int intra, int plane, int32_t *cf,
                     int *txtp, uint8_t *res_ctx);
    void emit_intra(const Block &b, int edge_flags, const uint8_t *pal_idx, const uint16_t (*pal)[8]);
    uint32_t store_coefs(const int32_t *cf, int tx, int txtp, int eob, uint8_t *flags);
    void add_deps(int plane, int x0, int y0, int x1, int y1, std::vector<int32_t> &out);
    void mask_edges_intra(int by4, int bx4, int w4_, int h4_, int tx, uint8_t *actx, uint8_t *lctx, uint16_t (*masks)[32][3][2]);
    void mask_edges_chroma(int cby4, int cbx4, int cw4, int ch4, int skip_inter, int tx, uint8_t *actx, uint8_t *lctx,
                           uint16_t (*masks)[32][2][2]);
    void create_lf_mask_intra(const Block &b, int has_chroma);
    void tile_fixups();

    // motion-vector state: the frame's refmvs blocks (per 4x4, padded by 8 units on each side)
    // and the per-4x4 Filter2d of inter blocks (frame_thread.b[].filter2d)
    Span<RefMvBlock> rmv;
    Span<uint8_t> f2d_map;
    int rmv_stride = 0;
    std::vector<int32_t> dep_tmp;     // one block's dependency list (reused)
    std::vector<uint32_t> dep_seen;   // add_deps: per owner, the stamp of the list holding it
    uint32_t dep_stamp = 0;
    RefMvBlock &rmv_at(int y4, int x4) { return rmv[(size_t)(y4 + 8) * rmv_stride + (x4 + 8)]; }
    uint8_t &f2d_at(int y4, int x4) { return f2d_map[(size_t)(y4 + 8) * rmv_stride + (x4 + 8)]; }
    void splat(const RefMvBlock &r, int bw4, int bh4);
    void splat_rmv(int bs, int bw4, int bh4, Mv mv, bool valid);
    void find_dv(int bs, int edge_flags, Mv stack[2]);
    int read_mv_comp(CdfMvComp &c, int have_fp);
    void read_mv_residual(Mv &mv, CdfMv &cdf, int have_fp);
    void read_tx_tree(int from, int depth, uint16_t *masks, int x_off, int y_off, int tbx, int tby);
    void read_vartx_tree(Block &b, int bs);
    void ibc_residual_tree(const Block &b, Mv mv, int tx, int depth, const uint16_t *split, int x_off, int y_off,
                           int tbx, int tby, uint8_t (*txtp_map)[32]);
    void push_ibc(const Block &b, Mv mv, int plane, int tx, int tbx, int tby, int px, int py, int eob_txtp_read,
                  uint8_t *actx, uint8_t *lctx, int nact, int nlct, int *txtp);
    int decode_ibc(Block &b, int bs, int edge_flags, int has_chroma);

    // ---- refmvs.cpp: rav1d_refmvs_* (refmvs.rs; C refmvs.c) --------------------------------
    int iw4 = 0, ih4 = 0, iw8 = 0, ih8 = 0;
    uint8_t sign_bias[7] = {}, mfmv_sign[7] = {};
    int8_t pocdiff[7] = {};
    int n_mfmvs = 0, mfmv_ref[3] = {}, mfmv_ref2cur[3] = {}, mfmv_ref2ref[3][7] = {};
    int rp_stride = 0;
    Span<TmvBlock> rp_proj;           // projected temporal MVs (8x8 rows of the frame)
    std::shared_ptr<std::vector<TmvBlock>> rp;   // this frame's saved MVs (save_tmvs)
    const TmvBlock *rp_ref[7] = {};
    void refmvs_init_frame();
    void load_tmvs(int row_start8, int row_end8, int col_start8, int col_end8);
    void save_tmvs(int row_start8, int row_end8, int col_start8, int col_end8);
    void refmvs_find(MvCand stack[8], int *cnt, int *ctx, int ref0, int ref1, int bs, int edge_flags);
    Mv gmv_2d(int ref, int bw4, int bh4) const;
    void fix_mv(Mv &mv) const;

    // ---- inter.cpp: decode_b's inter branch and recon_b_inter's descriptors ---------------
    WarpParams gmv[7];                 // frame_hdr.gmv with the shear parameters derived
    int gmv_warp_allowed[7] = {};
    int svc_scale[7][2] = {}, svc_step[7][2] = {};
    int jnt_weights[7][7] = {};
    WarpParams warpmv;                 // t.warpmv of the current block
    void inter_frame_init();
    int decode_inter(Block &b, int bs, int edge_flags, int has_chroma, int have_left, int have_top, const SegData *seg,
                     int seg_pred);
    void find_matching_ref(int edge_flags, int bw4, int bh4, int w4b, int h4b, int have_left, int have_top, int ref,
                           uint64_t masks[2]);
    void derive_warpmv(int bw4, int bh4, const uint64_t masks[2], Mv mv, WarpParams &wm);
    void mask_edges_inter(int by4, int bx4, int w4_, int h4_, int skip, int max_tx, const uint16_t *tx_masks,
                          uint8_t *actx, uint8_t *lctx, uint16_t (*masks)[32][3][2]);
    void create_lf_mask_inter(const Block &b, int has_chroma);
    int emit_inter_pred(const Block &b, int has_chroma);
    void emit_inter_residual(const Block &b, int has_chroma);
    int push_obmc(const Block &b, int bw4, int bh4, int w4b, int h4b);
    void push_warp(const Block &b, int plane, const WarpParams &wm, int ref, int prep, uint32_t tmp_off);
    uint32_t add_mask(const uint8_t *m, int n);
    void emit_interintra(const Block &b, int has_chroma);
};

// wedge.rs / C wedge.c: the wedge masks (wedge_idx 16, sign 2) and the inter-intra masks
// (4 modes), per block size and layout class (0 444, 1 422, 2 420); nullptr where the size has
// none
const uint8_t *wedge_mask(int bs, int layout_cls, int sign, int idx);
const uint8_t *ii_mask(int bs, int layout_cls, int mode);
// warpmv.rs / C warpmv.c
int get_shear_params(WarpParams &wm);
int find_affine_int(const int (*pts)[2][2], int np, int bw4, int bh4, Mv mv, WarpParams &wm, int bx4, int by4);
void set_affine_mv2d(int bw4, int bh4, Mv mv, WarpParams &wm, int bx4, int by4);

}  // namespace fd
}  // namespace av1
