// frame.h — per-frame state of the front-end and the pass-2 work list it produces.
#pragma once
#include <array>
#include <memory>
#include <vector>

#include "av1.h"
#include "mi_av1dec.h"

namespace mi_plan { struct IntraQueue; }

namespace av1 {

// Above (frame-wide, indexed by 4x4 column) or left (indexed by 4x4 row & 31) block context:
// the reference's BlockContext (src/env.rs; C src/env.h:39-56).
struct BlockCtx {
    std::vector<uint8_t> mode, lcoef, ccoef[2], seg_pred, skip, skip_mode, intra, comp_type;
    std::vector<uint8_t> filter[2], tx_lpf_y, tx_lpf_uv, partition, uvmode, pal_sz;
    std::vector<int8_t> ref[2], tx_intra, tx;
    void alloc(int n);
    void reset(bool keyframe);
};

// One motion vector / reference pair per 4x4 unit (refmvs.rs refmvs_block)
struct Mv { int16_t y, x; };
inline bool operator==(Mv a, Mv b) { return a.y == b.y && a.x == b.x; }
struct RefMvBlock {
    Mv mv[2];
    int8_t ref[2];     // 0 intra, 1..7 = LAST..ALTREF, -1 none
    uint8_t bs, mf;    // mf: 1 = globalmv with a warped global model, 2 = newmv
};
// One saved motion vector per 8x8 for later frames' temporal prediction (refmvs.rs
// refmvs_temporal_block; C refmvs.h): ref 0 = none
struct TmvBlock {
    Mv mv;
    int8_t ref;
};

struct LfLvl { uint8_t v[8][4][8][2]; };   // [seg][plane/dir][ref][mode] (lf_mask.rs lflvl)

// The pass-2 work of one frame (descriptors of include/mi_av1dsp.h) plus the frame-level
// parameters of the loop filters and film grain.
struct FrameWork {
    int w, h, up_w, render_w, render_h, bpc, layout, ss_hor, ss_ver, sb128, intra_only;
    // intra path in decode order: prediction blocks with their residuals and dependencies
    std::vector<MiIntraBlock> intra;
    std::vector<MiTxBlock> intra_tx;
    std::vector<int32_t> dep_start, deps;
    // residuals of inter blocks (no intra dependency)
    std::vector<MiTxBlock> inter_tx;
    // inter prediction (recon_b_inter's mc / obmc / warp_affine / compound calls as descriptors,
    // run before the residuals): main units (put, compound, MI_MC_PREP sides), OBMC laps (all
    // above laps, then all left laps), warped 8x8s, scaled-reference units, compound combines
    // (all luma, then all chroma), the mask arena (MASK inputs, SEG outputs) and the int16
    // elements of the tmp arena the prep sides write
    std::vector<MiMcBlock> mc, obmc_h, obmc_v, scaled;
    std::vector<MiWarpBlock> warp;
    std::vector<MiMcCombine> combine_y, combine_uv;
    std::vector<uint8_t> masks;
    size_t ntmp = 0;
    // coefficient arena: int16 (8 bpc) or int32 (10/12 bpc) values, as bytes
    std::vector<uint8_t> coef;
    size_t ncoef;
    std::vector<uint8_t> idx;            // palette indices / inter-intra masks
    std::vector<uint8_t> pal;            // palette colours (pixels of bpc)
    // deblocking
    int filter_y, filter_uv;
    std::vector<uint8_t> lf_level;       // [b4 rows][b4_stride][4]
    int b4_stride;
    std::vector<MiAv1Filter> lf_masks;   // [sb128h][sb128w]
    int sb128w, sb128h;
    uint8_t lim_e[64], lim_i[64];
    // cdef
    int cdef_on, cdef_damping;
    uint8_t cdef_y[8], cdef_uv[8];
    // loop restoration
    std::vector<MiAv1Restoration> lr_mask;   // [sb128h][sr_sb128w]
    int sr_sb128w, restore_planes, lr_unit_size[2];
    // film grain (applied to the output only)
    int fg_present;
    MiFilmGrainData fg;
    // the intra queue of the frame executor (csrc/intra_plan.h), planned by plan_intra_queue
    std::shared_ptr<const mi_plan::IntraQueue> q;
};

// The MiDecFrame of a FrameWork, every in-loop filter as the frame signals it, with the intra
// queue when planned (plan.cpp)
void frame_view(const FrameWork &w, MiDecFrame &f);
// Plan the frame's intra queue into w.q (ranges of blocks on the pool's workers when given)
class WorkerPool;
void plan_intra_queue(FrameWork &w, WorkerPool *pool);

}  // namespace av1
