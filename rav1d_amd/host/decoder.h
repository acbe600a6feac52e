// decoder.h — the front-end decoder: sequence / frame state, reference slots, and the
// per-frame block decoder that turns a frame's tile data into a FrameWork.
#pragma once
#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "av1.h"
#include "frame.h"

namespace av1 {

// What a reference slot remembers of a decoded frame (picture identity, header, entropy and
// motion state for later frames: decode.rs submit_frame / refs[]).
struct RefSlot {
    int pic_id = -1;
    std::shared_ptr<const FrameHdr> hdr;
    std::shared_ptr<const Cdf> cdf;
    std::shared_ptr<const std::vector<uint8_t>> segmap;
    std::shared_ptr<const std::vector<RefMvBlock>> mvs;   // 8x8-subsampled temporal MVs
    int refpoc[7];
    int bw, bh;   // 4x4-unit frame size the segmap / mvs belong to
    int showable;
};

// One entry of the decoder's output queue: a frame to reconstruct (work != null) and/or a
// picture to output (show_pic >= 0).
struct DecEvent {
    std::shared_ptr<FrameWork> work;
    int pic_id = -1;                 // id of the picture `work` reconstructs
    int ref_pic[7] = {-1, -1, -1, -1, -1, -1, -1};   // pictures its inter prediction reads
    int show_pic = -1;               // picture to output after this event (-1: none)
    MiFilmGrainData fg{};            // grain of the shown picture (if fg_present)
    int fg_present = 0;
    std::vector<int> release;        // pictures no slot references any more
};

class Decoder {
public:
    Decoder();
    // Feed one temporal unit (or any whole number of OBUs). Returns 0 or -errno.
    int send(const uint8_t *data, size_t size);
    bool pop(DecEvent &ev);
    std::string error;

private:
    int parse_obu(const uint8_t *data, size_t size, size_t *used);
    int parse_seq_hdr(Bits &gb, SeqHdr &s);
    int parse_frame_hdr(Bits &gb, FrameHdr &h);
    int read_frame_size(Bits &gb, FrameHdr &h, bool use_ref);
    int submit_frame();
    void update_refs(int pic_id, const std::shared_ptr<const FrameHdr> &hdr,
                     const std::shared_ptr<const Cdf> &cdf, const std::shared_ptr<const std::vector<uint8_t>> &segmap,
                     const std::shared_ptr<const std::vector<RefMvBlock>> &mvs, const int *refpoc, int bw, int bh);
    void release_unused(DecEvent &ev, const int *old_ids);

    std::unique_ptr<SeqHdr> seq_;
    std::shared_ptr<FrameHdr> frame_hdr_;
    RefSlot refs_[8];
    struct TileData { const uint8_t *data; size_t size; int start, end; };
    std::vector<TileData> tiles_;
    std::vector<std::vector<uint8_t>> tile_bufs_;
    int n_tiles_ = 0;
    int next_pic_ = 0;
    std::deque<DecEvent> out_;
};

// Decode one frame's tiles (decode.rs decode_frame_init + decode_tile_sbrow over every tile)
// into `work`. Returns 0 or -errno. Fills the state later frames need.
struct FrameResult {
    std::shared_ptr<Cdf> out_cdf;                           // refresh_context
    std::shared_ptr<std::vector<uint8_t>> segmap;
    std::shared_ptr<std::vector<RefMvBlock>> mvs;
};
struct FrameInputs {
    const SeqHdr *seq;
    const FrameHdr *hdr;
    const Cdf *in_cdf;                                      // nullptr: defaults for base_q_idx
    const RefSlot *refs[7];                                 // slots of refidx[0..6] (inter)
    std::shared_ptr<const std::vector<uint8_t>> prev_segmap;
    struct Tile { const uint8_t *data; size_t size; };
    std::vector<Tile> tiles;                                // in tile order
};
int decode_frame(const FrameInputs &in, FrameWork &work, FrameResult &res, std::string &err);

}  // namespace av1
