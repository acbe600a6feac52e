// decoder.h — the front-end decoder: sequence / frame state, reference slots, and the
// per-frame block decoder that turns a frame's tile data into a FrameWork.
#pragma once
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <memory>
#include <string>
#include <vector>

#include "av1.h"
#include "frame.h"

namespace av1 {

// What a reference slot remembers of a decoded frame (picture identity, header, entropy and
// motion state for later frames: decode.rs submit_frame / refs[]).
struct FrameJob;

struct RefSlot {
    int pic_id = -1;
    // set while the frame that refreshed this slot is still being decoded on a worker thread:
    // cdf (when cdf_from_job), segmap and mvs come from the job's result (Decoder::resolve)
    std::shared_ptr<FrameJob> job;
    bool cdf_from_job = false, mvs_from_job = false;
    std::shared_ptr<const FrameHdr> hdr;
    std::shared_ptr<const Cdf> cdf;
    std::shared_ptr<const std::vector<uint8_t>> segmap;
    std::shared_ptr<const std::vector<TmvBlock>> mvs;   // 8x8-subsampled temporal MVs (save_tmvs)
    int refpoc[7];
    int bw, bh;   // 4x4-unit frame size the segmap / mvs belong to
    int showable;
};

// One entry of the decoder's output queue: a frame to reconstruct (work != null) and/or a
// picture to output (show_pic >= 0).
struct DecEvent {
    std::shared_ptr<FrameWork> work;
    std::shared_ptr<FrameJob> job;   // the worker decoding `work` (threads > 1), joined by pop()
    int pic_id = -1;                 // id of the picture `work` reconstructs
    int ref_pic[7] = {-1, -1, -1, -1, -1, -1, -1};   // pictures its inter prediction reads
    int show_pic = -1;               // picture to output after this event (-1: none)
    MiFilmGrainData fg{};            // grain of the shown picture (if fg_present)
    int fg_present = 0;
    int mtrx_identity = 0;           // the grain's chroma clip (seq_hdr.mtrx == MC_IDENTITY)
    std::vector<int> release;        // pictures no slot references any more
};

class Decoder {
public:
    Decoder();
    // Feed one temporal unit (or any whole number of OBUs). Returns 0 or -errno.
    int send(const uint8_t *data, size_t size);
    // 1 and ev filled, 0 when no event is queued, or -errno (a frame decoded on a worker
    // thread failed; error explains). Waits for the oldest frame's worker.
    int pop(DecEvent &ev);
    // Frame threads (rav1d's n_fc): frames are decoded on up to n worker threads while send()
    // parses on (an inter frame's job waits for the jobs of its references), each frame's
    // tiles on up to n threads; events still come out in decode order. 1 (default): synchronous.
    void set_threads(int n) { threads_ = n < 1 ? 1 : n > 64 ? 64 : n; }
    ~Decoder();
    std::string error;

private:
    int parse_obu(const uint8_t *data, size_t size, size_t *used);
    int parse_seq_hdr(Bits &gb, SeqHdr &s);
    int parse_frame_hdr(Bits &gb, FrameHdr &h);
    int read_frame_size(Bits &gb, FrameHdr &h, bool use_ref);
    int submit_frame();
    void update_refs(int pic_id, const std::shared_ptr<const FrameHdr> &hdr,
                     const std::shared_ptr<const Cdf> &cdf, const std::shared_ptr<const std::vector<uint8_t>> &segmap,
                     const std::shared_ptr<const std::vector<TmvBlock>> &mvs, const int *refpoc, int bw, int bh);
    void release_unused(DecEvent &ev, const int *old_ids);
    void resolve(RefSlot &r);
    void resolve_all();

    std::unique_ptr<SeqHdr> seq_;
    std::shared_ptr<FrameHdr> frame_hdr_;
    RefSlot refs_[8];
    struct TileData { const uint8_t *data; size_t size; int start, end; };
    std::vector<TileData> tiles_;
    std::vector<std::shared_ptr<std::vector<uint8_t>>> tile_bufs_;
    int threads_ = 1;
    std::deque<std::shared_ptr<FrameJob>> running_;
    int n_tiles_ = 0;
    int next_pic_ = 0;
    std::deque<DecEvent> out_;
};

// Decode one frame's tiles (decode.rs decode_frame_init + decode_tile_sbrow over every tile)
// into `work`. Returns 0 or -errno. Fills the state later frames need.
struct FrameResult {
    std::shared_ptr<Cdf> out_cdf;                           // refresh_context
    std::shared_ptr<std::vector<uint8_t>> segmap;
    std::shared_ptr<std::vector<TmvBlock>> mvs;
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
// threads > 1: the frame's tiles on up to that many threads
int decode_frame(const FrameInputs &in, FrameWork &work, FrameResult &res, std::string &err, int threads = 1);

// One frame decoded on a worker thread: copies of everything the decoder may replace while
// it runs (sequence header, frame header, the temporal unit bytes, the reference slots it
// reads). An inter frame's job first waits for the jobs of the frames its references come from
// (their entropy state, segment map and saved motion vectors), as rav1d's frame threads wait
// on their references' progress (thread_task.rs), then decodes its tiles.
struct FrameJob {
    SeqHdr seq;
    std::shared_ptr<const FrameHdr> hdr;
    std::shared_ptr<const Cdf> in_cdf;
    std::vector<std::shared_ptr<std::vector<uint8_t>>> bufs;
    FrameInputs in;
    RefSlot refs[7];          // inter: refs_[refidx[i]] as they were at submission
    int primary = -1;         // index into refs of primary_ref_frame (-1: none)
    bool seg_from_primary = false;
    std::shared_ptr<FrameWork> work;
    FrameResult res;
    std::string err;
    int rc = 0;
    std::thread th;
    // completion: set once by the job's thread; wait() may be called from any thread
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    void finish() {
        std::lock_guard<std::mutex> g(m);
        done = true;
        cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [this] { return done; });
    }
    ~FrameJob() {
        if (th.joinable()) th.join();
    }
};

}  // namespace av1
