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
#include "pool.h"

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
    void set_threads(int n);
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
    std::unique_ptr<WorkerPool> pool_;   // threads_ - 1 workers (threads_ > 1)
    std::deque<std::shared_ptr<FrameJob>> running_;
    int n_tiles_ = 0;
    int next_pic_ = 0;
    std::deque<DecEvent> out_;
};

// What a frame decoding on a worker makes available to the frames that reference it before it
// ends (rav1d's frame-thread progress, thread_task.rs / picture.rs progress): its saved-MV and
// segment-id buffers once allocated (published), its entropy state once the context-update tile
// is decoded, and the 4x4 rows of those buffers that are final. A failed frame wakes every
// waiter with failure.
struct FrameProgress {
    std::shared_ptr<const std::vector<TmvBlock>> mvs;      // (set before published)
    std::shared_ptr<const std::vector<uint8_t>> segmap;
    std::shared_ptr<const Cdf> cdf;                         // (set before cdf_ready)

    // (once: later calls are ignored)
    void publish(std::shared_ptr<const std::vector<TmvBlock>> m, std::shared_ptr<const std::vector<uint8_t>> sm);
    void publish_cdf(std::shared_ptr<const Cdf> c);
    // rows [0, n) final (n only grows); tiled decode: superblock row sby of one tile column
    void rows_done(int n);
    void set_tiling(int cols, int sb_shift, int sbh);
    void tile_row_done(int sby);
    void fail();
    // false: the frame failed
    bool wait_published();
    bool wait_cdf();
    bool wait_rows(int n);

private:
    std::mutex m_;
    std::condition_variable cv_;
    bool published_ = false, cdf_ready_ = false, failed_ = false;
    int rows_ = 0;
    int cols_ = 1, sb_shift_ = 0, front_ = 0;
    std::vector<int> row_cols_;
};

// Decode one frame's tiles (decode.rs decode_frame_init + decode_tile_sbrow over every tile)
// into `work`. Returns 0 or -errno. Fills the state later frames need.
struct FrameResult {
    std::shared_ptr<const Cdf> out_cdf;                     // refresh_context
    std::shared_ptr<const std::vector<uint8_t>> segmap;
    std::shared_ptr<const std::vector<TmvBlock>> mvs;
};
struct FrameInputs {
    const SeqHdr *seq;
    const FrameHdr *hdr;
    const Cdf *in_cdf;                                      // nullptr: defaults for base_q_idx
    const RefSlot *refs[7];                                 // slots of refidx[0..6] (inter)
    std::shared_ptr<const std::vector<uint8_t>> prev_segmap;
    struct Tile { const uint8_t *data; size_t size; };
    std::vector<Tile> tiles;                                // in tile order
    WorkerPool *pool = nullptr;                             // tile threads (nullptr: this thread)
    // frame threads: this frame's progress (signalled as it decodes) and the progress of the
    // references still decoding whose saved MVs (ref_prog[i]) or segment ids (prev_segmap_prog)
    // it reads (nullptr: complete)
    FrameProgress *progress = nullptr;
    FrameProgress *in_cdf_prog = nullptr;                   // in_cdf: this frame's cdf once ready
    FrameProgress *ref_prog[7] = {};
    FrameProgress *prev_segmap_prog = nullptr;
    // the saved-MV and segment-id buffers, allocated by the caller before the references are
    // resolved so that later frames can be given them early (frame_buffers; nullptr: allocated
    // by decode_frame)
    std::shared_ptr<std::vector<TmvBlock>> rp_buf;
    std::shared_ptr<std::vector<uint8_t>> segmap_buf;
};
// The saved-MV (inter frames) and segment-id buffers of a frame, zeroed
void frame_buffers(const FrameHdr &h, std::shared_ptr<std::vector<TmvBlock>> &rp,
                   std::shared_ptr<std::vector<uint8_t>> &segmap);
int decode_frame(const FrameInputs &in, FrameWork &work, FrameResult &res, std::string &err);

// One frame decoded on a worker thread: copies of everything the decoder may replace while
// it runs (sequence header, frame header, the temporal unit bytes, the reference slots it
// reads). A frame's job waits for the entropy state of its primary reference's job, then
// decodes its tiles, each superblock row once the references still decoding have finished
// the saved MVs and segment ids of that row, as rav1d's frame threads wait on their
// references' progress (thread_task.rs).
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
    FrameProgress prog;
    std::string err;
    int rc = 0;
    std::thread th;
    // completion, set by the job's thread: the result later frames read (rc, err, res:
    // finish_result), then the whole job (work with its intra queue: finish); the waits may be
    // called from any thread
    std::mutex m;
    std::condition_variable cv;
    bool res_done = false, done = false;
    void finish_result() {
        std::lock_guard<std::mutex> g(m);
        res_done = true;
        cv.notify_all();
    }
    void finish() {
        std::lock_guard<std::mutex> g(m);
        res_done = done = true;
        cv.notify_all();
    }
    void wait_result() {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [this] { return res_done; });
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
