// intra_plan.h — the intra queue of one frame (host C++, shared by the frame executor,
// frame_exec.cpp, and the front-end, which runs it in its frame jobs so that the executor's host
// pass does not: mi_av1dec.h MiDecFrame.q_*).
//
// The persistent intra kernel (ipred.hip) takes the frame's transform blocks in queue order:
// vertical strips, one per XCD, each strip's blocks by dependency level, decode order within a
// level; the dependency lists follow the queue positions. Only host code: no HIP types.
#pragma once
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/mi_av1dec.h"

namespace mi_plan {

inline bool inter_present(const MiDecFrame *f) {
    return f->n_mc || f->n_obmc_h || f->n_obmc_v || f->n_warp || f->n_scaled || f->n_combine_y || f->n_combine_uv;
}

// par(n, min_n, fn): fn(lo, hi, t) over [0, n) in contiguous ranges (possibly on several
// threads); returns the number of ranges
// ---- one frame's intra blocks over every XCD (mi_internal::intra_recon strips) ----
//
// The persistent reconstruction hands pixels from block to block through the reading XCD's L2
// (ipred.hip), so a line must never be read on an XCD while another XCD may still write it.
// The frame is cut into up to 8 vertical strips, strip q reconstructed on XCD q, with every
// boundary a 128-B line boundary in every plane (and a multiple of 64 luma px). A block that
// reads pixels of another strip (its left column, top-left and top-right edges at a strip
// boundary) gets, besides the owners of those pixels, every block writing the lines they lie
// in: when it first reads such a line on its XCD, the line is final. All those writers precede
// the block in decode order (the lines lie in superblocks decoded before it: the left
// neighbour superblock or the superblock row above; an intra block copy source lies a
// superblock row above or 256 px left of the current superblock, spec 7.11.2 / rav1d
// decode.rs); if one did not, the frame stays on one XCD. Returns the number of strips (1: no
// split); strip[i] per block, extra deps as CSR. With edge granules (frame_run) a block reads
// the picture only for intra block copy and CfL's luma: edges need no extra deps.
template <typename Par>
int intra_strips(const MiDecFrame *f, std::vector<int8_t> &strip, std::vector<int32_t> &xs,
                 std::vector<int32_t> &xd, bool granules, Par &&par) {
    const int n = f->n_intra;
    const int maxs = 8;
    if (n < 64) return 1;
    const int pxb = f->bpc == 8 ? 1 : 2;
    const int ssh = f->layout == 1 || f->layout == 2, ssv = f->layout == 1;
    const int nplanes = f->layout ? 3 : 1;
    const int unit = (128 / pxb) << (f->layout ? ssh : 0);   // luma px per line of the widest plane
    const int units = (f->w + unit - 1) / unit;
    const int ns = std::min(maxs, units);
    if (ns < 2) return 1;
    std::vector<int> sx(ns + 1);
    for (int q = 0; q <= ns; q++) sx[q] = (int)((int64_t)q * units / ns) * unit;
    // the strip of every `unit`-wide column group (a table instead of a binary search per block)
    std::vector<int8_t> strip_of(units + 1);
    for (int u = 0, q = 0; u <= units; u++) {
        while (q + 1 < ns && sx[q + 1] <= u * unit) q++;
        strip_of[u] = (int8_t)q;
    }
    auto strip_at = [&](int xl) { return strip_of[std::min(xl / unit, units)]; };
    // strip of every block (by its luma column) and the owner of every 4x4 unit of each plane
    strip.resize(n);
    // with edge granules only intra block copy reads pixels across strips (CfL's luma lies in
    // its own strip): without such blocks there are no extra deps and no owner map is needed
    bool need_own = !granules;
    for (int i = 0; !need_own && i < n; i++) need_own = f->intra[i].mode == MI_INTRA_IBC;
    if (!need_own) {
        for (int i = 0; i < n; i++) {
            const MiIntraBlock &b = f->intra[i];
            const int xl = b.plane ? b.x << ssh : b.x;
            strip[i] = strip_at(xl);
        }
        xs.assign(n + 1, 0);
        xd.clear();
        return ns;
    }
    using sclk = std::chrono::steady_clock;
    const auto s0 = sclk::now();
    const int aw = (f->w + 127) & ~127, ah = (f->h + 127) & ~127;
    int pw4[3], ph4[3];
    // (per-thread scratch kept across frames: a fresh multi-MB map per frame costs its page
    // faults; bound by reference here, since the pool threads below must see this thread's)
    static thread_local std::vector<int32_t> own_tl[3];
    std::vector<int32_t> (&own)[3] = own_tl;
    for (int p = 0; p < nplanes; p++) {
        pw4[p] = (p ? aw >> ssh : aw) >> 2;
        ph4[p] = (p ? ah >> ssv : ah) >> 2;
        own[p].assign((size_t)pw4[p] * ph4[p], -1);
    }
    // The owner of a cell is its LAST writer in decode order: an inter-intra item and the
    // residual items over the same rectangle (MI_INTRA_II then MI_INTRA_RESID) overlap, and the
    // residual must win. One range walks the blocks in decode order, so a plain store leaves the
    // last writer; with several ranges on several threads a cell keeps the maximum index (a
    // relaxed CAS loop; the pool's join orders it before the reads below). The CAS costs ~6 ms
    // on a 4K10 intra frame's 168 K blocks on one thread, the plain store 0.5.
    par(n, 32768, [&](int lo, int hi, int) {
        const bool whole = lo == 0 && hi == n;
        for (int i = lo; i < hi; i++) {
            const MiIntraBlock &b = f->intra[i];
            const int xl = b.plane ? b.x << ssh : b.x;
            strip[i] = strip_at(xl);
            for (int y = b.y >> 2; y < (b.y + b.h) >> 2; y++) {
                int32_t *row = &own[b.plane][(size_t)y * pw4[b.plane]];
                for (int x = b.x >> 2; x < (b.x + b.w) >> 2; x++) {
                    int32_t *cell = row + x;
                    if (whole) {
                        *cell = i;
                        continue;
                    }
                    int32_t cur = __atomic_load_n(cell, __ATOMIC_RELAXED);
                    while (cur < i && !__atomic_compare_exchange_n(cell, &cur, i, true, __ATOMIC_RELAXED,
                                                                   __ATOMIC_RELAXED)) {
                    }
                }
            }
        }
    });
    const auto s1 = sclk::now();
    xs.assign(n + 1, 0);
    xd.clear();
    const int lpx = 128 / pxb;                                // plane px per line
    // the blocks writing a line that block i reads across a strip boundary (false: a later
    // writer, so the frame stays on one XCD)
    auto scan_block = [&](int i, std::vector<int32_t> &add) -> bool {
        const MiIntraBlock &b = f->intra[i];
        const int p = b.plane;
        add.clear();
        {
            // most blocks read only their own strip: nothing to scan
            bool cross = false;
            for (int d = f->dep_start[i]; d < f->dep_start[i + 1] && !cross; d++) cross = strip[f->deps[d]] != strip[i];
            if (!cross) return true;
        }
        // the pixels this block may read: its edges (rows y-1 .. y+2h-1, columns x-1 .. x+2w-1),
        // or for intra block copy the source rectangle (+1 for the bilinear phase, +-1 margin)
        int bx0 = std::max(0, (int)b.x - 1), by0 = std::max(0, (int)b.y - 1);
        int bx1 = b.x + 2 * b.w, by1 = b.y + 2 * b.h;
        if (b.mode == MI_INTRA_IBC) {
            const int mvx = (int16_t)(b.reserved & 0xffff), mvy = (int16_t)(b.reserved >> 16);
            const int sh = b.filt_idx & 1, sv = (b.filt_idx >> 1) & 1;
            const int sx = b.x + (mvx >> (3 + sh)), sy = b.y + (mvy >> (3 + sv));
            bx0 = std::max(0, sx - 1);
            by0 = std::max(0, sy - 1);
            bx1 = sx + b.w + 2;
            by1 = sy + b.h + 2;
        }
        for (int d = f->dep_start[i]; d < f->dep_start[i + 1]; d++) {
            const int j = f->deps[d];
            if (strip[j] == strip[i]) continue;
            const MiIntraBlock &o = f->intra[j];
            if (granules && o.plane == p && b.mode != MI_INTRA_IBC) continue;   // an edge: granules
            if (o.plane != p) return false;                   // (CfL luma: same strip by construction)
            const int x0 = std::max(bx0, (int)o.x), x1 = std::min(bx1, o.x + o.w);
            const int y0 = std::max(by0, (int)o.y), y1 = std::min(by1, o.y + o.h);
            if (x0 >= x1 || y0 >= y1) continue;
            const int l0 = x0 / lpx, l1 = (x1 - 1) / lpx;     // lines of those rows
            for (int y = y0 >> 2; y <= (y1 - 1) >> 2; y++)
                for (int u = (l0 * lpx) >> 2; u < std::min(pw4[p], ((l1 + 1) * lpx) >> 2); u++) {
                    const int w = own[p][(size_t)y * pw4[p] + u];
                    if (w < 0 || w == j) continue;
                    if (w >= i) return false;                 // a later writer: no split
                    add.push_back(w);
                }
        }
        std::sort(add.begin(), add.end());
        add.erase(std::unique(add.begin(), add.end()), add.end());
        return true;
    };
    // the extra dependencies per block range (each range its own CSR part), then concatenated
    std::vector<int32_t> part_xd[8];
    int part_lo[9] = {};
    int split_ok = 1;
    const int nparts = par(n, 32768, [&](int lo, int hi, int t) {
        part_lo[t] = lo;
        std::vector<int32_t> &pxd = part_xd[t];
        // a range re-run on the caller's thread after its worker threw (PlanPool::run) must
        // not keep the failed attempt's entries
        pxd.clear();
        std::vector<int32_t> add;
        for (int i = lo; i < hi; i++) {
            xs[i] = (int32_t)pxd.size();
            if (!__atomic_load_n(&split_ok, __ATOMIC_RELAXED) || !scan_block(i, add)) {
                __atomic_store_n(&split_ok, 0, __ATOMIC_RELAXED);
                return;
            }
            pxd.insert(pxd.end(), add.begin(), add.end());
        }
    });
    static const bool sprof = getenv("MI_FX_PROFILE") != nullptr;
    if (sprof) {
        auto ms = [](sclk::time_point a, sclk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "intra_strips owner map %.3f scan %.3f ms\n", ms(s0, s1), ms(s1, sclk::now()));
    }
    if (!split_ok) return 1;
    for (int t = 0; t < nparts; t++) {
        const int lo = part_lo[t], hi = t + 1 < nparts ? part_lo[t + 1] : n;
        const int32_t base = (int32_t)xd.size();
        for (int i = lo; i < hi; i++) xs[i] += base;
        xd.insert(xd.end(), part_xd[t].begin(), part_xd[t].end());
    }
    xs[n] = (int32_t)xd.size();
    return ns;
}


struct IntraQueue {
    std::vector<MiIntraBlock> blocks;
    std::vector<MiTxBlock> tx;
    std::vector<int32_t> dep_start, deps, strip_start;
    bool inter = false, granules = false;
    // MI_IR_TIMELINE diagnostics (filled only when `timeline` is set): every dependency (with the
    // strips' extra ones) in queue order
    bool timeline = false;
    std::vector<int32_t> tl_ds, tl_deps, tl_strip;
    double ms = 0;
};

template <typename Par>
void plan_intra(const MiDecFrame *f, IntraQueue &q, Par &&par) {
    const int n = f->n_intra;
    std::vector<MiIntraBlock> &blocks = q.blocks;
    std::vector<MiTxBlock> &tx = q.tx;
    std::vector<int32_t> &dep_start = q.dep_start, &deps = q.deps, &strip_start = q.strip_start;
    std::vector<int32_t> &tl_ds = q.tl_ds, &tl_deps = q.tl_deps, &tl_strip = q.tl_strip;
    blocks.resize(n);
    tx.resize(n);
    dep_start.assign(n + 1, 0);
    deps.clear();
    strip_start.clear();
    tl_ds.clear();
    tl_deps.clear();
    tl_strip.clear();
    // dependency levels (deps always point backwards): level order lets the persistent
    // kernel's workers run every block of a level side by side. A single frame is split into
    // vertical strips, one per XCD (intra_strips), each strip's blocks in level order.
    using clk = std::chrono::steady_clock;
    const auto t_lv = clk::now();
    // edge granules (ipred.hip gran_fetch) when every pixel an intra edge reads is written in the
    // same launch: no inter units, no inter-intra blends or inter residuals. A block then waits
    // on flags only for the pixels it reads beyond its edges (CfL's luma, intra block copy's
    // source); the levels still follow every dependency.
    const bool inter = q.inter = inter_present(f) || f->n_inter_tx;
    bool &granules = q.granules;
    granules = !inter && n > 0;
    for (int i = 0; granules && i < n; i++)
        if ((f->intra[i].flags & MI_INTRA_II) || f->intra[i].mode == MI_INTRA_RESID) granules = false;
    if (n) {
        // per-thread scratch kept across frames (no per-frame page faults)
        // (the scratch is bound by reference: the pool threads must see this thread's vectors)
        static thread_local std::vector<int32_t> xs_tl, xd_tl;   // extra dependencies of the strip split (CSR)
        static thread_local std::vector<int8_t> strip_tl;
        std::vector<int32_t> &xs = xs_tl, &xd = xd_tl;
        std::vector<int8_t> &strip = strip_tl;
        const int nstrips = intra_strips(f, strip, xs, xd, granules, par);
        const auto t_a = clk::now();
        auto each_dep = [&](int i, auto &&fn) {
            for (int d = f->dep_start[i]; d < f->dep_start[i + 1]; d++) fn(f->deps[d]);
            if (nstrips > 1)
                for (int d = xs[i]; d < xs[i + 1]; d++) fn(xd[d]);
        };
        static thread_local std::vector<int32_t> level_tl, pos_tl;
        std::vector<int32_t> &level = level_tl, &pos = pos_tl;
        level.assign(n, 0);
        pos.resize(n);
        int maxl = 0;
        // MI_IR_NOLEVELS=1 (experiment): decode order within a strip, no level pass
        for (int i = 0; i < n; i++) {
            int l = 0;
            each_dep(i, [&](int d) { l = std::max(l, level[d] + 1); });
            level[i] = l;
            maxl = std::max(maxl, l);
        }
        const auto t_b = clk::now();
        // counting sort by (strip, level), decode order within
        const int nkeys = nstrips * (maxl + 1);
        auto key = [&](int i) { return (nstrips > 1 ? strip[i] * (maxl + 1) : 0) + level[i]; };
        std::vector<int32_t> cnt(nkeys + 1, 0);
        for (int i = 0; i < n; i++) cnt[key(i) + 1]++;
        for (int k = 0; k < nkeys; k++) cnt[k + 1] += cnt[k];
        if (nstrips > 1) {
            strip_start.resize(nstrips + 1);
            for (int q = 0; q <= nstrips; q++) strip_start[q] = cnt[q * (maxl + 1)];
        }
        for (int i = 0; i < n; i++) pos[i] = cnt[key(i)]++;
        static thread_local std::vector<int32_t> inv_tl;
        std::vector<int32_t> &inv = inv_tl;
        inv.resize(n);
        for (int i = 0; i < n; i++) inv[pos[i]] = i;
        const auto t_c = clk::now();
        // the queue-ordered copies, walking the units in decode order (their deps point to
        // recent units: the reads stay in cache) and scattering the writes: count each unit's
        // kernel deps, prefix sum in queue order, then fill
        auto kdeps = [&](int i, auto &&fn) {
            const MiIntraBlock &b = f->intra[i];
            if (!granules || b.mode == MI_INTRA_IBC || b.mode == MI_IPRED_CFL) {
                each_dep(i, [&](int d) { fn(pos[d]); });
            } else {
                for (int d = f->dep_start[i]; d < f->dep_start[i + 1]; d++)
                    if (f->intra[f->deps[d]].plane != b.plane) fn(pos[f->deps[d]]);
            }
        };
        // (ranges of decode order on several threads: every unit has its own queue slot)
        dep_start[0] = 0;
        par(n, 32768, [&](int lo, int hi, int) {
            for (int i = lo; i < hi; i++) {
                const int k = pos[i];
                blocks[k] = f->intra[i];
                tx[k] = f->intra_tx[i];
                int c = 0;
                kdeps(i, [&](int) { c++; });
                dep_start[k + 1] = c;
            }
        });
        for (int k = 0; k < n; k++) dep_start[k + 1] += dep_start[k];
        deps.resize(dep_start[n]);
        par(n, 32768, [&](int lo, int hi, int) {
            for (int i = lo; i < hi; i++) {
                int o = dep_start[pos[i]];
                kdeps(i, [&](int d) { deps[o++] = d; });
            }
        });
        static const bool prof = getenv("MI_FX_PROFILE") != nullptr;
        if (prof) {
            auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            fprintf(stderr, "frame_run n=%d strips %.3f levels %.3f sort %.3f permute %.3f ms\n", n, ms(t_lv, t_a),
                    ms(t_a, t_b), ms(t_b, t_c), ms(t_c, clk::now()));
        }
        if (q.timeline) {
            // every dependency (with the strips' extra ones), in queue order
            tl_ds.assign(n + 1, 0);
            for (int k = 0; k < n; k++) {
                tl_ds[k] = (int32_t)tl_deps.size();
                each_dep(inv[k], [&](int d) { tl_deps.push_back(pos[d]); });
            }
            tl_ds[n] = (int32_t)tl_deps.size();
            tl_strip.assign(strip_start.begin(), strip_start.end());
        }
    }
    if (deps.empty()) deps.push_back(0);
    q.ms = std::chrono::duration<double, std::milli>(clk::now() - t_lv).count();
}

}  // namespace mi_plan
