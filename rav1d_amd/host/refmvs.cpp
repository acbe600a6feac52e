// refmvs.cpp — motion-vector prediction of the front-end: the spatial / temporal candidate list
// of one block (rav1d_refmvs_find, refmvs.rs:830; C refmvs.c:348-651), the temporal MVs of the
// reference frames projected onto the current frame (load_tmvs, refmvs.rs:1319; C
// refmvs.c:690-761) and this frame's MVs saved for later frames (save_tmvs, refmvs.rs:1521; C
// refmvs.c:763-797), plus the per-frame setup (rav1d_refmvs_init_frame; C refmvs.c:799-895).
//
// The reference keeps a 35-row window of 4x4 entries per tile row and a 16-row ring of projected
// 8x8 entries; here both are whole-frame arrays (FrameDec::rmv, rp_proj), which holds the same
// values at every position a block reads (rows above the current superblock row, the current
// row's decoded blocks, and the current sbrow's projections).
#include <climits>
#include <cstdlib>

#include "framedec.h"

namespace av1 {
namespace fd {

static const Mv kInvalid = { INT16_MIN, INT16_MIN };

static int poc_diff(int nbits, int poc0, int poc1) {
    if (!nbits) return 0;
    const int mask = 1 << (nbits - 1);
    const int diff = poc0 - poc1;
    return (diff & (mask - 1)) - (diff & mask);
}

static inline int apply_sign(int v, int s) { return s < 0 ? -v : v; }

// fix_mv_precision (env.rs; C env.h:463-477)
void FrameDec::fix_mv(Mv &mv) const {
    if (h.force_integer_mv) {
        mv.x = (int16_t)((mv.x - (mv.x >> 15) + 3) & ~7u);
        mv.y = (int16_t)((mv.y - (mv.y >> 15) + 3) & ~7u);
    } else if (!h.hp) {
        mv.x = (int16_t)((mv.x - (mv.x >> 15)) & ~1u);
        mv.y = (int16_t)((mv.y - (mv.y >> 15)) & ~1u);
    }
}

// get_gmv_2d (env.rs; C env.h:479-519) for the current block position
Mv FrameDec::gmv_2d(int ref, int bw4, int bh4) const {
    const WarpParams &g = h.gmv[ref];
    Mv res{ 0, 0 };
    if (g.type == WM_IDENTITY) return res;
    if (g.type == WM_TRANSLATION) {
        res.y = (int16_t)(g.matrix[0] >> 13);
        res.x = (int16_t)(g.matrix[1] >> 13);
    } else {
        const int x = bx * 4 + bw4 * 2 - 1, y = by * 4 + bh4 * 2 - 1;
        const int xc = (g.matrix[2] - (1 << 16)) * x + g.matrix[3] * y + g.matrix[0];
        const int yc = (g.matrix[5] - (1 << 16)) * y + g.matrix[4] * x + g.matrix[1];
        const int shift = 16 - (3 - !h.hp), round = (1 << shift) >> 1;
        res.y = (int16_t)apply_sign(((std::abs(yc) + round) >> shift) << !h.hp, yc);
        res.x = (int16_t)apply_sign(((std::abs(xc) + round) >> shift) << !h.hp, xc);
    }
    if (h.force_integer_mv) {
        res.x = (int16_t)((res.x - (res.x >> 15) + 3) & ~7u);
        res.y = (int16_t)((res.y - (res.y >> 15) + 3) & ~7u);
    }
    return res;
}

void FrameDec::refmvs_init_frame() {
    iw8 = (h.width[0] + 7) >> 3;
    ih8 = (h.height + 7) >> 3;
    iw4 = iw8 << 1;
    ih4 = ih8 << 1;
    rp_stride = b4_stride >> 1;
    const int nbits = s.order_hint_n_bits;
    const int poc = h.frame_offset;
    int ref_poc[7];
    for (int i = 0; i < 7; i++) {
        ref_poc[i] = in_.refs[i]->hdr->frame_offset;
        const int d = poc_diff(nbits, ref_poc[i], poc);
        sign_bias[i] = d > 0;
        mfmv_sign[i] = d < 0;
        pocdiff[i] = (int8_t)iclip(poc_diff(nbits, poc, ref_poc[i]), -31, 31);
        const RefSlot *r = in_.refs[i];
        rp_ref[i] = (h.use_ref_frame_mvs && r->mvs && r->bw == bw && r->bh == bh) ? r->mvs->data() : nullptr;
    }
    n_mfmvs = 0;
    if (h.use_ref_frame_mvs && nbits) {
        int total = 2;
        if (rp_ref[0] && in_.refs[0]->refpoc[6] != ref_poc[3]) {   // alt-of-last != gold
            mfmv_ref[n_mfmvs++] = 0;
            total = 3;
        }
        if (rp_ref[4] && poc_diff(nbits, ref_poc[4], poc) > 0) mfmv_ref[n_mfmvs++] = 4;
        if (rp_ref[5] && poc_diff(nbits, ref_poc[5], poc) > 0) mfmv_ref[n_mfmvs++] = 5;
        if (n_mfmvs < total && rp_ref[6] && poc_diff(nbits, ref_poc[6], poc) > 0) mfmv_ref[n_mfmvs++] = 6;
        if (n_mfmvs < total && rp_ref[1]) mfmv_ref[n_mfmvs++] = 1;
        for (int n = 0; n < n_mfmvs; n++) {
            const int rpoc = ref_poc[mfmv_ref[n]];
            const int diff1 = poc_diff(nbits, rpoc, poc);
            if (std::abs(diff1) > 31) {
                mfmv_ref2cur[n] = INT_MIN;
            } else {
                mfmv_ref2cur[n] = mfmv_ref[n] < 4 ? -diff1 : diff1;
                for (int m = 0; m < 7; m++) {
                    const int diff2 = poc_diff(nbits, rpoc, in_.refs[mfmv_ref[n]]->refpoc[m]);
                    mfmv_ref2ref[n][m] = (unsigned)diff2 > 31u ? 0 : diff2;
                }
            }
        }
    }
    TmvBlock inv{};
    inv.mv = kInvalid;
    if (master_) {
        S->rp_proj.assign((size_t)rp_stride * (sb128h * 16 + 16), inv);
        const size_t n = (size_t)rp_stride * sb128h * 16;
        if (in_.rp_buf && in_.rp_buf->size() == n) S->rp = in_.rp_buf;
        else S->rp = std::make_shared<std::vector<TmvBlock>>(n, TmvBlock{});
    }
    rp_proj.bind(S->rp_proj);
    rp = S->rp;
}

// mv_projection (refmvs.rs; C refmvs.c:175-191)
static Mv mv_projection(Mv mv, int num, int den) {
    static const uint16_t div_mult[32] = {
        0,    16384, 8192, 5461, 4096, 3276, 2730, 2340, 2048, 1820, 1638, 1489, 1365, 1260, 1170, 1092,
        1024, 963,   910,  862,  819,  780,  744,  712,  682,  655,  630,  606,  585,  564,  546,  528,
    };
    const int frac = num * div_mult[den];
    const int y = mv.y * frac, x = mv.x * frac;
    Mv r;
    r.y = (int16_t)iclip((y + 8192 + (y >> 31)) >> 14, -0x3fff, 0x3fff);
    r.x = (int16_t)iclip((x + 8192 + (x >> 31)) >> 14, -0x3fff, 0x3fff);
    return r;
}

// over the 8x8 columns [col_start8, col_end8): the frame (decode_frame_main) or one tile (rav1d's
// tile threads pass the tile's columns, thread_task.rs)
void FrameDec::load_tmvs(int row_start8, int row_end8, int col_start8, int col_end8) {
    row_end8 = imin(row_end8, ih8);
    col_end8 = imin(col_end8, iw8);
    const int col_start8i = imax(col_start8 - 8, 0), col_end8i = imin(col_end8 + 8, iw8);
    const ptrdiff_t stride = rp_stride;
    for (int y = row_start8; y < row_end8; y++)
        for (int x = col_start8; x < col_end8; x++) rp_proj[(size_t)y * stride + x].mv = kInvalid;
    for (int n = 0; n < n_mfmvs; n++) {
        const int ref2cur = mfmv_ref2cur[n];
        if (ref2cur == INT_MIN) continue;
        const int ref = mfmv_ref[n], ref_sign = ref - 4;
        const TmvBlock *r = rp_ref[ref] + (size_t)row_start8 * stride;
        for (int y = row_start8; y < row_end8; y++) {
            const int y_sb_align = y & ~7;
            const int y_proj_start = imax(y_sb_align, row_start8), y_proj_end = imin(y_sb_align + 8, row_end8);
            for (int x = col_start8i; x < col_end8i; x++) {
                const TmvBlock *rb = &r[x];
                const int b_ref = rb->ref;
                if (!b_ref) continue;
                const int ref2ref = mfmv_ref2ref[n][b_ref - 1];
                if (!ref2ref) continue;
                const Mv b_mv = rb->mv;
                const Mv off = mv_projection(b_mv, ref2cur, ref2ref);
                int pos_x = x + apply_sign(std::abs(off.x) >> 6, off.x ^ ref_sign);
                const int pos_y = y + apply_sign(std::abs(off.y) >> 6, off.y ^ ref_sign);
                if (pos_y >= y_proj_start && pos_y < y_proj_end) {
                    const size_t pos = (size_t)pos_y * stride;
                    for (;;) {
                        const int x_sb_align = x & ~7;
                        if (pos_x >= imax(x_sb_align - 8, col_start8) && pos_x < imin(x_sb_align + 16, col_end8)) {
                            rp_proj[pos + pos_x].mv = rb->mv;
                            rp_proj[pos + pos_x].ref = (int8_t)ref2ref;
                        }
                        if (++x >= col_end8i) break;
                        rb++;
                        if (rb->ref != b_ref || !(rb->mv == b_mv)) break;
                        pos_x++;
                    }
                } else {
                    for (;;) {
                        if (++x >= col_end8i) break;
                        rb++;
                        if (rb->ref != b_ref || !(rb->mv == b_mv)) break;
                    }
                }
                x--;
            }
            r += stride;
        }
    }
}

void FrameDec::save_tmvs(int row_start8, int row_end8, int col_start8, int col_end8) {
    row_end8 = imin(row_end8, ih8);
    col_end8 = imin(col_end8, iw8);
    for (int y = row_start8; y < row_end8; y++) {
        TmvBlock *out = rp->data() + (size_t)y * rp_stride;
        for (int x = col_start8; x < col_end8;) {
            const RefMvBlock &c = rmv_at(2 * y + 1, 2 * x + 1);
            const int bw8 = (k_bdim[c.bs].w4 + 1) >> 1;
            TmvBlock t{};
            if (c.ref[1] > 0 && mfmv_sign[c.ref[1] - 1] && (std::abs(c.mv[1].y) | std::abs(c.mv[1].x)) < 4096) {
                t.mv = c.mv[1];
                t.ref = c.ref[1];
            } else if (c.ref[0] > 0 && mfmv_sign[c.ref[0] - 1] && (std::abs(c.mv[0].y) | std::abs(c.mv[0].x)) < 4096) {
                t.mv = c.mv[0];
                t.ref = c.ref[0];
            }
            for (int n = 0; n < bw8; n++, x++) out[x] = t;
        }
    }
}

namespace {

struct Finder {
    MvCand *st;
    int *cnt;
    int ref0, ref1;
    Mv gmv[2];
    void add(const RefMvBlock &b, int weight, int *have_newmv, int *have_refmv) {
        if (b.mv[0] == kInvalid) return;   // intra block, no block copy
        if (ref1 == -1) {
            for (int n = 0; n < 2; n++) {
                if (b.ref[n] != ref0) continue;
                const Mv c = ((b.mf & 1) && !(gmv[0] == kInvalid)) ? gmv[0] : b.mv[n];
                *have_refmv = 1;
                *have_newmv |= b.mf >> 1;
                const int last = *cnt;
                for (int m = 0; m < last; m++)
                    if (st[m].mv[0] == c) {
                        st[m].weight += weight;
                        return;
                    }
                if (last < 8) {
                    st[last].mv[0] = c;
                    st[last].weight = weight;
                    *cnt = last + 1;
                }
                return;
            }
        } else if (b.ref[0] == ref0 && b.ref[1] == ref1) {
            Mv c[2];
            c[0] = ((b.mf & 1) && !(gmv[0] == kInvalid)) ? gmv[0] : b.mv[0];
            c[1] = ((b.mf & 1) && !(gmv[1] == kInvalid)) ? gmv[1] : b.mv[1];
            *have_refmv = 1;
            *have_newmv |= b.mf >> 1;
            const int last = *cnt;
            for (int n = 0; n < last; n++)
                if (st[n].mv[0] == c[0] && st[n].mv[1] == c[1]) {
                    st[n].weight += weight;
                    return;
                }
            if (last < 8) {
                st[last].mv[0] = c[0];
                st[last].mv[1] = c[1];
                st[last].weight = weight;
                *cnt = last + 1;
            }
        }
    }
};

}  // namespace

void FrameDec::refmvs_find(MvCand stack[8], int *cnt, int *ctx, int ref0, int ref1, int bs, int edge_flags) {
    const int bw4 = k_bdim[bs].w4, bh4 = k_bdim[bs].h4;
    const int col_end = imin(ts->col_end, iw4), row_end = imin(ts->row_end, ih4);
    const int w4b = imin(imin(bw4, 16), col_end - bx), h4b = imin(imin(bh4, 16), row_end - by);
    for (int i = 0; i < 8; i++) stack[i] = MvCand{ { { 0, 0 }, { 0, 0 } }, 0 };
    Finder F{ stack, cnt, ref0, ref1, { kInvalid, kInvalid } };
    Mv tgmv[2] = { { 0, 0 }, { 0, 0 } };
    *cnt = 0;
    if (ref0 > 0) {
        tgmv[0] = gmv_2d(ref0 - 1, bw4, bh4);
        F.gmv[0] = h.gmv[ref0 - 1].type > WM_TRANSLATION ? tgmv[0] : kInvalid;
    }
    if (ref1 > 0) {
        tgmv[1] = gmv_2d(ref1 - 1, bw4, bh4);
        F.gmv[1] = h.gmv[ref1 - 1].type > WM_TRANSLATION ? tgmv[1] : kInvalid;
    }

    // scan_row / scan_col (C refmvs.c:97-173)
    auto scan_row = [&](int y4, int x4, int max_rows, int step, int *have_newmv, int *have) -> int {
        const RefMvBlock *b0 = &rmv_at(y4, x4);
        const int cbw4 = k_bdim[b0->bs].w4;
        int len = imax(step, imin(bw4, cbw4));
        if (bw4 <= cbw4) {
            const int weight = bw4 == 1 ? 2 : imax(2, imin(2 * max_rows, (int)k_bdim[b0->bs].h4));
            F.add(*b0, len * weight, have_newmv, have);
            return weight >> 1;
        }
        for (int x = 0;;) {
            F.add(b0[x], len * 2, have_newmv, have);
            x += len;
            if (x >= w4b) return 1;
            len = imax(step, (int)k_bdim[b0[x].bs].w4);
        }
    };
    auto scan_col = [&](int y4, int x4, int max_cols, int step, int *have_newmv, int *have) -> int {
        const RefMvBlock *b0 = &rmv_at(y4, x4);
        const int cbh4 = k_bdim[b0->bs].h4;
        int len = imax(step, imin(bh4, cbh4));
        if (bh4 <= cbh4) {
            const int weight = bh4 == 1 ? 2 : imax(2, imin(2 * max_cols, (int)k_bdim[b0->bs].w4));
            F.add(*b0, len * weight, have_newmv, have);
            return weight >> 1;
        }
        for (int y = 0;;) {
            F.add(rmv_at(y4 + y, x4), len * 2, have_newmv, have);
            y += len;
            if (y >= h4b) return 1;
            len = imax(step, (int)k_bdim[rmv_at(y4 + y, x4).bs].h4);
        }
    };

    int have_newmv = 0, have_col_mvs = 0, have_row_mvs = 0, dummy = 0;
    unsigned max_rows = 0, n_rows = ~0u, max_cols = 0, n_cols = ~0u;
    if (by > ts->row_start) {
        max_rows = imin((by - ts->row_start + 1) >> 1, 2 + (bh4 > 1));
        n_rows = scan_row(by - 1, bx, max_rows, bw4 >= 16 ? 4 : 1, &have_newmv, &have_row_mvs);
    }
    if (bx > ts->col_start) {
        max_cols = imin((bx - ts->col_start + 1) >> 1, 2 + (bw4 > 1));
        n_cols = scan_col(by, bx - 1, max_cols, bh4 >= 16 ? 4 : 1, &have_newmv, &have_col_mvs);
    }
    // top / right
    if (n_rows != ~0u && (edge_flags & E444_TR) && imax(bw4, bh4) <= 16 && bw4 + bx < col_end)
        F.add(rmv_at(by - 1, bx + bw4), 4, &have_newmv, &have_row_mvs);
    const int nearest_match = have_col_mvs + have_row_mvs;
    const int nearest_cnt = *cnt;
    for (int n = 0; n < nearest_cnt; n++) stack[n].weight += 640;

    // temporal (C refmvs.c:416-452)
    int globalmv_ctx = h.use_ref_frame_mvs;
    if (n_mfmvs > 0) {
        const ptrdiff_t stride = rp_stride;
        const int by8 = by >> 1, bx8 = bx >> 1;
        const TmvBlock *rbi = &rp_proj[(size_t)by8 * stride + bx8];
        auto add_t = [&](const TmvBlock &rb, int *gctx) {
            if (rb.mv == kInvalid) return;
            Mv mv = mv_projection(rb.mv, pocdiff[ref0 - 1], rb.ref);
            fix_mv(mv);
            const int last = *cnt;
            if (ref1 == -1) {
                if (gctx) *gctx = (std::abs(mv.x - tgmv[0].x) | std::abs(mv.y - tgmv[0].y)) >= 16;
                for (int n = 0; n < last; n++)
                    if (stack[n].mv[0] == mv) {
                        stack[n].weight += 2;
                        return;
                    }
                if (last < 8) {
                    stack[last].mv[0] = mv;
                    stack[last].weight = 2;
                    *cnt = last + 1;
                }
            } else {
                Mv mv1 = mv_projection(rb.mv, pocdiff[ref1 - 1], rb.ref);
                fix_mv(mv1);
                for (int n = 0; n < last; n++)
                    if (stack[n].mv[0] == mv && stack[n].mv[1] == mv1) {
                        stack[n].weight += 2;
                        return;
                    }
                if (last < 8) {
                    stack[last].mv[0] = mv;
                    stack[last].mv[1] = mv1;
                    stack[last].weight = 2;
                    *cnt = last + 1;
                }
            }
        };
        const int step_h = bw4 >= 16 ? 2 : 1, step_v = bh4 >= 16 ? 2 : 1;
        const int w8 = imin((w4b + 1) >> 1, 8), h8 = imin((h4b + 1) >> 1, 8);
        const TmvBlock *rb = rbi;
        for (int y = 0; y < h8; y += step_v) {
            for (int x = 0; x < w8; x += step_h) add_t(rb[x], !(x | y) ? &globalmv_ctx : nullptr);
            rb += stride * step_v;
        }
        if (imin(bw4, bh4) >= 2 && imax(bw4, bh4) < 16) {
            const int bh8 = bh4 >> 1, bw8 = bw4 >> 1;
            rb = &rbi[bh8 * stride];
            const int has_bottom = by8 + bh8 < imin(row_end >> 1, (by8 & ~7) + 8);
            if (has_bottom && bx8 - 1 >= imax(ts->col_start >> 1, bx8 & ~7)) add_t(rb[-1], nullptr);
            if (bx8 + bw8 < imin(col_end >> 1, (bx8 & ~7) + 8)) {
                if (has_bottom) add_t(rb[bw8], nullptr);
                if (by8 + bh8 - 1 < imin(row_end >> 1, (by8 & ~7) + 8)) add_t(rb[bw8 - stride], nullptr);
            }
        }
    }

    // top / left, then the secondary rows and columns (8x8 resolution)
    if ((n_rows | n_cols) != ~0u) F.add(rmv_at(by - 1, bx - 1), 4, &dummy, &have_row_mvs);
    for (int n = 2; n <= 3; n++) {
        if ((unsigned)n > n_rows && (unsigned)n <= max_rows)
            n_rows += scan_row(((by - 2 * n + 1) | 1), bx | 1, 1 + max_rows - n, bw4 >= 16 ? 4 : 2, &dummy,
                               &have_row_mvs);
        if ((unsigned)n > n_cols && (unsigned)n <= max_cols)
            n_cols += scan_col(by | 1, (bx - n * 2 + 1) | 1, 1 + max_cols - n, bh4 >= 16 ? 4 : 2, &dummy,
                               &have_col_mvs);
    }
    const int ref_match_count = have_col_mvs + have_row_mvs;

    int refmv_ctx = 0, newmv_ctx = 0;
    switch (nearest_match) {
    case 0:
        refmv_ctx = imin(2, ref_match_count);
        newmv_ctx = ref_match_count > 0;
        break;
    case 1:
        refmv_ctx = imin(ref_match_count * 3, 4);
        newmv_ctx = 3 - have_newmv;
        break;
    case 2:
        refmv_ctx = 5;
        newmv_ctx = 5 - have_newmv;
        break;
    }

    // sorting: the nearest candidates, then the rest (bubble sorts, stable for equal weights)
    for (int len = nearest_cnt; len;) {
        int last = 0;
        for (int n = 1; n < len; n++)
            if (stack[n - 1].weight < stack[n].weight) {
                std::swap(stack[n - 1], stack[n]);
                last = n;
            }
        len = last;
    }
    for (int len = *cnt; len > nearest_cnt;) {
        int last = nearest_cnt;
        for (int n = nearest_cnt + 1; n < len; n++)
            if (stack[n - 1].weight < stack[n].weight) {
                std::swap(stack[n - 1], stack[n]);
                last = n;
            }
        len = last;
    }

    const int left = -(bx + bw4 + 4) * 4 * 8, right = (iw4 - bx + 4) * 4 * 8;
    const int top = -(by + bh4 + 4) * 4 * 8, bottom = (ih4 - by + 4) * 4 * 8;
    if (ref1 > 0) {
        if (*cnt < 2) {
            // extended candidates from non-matching neighbours (C refmvs.c:239-294, 526-582)
            const int sign0 = sign_bias[ref0 - 1], sign1 = sign_bias[ref1 - 1];
            const int sz4 = imin(w4b, h4b);
            MvCand *same = &stack[*cnt];
            MvCand *diff = &same[2];
            int same_count[4] = { 0, 0, 0, 0 };
            int *diff_count = &same_count[2];
            auto add_ext = [&](const RefMvBlock &c) {
                for (int n = 0; n < 2; n++) {
                    const int cr = c.ref[n];
                    if (cr <= 0) break;
                    Mv cm = c.mv[n];
                    if (cr == ref0) {
                        if (same_count[0] < 2) same[same_count[0]++].mv[0] = cm;
                        if (diff_count[1] < 2) {
                            if (sign1 ^ sign_bias[cr - 1]) { cm.y = (int16_t)-cm.y; cm.x = (int16_t)-cm.x; }
                            diff[diff_count[1]++].mv[1] = cm;
                        }
                    } else if (cr == ref1) {
                        if (same_count[1] < 2) same[same_count[1]++].mv[1] = cm;
                        if (diff_count[0] < 2) {
                            if (sign0 ^ sign_bias[cr - 1]) { cm.y = (int16_t)-cm.y; cm.x = (int16_t)-cm.x; }
                            diff[diff_count[0]++].mv[0] = cm;
                        }
                    } else {
                        const Mv icm{ (int16_t)-cm.y, (int16_t)-cm.x };
                        if (diff_count[0] < 2) diff[diff_count[0]++].mv[0] = (sign0 ^ sign_bias[cr - 1]) ? icm : cm;
                        if (diff_count[1] < 2) diff[diff_count[1]++].mv[1] = (sign1 ^ sign_bias[cr - 1]) ? icm : cm;
                    }
                }
            };
            if (n_rows != ~0u)
                for (int x = 0; x < sz4;) {
                    const RefMvBlock &c = rmv_at(by - 1, bx + x);
                    add_ext(c);
                    x += k_bdim[c.bs].w4;
                }
            if (n_cols != ~0u)
                for (int y = 0; y < sz4;) {
                    const RefMvBlock &c = rmv_at(by + y, bx - 1);
                    add_ext(c);
                    y += k_bdim[c.bs].h4;
                }
            for (int n = 0; n < 2; n++) {
                int m = same_count[n];
                if (m >= 2) continue;
                const int lc = diff_count[n];
                if (lc) {
                    same[m].mv[n] = diff[0].mv[n];
                    if (++m == 2) continue;
                    if (lc == 2) {
                        same[1].mv[n] = diff[1].mv[n];
                        continue;
                    }
                }
                do {
                    same[m].mv[n] = tgmv[n];
                } while (++m < 2);
            }
            int n = *cnt;
            if (n == 1 && stack[0].mv[0] == same[0].mv[0] && stack[0].mv[1] == same[0].mv[1]) {
                stack[1].mv[0] = stack[2].mv[0];
                stack[1].mv[1] = stack[2].mv[1];
            }
            do {
                stack[n].weight = 2;
            } while (++n < 2);
            *cnt = 2;
        }
        for (int n = 0; n < *cnt; n++)
            for (int k = 0; k < 2; k++) {
                stack[n].mv[k].x = (int16_t)iclip(stack[n].mv[k].x, left, right);
                stack[n].mv[k].y = (int16_t)iclip(stack[n].mv[k].y, top, bottom);
            }
        switch (refmv_ctx >> 1) {
        case 0: *ctx = imin(newmv_ctx, 1); break;
        case 1: *ctx = 1 + imin(newmv_ctx, 3); break;
        case 2: *ctx = iclip(3 + newmv_ctx, 4, 7); break;
        }
        return;
    } else if (*cnt < 2 && ref0 > 0) {
        // add_single_extended_candidate (C refmvs.c:296-327, 612-629)
        const int sign = sign_bias[ref0 - 1];
        const int sz4 = imin(w4b, h4b);
        auto add_ext = [&](const RefMvBlock &c) {
            for (int n = 0; n < 2; n++) {
                const int cr = c.ref[n];
                if (cr <= 0) break;
                Mv cm = c.mv[n];
                if (sign ^ sign_bias[cr - 1]) { cm.y = (int16_t)-cm.y; cm.x = (int16_t)-cm.x; }
                int m;
                const int last = *cnt;
                for (m = 0; m < last; m++)
                    if (cm == stack[m].mv[0]) break;
                if (m == last) {
                    stack[m].mv[0] = cm;
                    stack[m].weight = 2;
                    *cnt = last + 1;
                }
            }
        };
        if (n_rows != ~0u)
            for (int x = 0; x < sz4 && *cnt < 2;) {
                const RefMvBlock &c = rmv_at(by - 1, bx + x);
                add_ext(c);
                x += k_bdim[c.bs].w4;
            }
        if (n_cols != ~0u)
            for (int y = 0; y < sz4 && *cnt < 2;) {
                const RefMvBlock &c = rmv_at(by + y, bx - 1);
                add_ext(c);
                y += k_bdim[c.bs].h4;
            }
    }
    for (int n = 0; n < *cnt; n++) {
        stack[n].mv[0].x = (int16_t)iclip(stack[n].mv[0].x, left, right);
        stack[n].mv[0].y = (int16_t)iclip(stack[n].mv[0].y, top, bottom);
    }
    for (int n = *cnt; n < 2; n++) stack[n].mv[0] = tgmv[0];
    *ctx = (refmv_ctx << 4) | (globalmv_ctx << 3) | newmv_ctx;
}

}  // namespace fd
}  // namespace av1
