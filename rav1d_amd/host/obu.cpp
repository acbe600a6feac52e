// obu.cpp — OBU layer: sequence header, frame header, tile-group framing and the reference
// slot bookkeeping of a decoder context. Restates obu.rs (C src/obu.c:60-1750: parse_seq_hdr,
// read_frame_size, parse_frame_hdr, parse_tile_hdr, dav1d_parse_obus) and the slot updates of
// decode.rs submit_frame (C src/decode.c:3363-3753).
#include <cerrno>
#include <climits>
#include <chrono>
#include <new>
#include <cstdio>

#include "decoder.h"

namespace av1 {

static int poc_diff(int bits, int a, int b) {
    if (!bits) return 0;
    const int mask = 1 << (bits - 1);
    const int d = a - b;
    return (d & (mask - 1)) - (d & mask);
}

Decoder::Decoder() {}

void Decoder::set_threads(int n) {
    n = n < 1 ? 1 : n > 64 ? 64 : n;
    if (n == threads_) return;
    for (auto &j : running_) j->wait();
    running_.clear();
    threads_ = n;
    pool_.reset(n > 1 ? new WorkerPool(n - 1) : nullptr);
}

int Decoder::parse_seq_hdr(Bits &gb, SeqHdr &s) {
    memset(&s, 0, sizeof(s));
    s.profile = gb.bits(3);
    if (s.profile > 2) return -EINVAL;
    s.still_picture = gb.bit();
    s.reduced_still = gb.bit();
    if (s.reduced_still && !s.still_picture) return -EINVAL;
    if (s.reduced_still) {
        s.num_op = 1;
        gb.bits(5);   // seq_level_idx
    } else {
        s.timing_info_present = gb.bit();
        if (s.timing_info_present) {
            gb.bits(32);
            gb.bits(32);
            s.equal_picture_interval = gb.bit();
            if (s.equal_picture_interval && gb.vlc() == 0xffffffffu) return -EINVAL;
            s.decoder_model_info_present = gb.bit();
            if (s.decoder_model_info_present) {
                s.buffer_delay_len = gb.bits(5) + 1;
                gb.bits(32);
                s.buffer_removal_delay_len = gb.bits(5) + 1;
                s.frame_presentation_delay_len = gb.bits(5) + 1;
            }
        }
        const int display_model_info_present = gb.bit();
        s.num_op = gb.bits(5) + 1;
        for (int i = 0; i < s.num_op; i++) {
            s.op_idc[i] = gb.bits(12);
            if (s.op_idc[i] && (!(s.op_idc[i] & 0xff) || !(s.op_idc[i] & 0xf00))) return -EINVAL;
            const int major = 2 + gb.bits(3);
            gb.bits(2);
            if (major > 3) gb.bit();   // tier
            if (s.decoder_model_info_present) {
                s.op_decoder_model_present[i] = gb.bit();
                if (s.op_decoder_model_present[i]) {
                    gb.bits(s.buffer_delay_len);
                    gb.bits(s.buffer_delay_len);
                    gb.bit();
                }
            }
            if (display_model_info_present && gb.bit()) gb.bits(4);
        }
    }
    s.width_n_bits = gb.bits(4) + 1;
    s.height_n_bits = gb.bits(4) + 1;
    s.max_width = gb.bits(s.width_n_bits) + 1;
    s.max_height = gb.bits(s.height_n_bits) + 1;
    if (!s.reduced_still) {
        s.frame_id_numbers_present = gb.bit();
        if (s.frame_id_numbers_present) {
            s.delta_frame_id_n_bits = gb.bits(4) + 2;
            s.frame_id_n_bits = gb.bits(3) + s.delta_frame_id_n_bits + 1;
        }
    }
    s.sb128 = gb.bit();
    s.filter_intra = gb.bit();
    s.intra_edge_filter = gb.bit();
    if (s.reduced_still) {
        s.screen_content_tools = 2;   // adaptive
        s.force_integer_mv = 2;
    } else {
        s.inter_intra = gb.bit();
        s.masked_compound = gb.bit();
        s.warped_motion = gb.bit();
        s.dual_filter = gb.bit();
        s.order_hint = gb.bit();
        if (s.order_hint) {
            s.jnt_comp = gb.bit();
            s.ref_frame_mvs = gb.bit();
        }
        s.screen_content_tools = gb.bit() ? 2 : gb.bit();
        s.force_integer_mv = s.screen_content_tools ? (gb.bit() ? 2 : gb.bit()) : 2;
        if (s.order_hint) s.order_hint_n_bits = gb.bits(3) + 1;
    }
    s.super_res = gb.bit();
    s.cdef = gb.bit();
    s.restoration = gb.bit();
    s.hbd = gb.bit();
    if (s.profile == 2 && s.hbd) s.hbd += gb.bit();
    s.bpc = 8 + 2 * s.hbd;
    if (s.profile != 1) s.monochrome = gb.bit();
    s.color_description_present = gb.bit();
    if (s.color_description_present) {
        s.pri = gb.bits(8);
        s.trc = gb.bits(8);
        s.mtrx = gb.bits(8);
    } else {
        s.pri = 2;
        s.trc = 2;
        s.mtrx = 2;
    }
    if (s.monochrome) {
        s.color_range = gb.bit();
        s.layout = 0;
        s.ss_hor = s.ss_ver = 1;
    } else if (s.pri == 1 && s.trc == 13 && s.mtrx == 0) {   // BT709 primaries, sRGB, identity
        s.layout = 3;
        s.color_range = 1;
        if (s.profile != 1 && !(s.profile == 2 && s.hbd == 2)) return -EINVAL;
    } else {
        s.color_range = gb.bit();
        switch (s.profile) {
        case 0: s.layout = 1; s.ss_hor = s.ss_ver = 1; break;
        case 1: s.layout = 3; break;
        case 2:
            if (s.hbd == 2) {
                s.ss_hor = gb.bit();
                if (s.ss_hor) s.ss_ver = gb.bit();
            } else {
                s.ss_hor = 1;
            }
            s.layout = s.ss_hor ? (s.ss_ver ? 1 : 2) : 3;
            break;
        }
        if (s.ss_hor & s.ss_ver) s.chr = gb.bits(2);
    }
    if (!s.monochrome) s.separate_uv_delta_q = gb.bit();
    s.film_grain_present = gb.bit();
    gb.bit();   // trailing one bit
    return gb.error ? -EINVAL : 0;
}

int Decoder::read_frame_size(Bits &gb, FrameHdr &h, bool use_ref) {
    const SeqHdr &s = *seq_;
    auto superres = [&]() {
        h.superres_enabled = s.super_res && gb.bit();
        if (h.superres_enabled) {
            const int d = h.superres_denom = 9 + gb.bits(3);
            h.width[0] = imax((h.width[1] * 8 + (d >> 1)) / d, imin(16, h.width[1]));
        } else {
            h.superres_denom = 8;
            h.width[0] = h.width[1];
        }
    };
    if (use_ref) {
        for (int i = 0; i < 7; i++) {
            if (gb.bit()) {
                const RefSlot &r = refs_[h.refidx[i]];
                if (!r.hdr) return -EINVAL;
                h.width[1] = r.hdr->width[1];
                h.height = r.hdr->height;
                h.render_width = r.hdr->render_width;
                h.render_height = r.hdr->render_height;
                superres();
                return 0;
            }
        }
    }
    if (h.frame_size_override) {
        h.width[1] = gb.bits(s.width_n_bits) + 1;
        h.height = gb.bits(s.height_n_bits) + 1;
    } else {
        h.width[1] = s.max_width;
        h.height = s.max_height;
    }
    superres();
    if (gb.bit()) {
        h.render_width = gb.bits(16) + 1;
        h.render_height = gb.bits(16) + 1;
    } else {
        h.render_width = h.width[1];
        h.render_height = h.height;
    }
    return 0;
}

static int tile_log2(int sz, int tgt) {
    int k = 0;
    while ((sz << k) < tgt) k++;
    return k;
}

int Decoder::parse_frame_hdr(Bits &gb, FrameHdr &h) {
    const SeqHdr &s = *seq_;
    h.show_existing_frame = !s.reduced_still && gb.bit();
    if (h.show_existing_frame) {
        h.existing_frame_idx = gb.bits(3);
        if (s.decoder_model_info_present && !s.equal_picture_interval) gb.bits(s.frame_presentation_delay_len);
        if (s.frame_id_numbers_present) {
            h.frame_id = gb.bits(s.frame_id_n_bits);
            const RefSlot &r = refs_[h.existing_frame_idx];
            if (!r.hdr || r.hdr->frame_id != h.frame_id) return -EINVAL;
        }
        return 0;
    }
    h.frame_type = s.reduced_still ? (int)FRAME_KEY : (int)gb.bits(2);
    h.show_frame = s.reduced_still || gb.bit();
    if (h.show_frame) {
        if (s.decoder_model_info_present && !s.equal_picture_interval) gb.bits(s.frame_presentation_delay_len);
        h.showable_frame = h.frame_type != FRAME_KEY;
    } else {
        h.showable_frame = gb.bit();
    }
    h.error_resilient = (h.frame_type == FRAME_KEY && h.show_frame) || h.frame_type == FRAME_SWITCH ||
                        s.reduced_still || gb.bit();
    h.disable_cdf_update = gb.bit();
    h.allow_screen_content_tools = s.screen_content_tools == 2 ? gb.bit() : s.screen_content_tools;
    if (h.allow_screen_content_tools)
        h.force_integer_mv = s.force_integer_mv == 2 ? gb.bit() : s.force_integer_mv;
    else
        h.force_integer_mv = 0;
    if (is_intra_frame(h)) h.force_integer_mv = 1;
    if (s.frame_id_numbers_present) h.frame_id = gb.bits(s.frame_id_n_bits);
    h.frame_size_override = s.reduced_still ? 0 : h.frame_type == FRAME_SWITCH ? 1 : gb.bit();
    h.frame_offset = s.order_hint ? gb.bits(s.order_hint_n_bits) : 0;
    h.primary_ref_frame = !h.error_resilient && !is_intra_frame(h) ? gb.bits(3) : 7;
    if (s.decoder_model_info_present) {
        if (gb.bit()) {   // buffer_removal_time_present
            for (int i = 0; i < s.num_op; i++) {
                if (!s.op_decoder_model_present[i]) continue;
                const int idc = s.op_idc[i];
                const int in_t = (idc >> h.temporal_id) & 1, in_s = (idc >> (h.spatial_id + 8)) & 1;
                if (!idc || (in_t && in_s)) gb.bits(s.buffer_removal_delay_len);
            }
        }
    }
    if (is_intra_frame(h)) {
        h.refresh_frame_flags = (h.frame_type == FRAME_KEY && h.show_frame) ? 0xff : gb.bits(8);
        if (h.refresh_frame_flags != 0xff && h.error_resilient && s.order_hint)
            for (int i = 0; i < 8; i++) gb.bits(s.order_hint_n_bits);
        if (read_frame_size(gb, h, false) < 0) return -EINVAL;
        h.allow_intrabc = h.allow_screen_content_tools && !h.superres_enabled && gb.bit();
        h.use_ref_frame_mvs = 0;
    } else {
        h.allow_intrabc = 0;
        h.refresh_frame_flags = h.frame_type == FRAME_SWITCH ? 0xff : gb.bits(8);
        if (h.error_resilient && s.order_hint)
            for (int i = 0; i < 8; i++) gb.bits(s.order_hint_n_bits);
        const int short_signaling = s.order_hint && gb.bit();
        if (short_signaling) {
            // frame_refs_short_signaling (spec 7.8)
            h.refidx[0] = gb.bits(3);
            h.refidx[1] = h.refidx[2] = -1;
            h.refidx[3] = gb.bits(3);
            h.refidx[4] = h.refidx[5] = h.refidx[6] = -1;
            int shifted[8];
            const int cur = 1 << (s.order_hint_n_bits - 1);
            for (int i = 0; i < 8; i++) {
                if (!refs_[i].hdr) return -EINVAL;
                shifted[i] = cur + poc_diff(s.order_hint_n_bits, refs_[i].hdr->frame_offset, h.frame_offset);
            }
            int used[8] = {0};
            used[h.refidx[0]] = used[h.refidx[3]] = 1;
            int latest = -1;
            for (int i = 0; i < 8; i++)
                if (!used[i] && shifted[i] >= cur && shifted[i] >= latest) {
                    h.refidx[6] = i;
                    latest = shifted[i];
                }
            if (latest != -1) used[h.refidx[6]] = 1;
            int earliest = INT_MAX;
            for (int i = 0; i < 8; i++)
                if (!used[i] && shifted[i] >= cur && shifted[i] < earliest) {
                    h.refidx[4] = i;
                    earliest = shifted[i];
                }
            if (earliest != INT_MAX) used[h.refidx[4]] = 1;
            earliest = INT_MAX;
            for (int i = 0; i < 8; i++)
                if (!used[i] && shifted[i] >= cur && shifted[i] < earliest) {
                    h.refidx[5] = i;
                    earliest = shifted[i];
                }
            if (earliest != INT_MAX) used[h.refidx[5]] = 1;
            for (int i = 1; i < 7; i++) {
                if (h.refidx[i] >= 0) continue;
                latest = -1;
                for (int j = 0; j < 8; j++)
                    if (!used[j] && shifted[j] < cur && shifted[j] >= latest) {
                        h.refidx[i] = j;
                        latest = shifted[j];
                    }
                if (latest != -1) used[h.refidx[i]] = 1;
            }
            earliest = INT_MAX;
            int ref = -1;
            for (int i = 0; i < 8; i++)
                if (shifted[i] < earliest) {
                    ref = i;
                    earliest = shifted[i];
                }
            for (int i = 0; i < 7; i++)
                if (h.refidx[i] < 0) h.refidx[i] = ref;
        }
        for (int i = 0; i < 7; i++) {
            if (!short_signaling) h.refidx[i] = gb.bits(3);
            if (s.frame_id_numbers_present) {
                const int delta = gb.bits(s.delta_frame_id_n_bits);
                const int id = (h.frame_id + (1 << s.frame_id_n_bits) - delta - 1) & ((1 << s.frame_id_n_bits) - 1);
                const RefSlot &r = refs_[h.refidx[i]];
                if (!r.hdr || r.hdr->frame_id != id) return -EINVAL;
            }
        }
        if (read_frame_size(gb, h, !h.error_resilient && h.frame_size_override) < 0) return -EINVAL;
        h.hp = !h.force_integer_mv && gb.bit();
        h.subpel_filter_mode = gb.bit() ? (int)FILTER_SWITCHABLE : (int)gb.bits(2);
        h.switchable_motion_mode = gb.bit();
        h.use_ref_frame_mvs = !h.error_resilient && s.ref_frame_mvs && s.order_hint && gb.bit();
    }
    h.refresh_context = !s.reduced_still && !h.disable_cdf_update && !gb.bit();

    // tile info
    auto &t = h.tiling;
    t.uniform = gb.bit();
    const int sbsz_min1 = (64 << s.sb128) - 1, sbsz_log2 = 6 + s.sb128;
    const int sbw = (h.width[0] + sbsz_min1) >> sbsz_log2, sbh = (h.height + sbsz_min1) >> sbsz_log2;
    const int max_tile_width_sb = 4096 >> sbsz_log2;
    int max_tile_area_sb = 4096 * 2304 >> (2 * sbsz_log2);
    t.min_log2_cols = tile_log2(max_tile_width_sb, sbw);
    t.max_log2_cols = tile_log2(1, imin(sbw, 64));
    t.max_log2_rows = tile_log2(1, imin(sbh, 64));
    const int min_log2_tiles = imax(tile_log2(max_tile_area_sb, sbw * sbh), t.min_log2_cols);
    if (t.uniform) {
        for (t.log2_cols = t.min_log2_cols; t.log2_cols < t.max_log2_cols && gb.bit(); t.log2_cols++) {}
        const int tw = 1 + ((sbw - 1) >> t.log2_cols);
        t.cols = 0;
        for (int x = 0; x < sbw; x += tw, t.cols++) t.col_start_sb[t.cols] = x;
        t.min_log2_rows = imax(min_log2_tiles - t.log2_cols, 0);
        for (t.log2_rows = t.min_log2_rows; t.log2_rows < t.max_log2_rows && gb.bit(); t.log2_rows++) {}
        const int th = 1 + ((sbh - 1) >> t.log2_rows);
        t.rows = 0;
        for (int y = 0; y < sbh; y += th, t.rows++) t.row_start_sb[t.rows] = y;
    } else {
        t.cols = 0;
        int widest = 0;
        max_tile_area_sb = sbw * sbh;
        for (int x = 0; x < sbw && t.cols < 64; t.cols++) {
            const int wsb = imin(sbw - x, max_tile_width_sb);
            const int tw = wsb > 1 ? 1 + (int)gb.uniform(wsb) : 1;
            t.col_start_sb[t.cols] = x;
            x += tw;
            widest = imax(widest, tw);
        }
        t.log2_cols = tile_log2(1, t.cols);
        if (min_log2_tiles) max_tile_area_sb >>= min_log2_tiles + 1;
        const int max_tile_height_sb = imax(max_tile_area_sb / widest, 1);
        t.rows = 0;
        for (int y = 0; y < sbh && t.rows < 64; t.rows++) {
            const int hsb = imin(sbh - y, max_tile_height_sb);
            const int th = hsb > 1 ? 1 + (int)gb.uniform(hsb) : 1;
            t.row_start_sb[t.rows] = y;
            y += th;
        }
        t.log2_rows = tile_log2(1, t.rows);
    }
    t.col_start_sb[t.cols] = sbw;
    t.row_start_sb[t.rows] = sbh;
    if (t.log2_cols || t.log2_rows) {
        t.update = gb.bits(t.log2_cols + t.log2_rows);
        if (t.update >= t.cols * t.rows) return -EINVAL;
        t.n_bytes = gb.bits(2) + 1;
    } else {
        t.n_bytes = t.update = 0;
    }

    // quantization
    auto &q = h.quant;
    q.yac = gb.bits(8);
    q.ydc_delta = gb.bit() ? gb.sbits(7) : 0;
    if (!s.monochrome) {
        const int diff_uv = s.separate_uv_delta_q ? gb.bit() : 0;
        q.udc_delta = gb.bit() ? gb.sbits(7) : 0;
        q.uac_delta = gb.bit() ? gb.sbits(7) : 0;
        if (diff_uv) {
            q.vdc_delta = gb.bit() ? gb.sbits(7) : 0;
            q.vac_delta = gb.bit() ? gb.sbits(7) : 0;
        } else {
            q.vdc_delta = q.udc_delta;
            q.vac_delta = q.uac_delta;
        }
    }
    q.qm = gb.bit();
    if (q.qm) {
        q.qm_y = gb.bits(4);
        q.qm_u = gb.bits(4);
        q.qm_v = s.separate_uv_delta_q ? (int)gb.bits(4) : q.qm_u;
    }

    // segmentation
    auto &sg = h.seg;
    sg.enabled = gb.bit();
    if (sg.enabled) {
        if (h.primary_ref_frame == 7) {
            sg.update_map = 1;
            sg.temporal = 0;
            sg.update_data = 1;
        } else {
            sg.update_map = gb.bit();
            sg.temporal = sg.update_map ? gb.bit() : 0;
            sg.update_data = gb.bit();
        }
        if (sg.update_data) {
            sg.preskip = 0;
            sg.last_active_segid = -1;
            for (int i = 0; i < 8; i++) {
                SegData &d = sg.d[i];
                auto feat = [&](int bits, int sgn) -> int {
                    if (!gb.bit()) return 0;
                    sg.last_active_segid = i;
                    return sgn ? gb.sbits(bits) : (int)gb.bits(bits);
                };
                d.delta_q = feat(9, 1);
                d.delta_lf_y_v = feat(7, 1);
                d.delta_lf_y_h = feat(7, 1);
                d.delta_lf_u = feat(7, 1);
                d.delta_lf_v = feat(7, 1);
                if (gb.bit()) {
                    d.ref = gb.bits(3);
                    sg.last_active_segid = i;
                    sg.preskip = 1;
                } else {
                    d.ref = -1;
                }
                if ((d.skip = gb.bit())) {
                    sg.last_active_segid = i;
                    sg.preskip = 1;
                }
                if ((d.globalmv = gb.bit())) {
                    sg.last_active_segid = i;
                    sg.preskip = 1;
                }
            }
        } else {
            const RefSlot &r = refs_[h.refidx[h.primary_ref_frame]];
            if (!r.hdr) return -EINVAL;
            memcpy(sg.d, r.hdr->seg.d, sizeof(sg.d));
            sg.preskip = r.hdr->seg.preskip;
            sg.last_active_segid = r.hdr->seg.last_active_segid;
        }
    } else {
        memset(sg.d, 0, sizeof(sg.d));
        for (int i = 0; i < 8; i++) sg.d[i].ref = -1;
        sg.preskip = 0;
        sg.last_active_segid = 0;
    }

    // delta q / lf
    h.delta.q_present = q.yac ? gb.bit() : 0;
    h.delta.q_res_log2 = h.delta.q_present ? gb.bits(2) : 0;
    h.delta.lf_present = h.delta.q_present && !h.allow_intrabc && gb.bit();
    h.delta.lf_res_log2 = h.delta.lf_present ? gb.bits(2) : 0;
    h.delta.lf_multi = h.delta.lf_present ? gb.bit() : 0;

    const int delta_lossless = !q.ydc_delta && !q.udc_delta && !q.uac_delta && !q.vdc_delta && !q.vac_delta;
    h.all_lossless = 1;
    for (int i = 0; i < 8; i++) {
        sg.qidx[i] = sg.enabled ? iclip(q.yac + sg.d[i].delta_q, 0, 255) : q.yac;
        sg.lossless[i] = !sg.qidx[i] && delta_lossless;
        h.all_lossless &= sg.lossless[i];
    }

    // loop filter
    auto &lf = h.lf;
    static const int def_ref_delta[8] = {1, 0, 0, 0, -1, 0, -1, -1};
    if (h.all_lossless || h.allow_intrabc) {
        lf.level_y[0] = lf.level_y[1] = lf.level_u = lf.level_v = 0;
        lf.sharpness = 0;
        lf.mode_ref_delta_enabled = 1;
        lf.mode_ref_delta_update = 1;
        memcpy(lf.ref_delta, def_ref_delta, sizeof(lf.ref_delta));
        lf.mode_delta[0] = lf.mode_delta[1] = 0;
    } else {
        lf.level_y[0] = gb.bits(6);
        lf.level_y[1] = gb.bits(6);
        if (!s.monochrome && (lf.level_y[0] || lf.level_y[1])) {
            lf.level_u = gb.bits(6);
            lf.level_v = gb.bits(6);
        }
        lf.sharpness = gb.bits(3);
        if (h.primary_ref_frame == 7) {
            memcpy(lf.ref_delta, def_ref_delta, sizeof(lf.ref_delta));
            lf.mode_delta[0] = lf.mode_delta[1] = 0;
        } else {
            const RefSlot &r = refs_[h.refidx[h.primary_ref_frame]];
            if (!r.hdr) return -EINVAL;
            memcpy(lf.ref_delta, r.hdr->lf.ref_delta, sizeof(lf.ref_delta));
            memcpy(lf.mode_delta, r.hdr->lf.mode_delta, sizeof(lf.mode_delta));
        }
        lf.mode_ref_delta_enabled = gb.bit();
        if (lf.mode_ref_delta_enabled) {
            lf.mode_ref_delta_update = gb.bit();
            if (lf.mode_ref_delta_update) {
                for (int i = 0; i < 8; i++)
                    if (gb.bit()) lf.ref_delta[i] = gb.sbits(7);
                for (int i = 0; i < 2; i++)
                    if (gb.bit()) lf.mode_delta[i] = gb.sbits(7);
            }
        }
    }

    // cdef
    if (!h.all_lossless && s.cdef && !h.allow_intrabc) {
        h.cdef.damping = gb.bits(2) + 3;
        h.cdef.n_bits = gb.bits(2);
        for (int i = 0; i < (1 << h.cdef.n_bits); i++) {
            h.cdef.y_strength[i] = gb.bits(6);
            if (!s.monochrome) h.cdef.uv_strength[i] = gb.bits(6);
        }
    } else {
        h.cdef.n_bits = 0;
        h.cdef.y_strength[0] = h.cdef.uv_strength[0] = 0;
    }

    // loop restoration
    if ((!h.all_lossless || h.superres_enabled) && s.restoration && !h.allow_intrabc) {
        // lr_type as coded is Remap_Lr_Type's index: 0 NONE, 1 SWITCHABLE, 2 WIENER, 3 SGRPROJ
        h.lr.type[0] = gb.bits(2);
        if (!s.monochrome) {
            h.lr.type[1] = gb.bits(2);
            h.lr.type[2] = gb.bits(2);
        } else {
            h.lr.type[1] = h.lr.type[2] = RESTORE_NONE;
        }
        if (h.lr.type[0] || h.lr.type[1] || h.lr.type[2]) {
            h.lr.unit_size[0] = 6 + s.sb128;
            if (gb.bit()) {
                h.lr.unit_size[0]++;
                if (!s.sb128) h.lr.unit_size[0] += gb.bit();
            }
            h.lr.unit_size[1] = h.lr.unit_size[0];
            if ((h.lr.type[1] || h.lr.type[2]) && s.ss_hor == 1 && s.ss_ver == 1)
                h.lr.unit_size[1] -= gb.bit();
        } else {
            h.lr.unit_size[0] = 8;
        }
    } else {
        h.lr.type[0] = h.lr.type[1] = h.lr.type[2] = RESTORE_NONE;
    }

    h.txfm_mode = h.all_lossless ? TXMODE_4X4_ONLY : gb.bit() ? TXMODE_SWITCHABLE : TXMODE_LARGEST;
    h.switchable_comp_refs = !is_intra_frame(h) ? gb.bit() : 0;
    h.skip_mode_allowed = 0;
    if (h.switchable_comp_refs && !is_intra_frame(h) && s.order_hint) {
        const int poc = h.frame_offset, nb = s.order_hint_n_bits;
        unsigned off_before = 0xffffffffu;
        int off_after = -1, before_idx = 0, after_idx = 0;
        for (int i = 0; i < 7; i++) {
            const RefSlot &r = refs_[h.refidx[i]];
            if (!r.hdr) return -EINVAL;
            const int rp = r.hdr->frame_offset;
            const int d = poc_diff(nb, rp, poc);
            if (d > 0) {
                if (off_after == -1 || poc_diff(nb, off_after, rp) > 0) {
                    off_after = rp;
                    after_idx = i;
                }
            } else if (d < 0 && (off_before == 0xffffffffu || poc_diff(nb, rp, (int)off_before) > 0)) {
                off_before = rp;
                before_idx = i;
            }
        }
        if (off_before != 0xffffffffu && off_after != -1) {
            h.skip_mode_refs[0] = imin(before_idx, after_idx);
            h.skip_mode_refs[1] = imax(before_idx, after_idx);
            h.skip_mode_allowed = 1;
        } else if (off_before != 0xffffffffu) {
            unsigned off_before2 = 0xffffffffu;
            int before2_idx = 0;
            for (int i = 0; i < 7; i++) {
                const int rp = refs_[h.refidx[i]].hdr->frame_offset;
                if (poc_diff(nb, rp, (int)off_before) < 0) {
                    if (off_before2 == 0xffffffffu || poc_diff(nb, rp, (int)off_before2) > 0) {
                        off_before2 = rp;
                        before2_idx = i;
                    }
                }
            }
            if (off_before2 != 0xffffffffu) {
                h.skip_mode_refs[0] = imin(before_idx, before2_idx);
                h.skip_mode_refs[1] = imax(before_idx, before2_idx);
                h.skip_mode_allowed = 1;
            }
        }
    }
    h.skip_mode_enabled = h.skip_mode_allowed ? gb.bit() : 0;
    h.warp_motion = !h.error_resilient && !is_intra_frame(h) && s.warped_motion && gb.bit();
    h.reduced_txtp_set = gb.bit();

    for (int i = 0; i < 7; i++) {
        h.gmv[i] = WarpParams{WM_IDENTITY, {0, 0, 1 << 16, 0, 0, 1 << 16}, {0, 0, 0, 0}};
    }
    if (!is_intra_frame(h)) {
        for (int i = 0; i < 7; i++) {
            WarpParams &g = h.gmv[i];
            g.type = !gb.bit() ? WM_IDENTITY : gb.bit() ? WM_ROT_ZOOM : gb.bit() ? WM_TRANSLATION : WM_AFFINE;
            if (g.type == WM_IDENTITY) continue;
            WarpParams def{WM_IDENTITY, {0, 0, 1 << 16, 0, 0, 1 << 16}, {0, 0, 0, 0}};
            const WarpParams *ref = &def;
            if (h.primary_ref_frame != 7) {
                const RefSlot &r = refs_[h.refidx[h.primary_ref_frame]];
                if (!r.hdr) return -EINVAL;
                ref = &r.hdr->gmv[i];
            }
            int32_t *m = g.matrix;
            const int32_t *rm = ref->matrix;
            int bits, shift;
            if (g.type >= WM_ROT_ZOOM) {
                m[2] = (1 << 16) + 2 * gb.subexp((rm[2] - (1 << 16)) >> 1, 12);
                m[3] = 2 * gb.subexp(rm[3] >> 1, 12);
                bits = 12;
                shift = 10;
            } else {
                bits = 9 - !h.hp;
                shift = 13 + !h.hp;
            }
            if (g.type == WM_AFFINE) {
                m[4] = 2 * gb.subexp(rm[4] >> 1, 12);
                m[5] = (1 << 16) + 2 * gb.subexp((rm[5] - (1 << 16)) >> 1, 12);
            } else {
                m[4] = -m[3];
                m[5] = m[2];
            }
            m[0] = gb.subexp(rm[0] >> shift, bits) * (1 << shift);
            m[1] = gb.subexp(rm[1] >> shift, bits) * (1 << shift);
        }
    }

    // film grain
    auto &fg = h.fg;
    fg.present = s.film_grain_present && (h.show_frame || h.showable_frame) && gb.bit();
    memset(&fg.data, 0, sizeof(fg.data));
    if (fg.present) {
        const unsigned seed = gb.bits(16);
        fg.update = h.frame_type != FRAME_INTER || gb.bit();
        if (!fg.update) {
            const int refidx = gb.bits(3);
            int i;
            for (i = 0; i < 7; i++)
                if (h.refidx[i] == refidx) break;
            if (i == 7 || !refs_[refidx].hdr) return -EINVAL;
            fg.data = refs_[refidx].hdr->fg.data;
            fg.data.seed = seed;
        } else {
            MiFilmGrainData &d = fg.data;
            d.seed = seed;
            d.num_y_points = gb.bits(4);
            if (d.num_y_points > 14) return -EINVAL;
            for (int i = 0; i < d.num_y_points; i++) {
                d.y_points[i][0] = gb.bits(8);
                if (i && d.y_points[i - 1][0] >= d.y_points[i][0]) return -EINVAL;
                d.y_points[i][1] = gb.bits(8);
            }
            d.chroma_scaling_from_luma = !s.monochrome && gb.bit();
            if (s.monochrome || d.chroma_scaling_from_luma || (s.ss_ver == 1 && s.ss_hor == 1 && !d.num_y_points)) {
                d.num_uv_points[0] = d.num_uv_points[1] = 0;
            } else {
                for (int pl = 0; pl < 2; pl++) {
                    d.num_uv_points[pl] = gb.bits(4);
                    if (d.num_uv_points[pl] > 10) return -EINVAL;
                    for (int i = 0; i < d.num_uv_points[pl]; i++) {
                        d.uv_points[pl][i][0] = gb.bits(8);
                        if (i && d.uv_points[pl][i - 1][0] >= d.uv_points[pl][i][0]) return -EINVAL;
                        d.uv_points[pl][i][1] = gb.bits(8);
                    }
                }
            }
            if (s.ss_hor == 1 && s.ss_ver == 1 && !!d.num_uv_points[0] != !!d.num_uv_points[1]) return -EINVAL;
            d.scaling_shift = gb.bits(2) + 8;
            d.ar_coeff_lag = gb.bits(2);
            const int num_y_pos = 2 * d.ar_coeff_lag * (d.ar_coeff_lag + 1);
            if (d.num_y_points)
                for (int i = 0; i < num_y_pos; i++) d.ar_coeffs_y[i] = (int8_t)(gb.bits(8) - 128);
            for (int pl = 0; pl < 2; pl++)
                if (d.num_uv_points[pl] || d.chroma_scaling_from_luma) {
                    const int n = num_y_pos + !!d.num_y_points;
                    for (int i = 0; i < n; i++) d.ar_coeffs_uv[pl][i] = (int8_t)(gb.bits(8) - 128);
                    if (!d.num_y_points) d.ar_coeffs_uv[pl][n] = 0;
                }
            d.ar_coeff_shift = gb.bits(2) + 6;
            d.grain_scale_shift = gb.bits(2);
            for (int pl = 0; pl < 2; pl++)
                if (d.num_uv_points[pl]) {
                    d.uv_mult[pl] = gb.bits(8) - 128;
                    d.uv_luma_mult[pl] = gb.bits(8) - 128;
                    d.uv_offset[pl] = gb.bits(9) - 256;
                }
            d.overlap_flag = gb.bit();
            d.clip_to_restricted_range = gb.bit();
        }
    }
    return gb.error ? -EINVAL : 0;
}

// Parse one OBU at data (size bytes available); *used = its total length.
int Decoder::parse_obu(const uint8_t *data, size_t size, size_t *used) {
    Bits gb;
    gb.init(data, size);
    gb.bit();   // forbidden
    const int type = gb.bits(4);
    const int has_ext = gb.bit(), has_len = gb.bit();
    gb.bit();
    int temporal_id = 0, spatial_id = 0;
    if (has_ext) {
        temporal_id = gb.bits(3);
        spatial_id = gb.bits(2);
        gb.bits(3);
    }
    const size_t len = has_len ? gb.uleb128() : size - 1 - has_ext;
    if (gb.error) return -EINVAL;
    const size_t hdr_bytes = gb.byte_pos();
    if (len > size - hdr_bytes) return -EINVAL;
    *used = hdr_bytes + len;
    const uint8_t *obu = data + hdr_bytes;

    if (type != 1 && type != 2 && has_ext && seq_ && seq_->op_idc[0]) {
        const int idc = seq_->op_idc[0];
        if (!((idc >> temporal_id) & 1) || !((idc >> (spatial_id + 8)) & 1)) return 0;
    }
    switch (type) {
    case 1: {   // sequence header
        Bits b;
        b.init(obu, len);
        auto s = std::make_unique<SeqHdr>();
        int r = parse_seq_hdr(b, *s);
        if (r < 0) {
            error = "bad sequence header";
            return r;
        }
        if (seq_ && memcmp(s.get(), seq_.get(), sizeof(SeqHdr))) {
            // a new sequence: forget everything decoded under the old one
            int old_ids[8];
            for (int i = 0; i < 8; i++) old_ids[i] = refs_[i].pic_id;
            for (auto &rs : refs_) rs = RefSlot();
            DecEvent ev;
            release_unused(ev, old_ids);
            if (!ev.release.empty()) out_.push_back(std::move(ev));
        }
        seq_ = std::move(s);
        break;
    }
    case 7:   // redundant frame header
        if (frame_hdr_) break;
        // fall through
    case 3:
    case 6: {
        if (!seq_) return -EINVAL;
        Bits b;
        b.init(obu, len);
        frame_hdr_ = std::make_shared<FrameHdr>();
        memset(frame_hdr_.get(), 0, sizeof(FrameHdr));
        frame_hdr_->temporal_id = temporal_id;
        frame_hdr_->spatial_id = spatial_id;
        int r = parse_frame_hdr(b, *frame_hdr_);
        if (r < 0) {
            frame_hdr_.reset();
            error = "bad frame header";
            return r;
        }
        tiles_.clear();
        n_tiles_ = 0;
        if (frame_hdr_->show_existing_frame) {
            if (type == 6) return -EINVAL;
            const int idx = frame_hdr_->existing_frame_idx;
            resolve(refs_[idx]);
            const RefSlot &rs = refs_[idx];
            if (!rs.hdr || rs.pic_id < 0) return -EINVAL;
            DecEvent ev;
            ev.show_pic = rs.pic_id;
            ev.fg_present = rs.hdr->fg.present;
            ev.fg = rs.hdr->fg.data;
            ev.mtrx_identity = seq_->mtrx == 0;
            if (rs.hdr->frame_type == FRAME_KEY) {
                // a shown key frame refreshes every slot (obu.rs show_existing_frame)
                int old_ids[8];
                for (int i = 0; i < 8; i++) old_ids[i] = refs_[i].pic_id;
                RefSlot key = rs;
                key.showable = 0;
                for (int i = 0; i < 8; i++) {
                    refs_[i] = key;
                    if (i != idx) refs_[i].mvs.reset();
                }
                release_unused(ev, old_ids);
            }
            out_.push_back(std::move(ev));
            frame_hdr_.reset();
            break;
        }
        if (type == 6) {
            b.byte_align();
            const size_t off = b.byte_pos();
            r = 0;
            // the tile group follows in the same OBU
            Bits tg;
            tg.init(obu + off, len - off);
            const int n = frame_hdr_->tiling.cols * frame_hdr_->tiling.rows;
            const int have_pos = n > 1 ? tg.bit() : 0;
            int start = 0, end = n - 1;
            if (have_pos) {
                const int nb = frame_hdr_->tiling.log2_cols + frame_hdr_->tiling.log2_rows;
                start = tg.bits(nb);
                end = tg.bits(nb);
            }
            tg.byte_align();
            const size_t toff = off + tg.byte_pos();
            if (start != n_tiles_ || start > end || toff > len) return -EINVAL;
            tiles_.push_back({obu + toff, len - toff, start, end});
            n_tiles_ += end - start + 1;
        } else {
            b.bit();   // trailing bit
        }
        break;
    }
    case 4: {   // tile group
        if (!frame_hdr_) return -EINVAL;
        Bits tg;
        tg.init(obu, len);
        const int n = frame_hdr_->tiling.cols * frame_hdr_->tiling.rows;
        const int have_pos = n > 1 ? tg.bit() : 0;
        int start = 0, end = n - 1;
        if (have_pos) {
            const int nb = frame_hdr_->tiling.log2_cols + frame_hdr_->tiling.log2_rows;
            start = tg.bits(nb);
            end = tg.bits(nb);
        }
        tg.byte_align();
        const size_t toff = tg.byte_pos();
        if (start != n_tiles_ || start > end || toff > len) return -EINVAL;
        tiles_.push_back({obu + toff, len - toff, start, end});
        n_tiles_ += end - start + 1;
        break;
    }
    default:   // temporal delimiter, metadata, padding, tile list: nothing for the pixels
        break;
    }
    if (frame_hdr_ && !frame_hdr_->show_existing_frame &&
        n_tiles_ == frame_hdr_->tiling.cols * frame_hdr_->tiling.rows && !tiles_.empty()) {
        const int r = submit_frame();
        frame_hdr_.reset();
        tiles_.clear();
        n_tiles_ = 0;
        if (r < 0) return r;
    }
    return 0;
}

void Decoder::release_unused(DecEvent &ev, const int *old_ids) {
    for (int i = 0; i < 8; i++) {
        const int id = old_ids[i];
        if (id < 0) continue;
        bool live = false;
        for (int j = 0; j < 8; j++) live |= refs_[j].pic_id == id;
        bool listed = false;
        for (int v : ev.release) listed |= v == id;
        if (!live && !listed) ev.release.push_back(id);
    }
}

void FrameProgress::publish(std::shared_ptr<const std::vector<TmvBlock>> m,
                            std::shared_ptr<const std::vector<uint8_t>> sm) {
    std::lock_guard<std::mutex> g(m_);
    if (published_) return;
    mvs = std::move(m);
    segmap = std::move(sm);
    published_ = true;
    cv_.notify_all();
}

void FrameProgress::publish_cdf(std::shared_ptr<const Cdf> c) {
    std::lock_guard<std::mutex> g(m_);
    cdf = std::move(c);
    cdf_ready_ = true;
    cv_.notify_all();
}

void FrameProgress::rows_done(int n) {
    std::lock_guard<std::mutex> g(m_);
    if (n > rows_) {
        rows_ = n;
        cv_.notify_all();
    }
}

void FrameProgress::set_tiling(int cols, int sb_shift, int sbh) {
    std::lock_guard<std::mutex> g(m_);
    cols_ = cols;
    sb_shift_ = sb_shift;
    front_ = 0;
    row_cols_.assign(sbh, 0);
}

void FrameProgress::tile_row_done(int sby) {
    std::lock_guard<std::mutex> g(m_);
    if (sby < 0 || sby >= (int)row_cols_.size()) return;
    row_cols_[sby]++;
    const int f0 = front_;
    while (front_ < (int)row_cols_.size() && row_cols_[front_] == cols_) front_++;
    if (front_ != f0 && (front_ << sb_shift_) > rows_) {
        rows_ = front_ << sb_shift_;
        cv_.notify_all();
    }
}

void FrameProgress::fail() {
    std::lock_guard<std::mutex> g(m_);
    failed_ = true;
    cv_.notify_all();
}

bool FrameProgress::wait_published() {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return published_ || failed_; });
    return !failed_;
}

bool FrameProgress::wait_cdf() {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return cdf_ready_ || failed_; });
    return !failed_;
}

bool FrameProgress::wait_rows(int n) {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [&] { return rows_ >= n || failed_; });
    return !failed_;
}

// A copy of a reference slot whose frame is still being decoded on a worker (the job's own
// thread, for the slots it read at submission): the buffers that frame publishes as it starts
// (saved MVs, segment ids: their rows are waited for as they are read) and, when `need_cdf`,
// its entropy state. The slot keeps the job for those waits.
static int resolve_copy(RefSlot &r, bool need_cdf) {
    if (!r.job) return 0;
    FrameProgress &p = r.job->prog;
    if (!p.wait_published() || (need_cdf && r.cdf_from_job && !p.wait_cdf())) return -EINVAL;
    if (need_cdf && r.cdf_from_job) {
        r.cdf = p.cdf;
        r.cdf_from_job = false;
    }
    r.segmap = p.segmap;
    r.mvs = r.mvs_from_job ? p.mvs : nullptr;
    return 0;
}

int Decoder::submit_frame() {
    const SeqHdr &s = *seq_;
    FrameHdr &h = *frame_hdr_;
    FrameInputs in;
    in.seq = &s;
    in.hdr = &h;
    in.in_cdf = nullptr;
    for (int i = 0; i < 7; i++) in.refs[i] = nullptr;
    // threads > 1: every frame on a worker (an inter frame's job resolves its references
    // itself); the slot CDF of a frame that does not refresh its context is its primary
    // reference's, whose own job may still be adapting it: waited for here
    const bool async = threads_ > 1;
    const bool intra = is_intra_frame(h);
    if (!async) {
        if (!intra) resolve_all();
        if (h.primary_ref_frame != 7) resolve(refs_[h.refidx[h.primary_ref_frame]]);
    } else if (h.primary_ref_frame != 7 && !h.refresh_context) {
        RefSlot &r = refs_[h.refidx[h.primary_ref_frame]];
        if (r.job && r.cdf_from_job) {
            r.cdf = r.job->prog.wait_cdf() ? r.job->prog.cdf : nullptr;   // (null: that frame failed)
            r.cdf_from_job = false;
        }
    }
    if (!intra) {
        for (int i = 0; i < 7; i++) {
            const RefSlot &r = refs_[h.refidx[i]];
            if (!r.hdr || r.pic_id < 0) {
                error = "missing reference";
                return -EINVAL;
            }
            in.refs[i] = &r;
        }
    }
    bool seg_from_primary = false;
    if (h.primary_ref_frame != 7) {
        const RefSlot &r = refs_[h.refidx[h.primary_ref_frame]];
        if (!r.hdr || (!r.cdf && !(r.job && r.cdf_from_job))) return -EINVAL;
        in.in_cdf = r.cdf.get();
        if (h.seg.enabled && (h.seg.temporal || !h.seg.update_map)) {
            const int rw = ((r.hdr->width[0] + 7) >> 3) << 1, rh = ((r.hdr->height + 7) >> 3) << 1;
            const int bw = ((h.width[0] + 7) >> 3) << 1, bh = ((h.height + 7) >> 3) << 1;
            if (rw == bw && rh == bh) {
                in.prev_segmap = r.segmap;
                seg_from_primary = true;
            }
        }
    }
    // split the tile groups into tiles (tile_size_bytes prefixes, decode.rs decode_frame_init_cdf)
    for (const TileData &t : tiles_) {
        const uint8_t *d = t.data;
        size_t sz = t.size;
        for (int j = t.start; j <= t.end; j++) {
            size_t tsz;
            if (j == t.end) {
                tsz = sz;
            } else {
                if ((size_t)h.tiling.n_bytes > sz) return -EINVAL;
                tsz = 0;
                for (int k = 0; k < h.tiling.n_bytes; k++) tsz |= (size_t)*d++ << (k * 8);
                tsz++;
                sz -= h.tiling.n_bytes;
                if (tsz > sz) return -EINVAL;
            }
            in.tiles.push_back({d, tsz});
            d += tsz;
            sz -= tsz;
        }
    }
    static const bool trace = getenv("MI_DEC_TRACE") != nullptr;   // (diagnostics)
    if (trace)
        fprintf(stderr, "frame %d: %dx%d type %d show %d tiles %dx%d upd %d refresh_ctx %d primary %d refresh_flags %02x ref_mvs %d seg %d/%d\n",
                next_pic_, h.width[0], h.height, h.frame_type, h.show_frame, h.tiling.cols, h.tiling.rows, h.tiling.update,
                h.refresh_context, h.primary_ref_frame, h.refresh_frame_flags, h.use_ref_frame_mvs, h.seg.enabled, h.seg.update_map);
    auto work = std::make_shared<FrameWork>();
    FrameResult res;
    std::shared_ptr<FrameJob> job;
    if (async) {
        // frame thread: the job owns copies of what the decoder may replace meanwhile
        while ((int)running_.size() >= threads_) {
            running_.front()->wait();
            running_.pop_front();
        }
        job = std::make_shared<FrameJob>();
        job->seq = s;
        job->hdr = frame_hdr_;
        job->bufs = tile_bufs_;
        job->in = in;
        job->in.seq = &job->seq;
        job->in.hdr = job->hdr.get();
        job->in.in_cdf = nullptr;
        job->in.prev_segmap = nullptr;
        for (int i = 0; i < 7; i++) {
            job->in.refs[i] = nullptr;
            if (!intra || (h.primary_ref_frame != 7 && i == h.primary_ref_frame)) {
                job->refs[i] = refs_[h.refidx[i]];
                if (!intra) job->in.refs[i] = &job->refs[i];
            }
        }
        job->primary = h.primary_ref_frame != 7 ? h.primary_ref_frame : -1;
        job->seg_from_primary = seg_from_primary;
        job->work = work;
        job->in.pool = pool_.get();
        FrameJob *j = job.get();
        const int pic = next_pic_;
        job->th = std::thread([j, intra, pic] {
            using clk = std::chrono::steady_clock;
            const auto t0 = clk::now();
            auto t1 = t0, t2 = t0;
            try {
                // this frame's maps, published before the references are waited for unless the
                // segment map is the primary reference's
                frame_buffers(*j->in.hdr, j->in.rp_buf, j->in.segmap_buf);
                const FrameHdr &fh = *j->in.hdr;
                if (!fh.seg.enabled || fh.seg.update_map || !j->seg_from_primary)
                    j->prog.publish(intra ? nullptr : j->in.rp_buf, fh.seg.enabled ? j->in.segmap_buf : nullptr);
                // the references' segment maps and motion vectors (their rows are waited for as
                // they are read) and the primary's entropy state (waited for by decode_frame
                // once the frame is set up, when its job is still adapting it)
                for (int i = 0; i < 7 && !j->rc; i++)
                    if (!intra || i == j->primary) {
                        j->rc = resolve_copy(j->refs[i], false);
                        if (j->refs[i].job) j->in.ref_prog[i] = &j->refs[i].job->prog;
                    }
                if (j->rc) {
                    j->err = "reference frame failed";
                } else {
                    if (j->primary >= 0) {
                        const RefSlot &p = j->refs[j->primary];
                        if (p.job && p.cdf_from_job) {
                            j->in.in_cdf_prog = &p.job->prog;
                        } else {
                            j->in_cdf = p.cdf;
                            j->in.in_cdf = p.cdf.get();
                        }
                        if (j->seg_from_primary) {
                            j->in.prev_segmap = p.segmap;
                            j->in.prev_segmap_prog = j->in.ref_prog[j->primary];
                        }
                    }
                    if (j->primary >= 0 && !j->in.in_cdf && !j->in.in_cdf_prog) {
                        j->rc = -EINVAL;
                        j->err = "missing reference entropy state";
                    } else {
                        t1 = clk::now();
                        j->in.progress = &j->prog;
                        j->rc = decode_frame(j->in, *j->work, j->res, j->err);
                    }
                }
                if (j->rc) j->prog.fail();
                // (the references' jobs are no longer waited for: drop them, or every job would
                // keep its references' jobs, and theirs, alive)
                for (RefSlot &r : j->refs) r.job.reset();
                for (FrameProgress *&p : j->in.ref_prog) p = nullptr;
                j->in.prev_segmap_prog = j->in.in_cdf_prog = nullptr;
                // later frames need only the result; the event also needs the intra queue
                j->finish_result();
                t2 = clk::now();
                if (!j->rc) plan_intra_queue(*j->work, j->in.pool);
            } catch (const std::bad_alloc &) {
                j->rc = -ENOMEM;
                j->err = "out of memory";
                j->prog.fail();
            }
            j->finish();
            static const bool jtrace = getenv("MI_DEC_TRACE") != nullptr;   // (diagnostics)
            if (jtrace) {
                auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
                fprintf(stderr, "  job %d: refs %.2f decode %.2f plan %.2f ms (start %.3f)\n", pic, ms(t0, t1), ms(t1, t2),
                        ms(t2, clk::now()), std::chrono::duration<double>(t0.time_since_epoch()).count());
            }
        });
        running_.push_back(job);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        const int r = decode_frame(in, *work, res, error);
        if (!r) plan_intra_queue(*work, nullptr);
        if (trace)
            fprintf(stderr, "  frame %.2f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        if (r < 0) return r;
    }

    DecEvent ev;
    ev.work = work;
    ev.job = job;
    ev.pic_id = next_pic_++;
    if (!intra)
        for (int i = 0; i < 7; i++) ev.ref_pic[i] = in.refs[i]->pic_id;
    if (h.show_frame) {
        ev.show_pic = ev.pic_id;
        ev.fg_present = h.fg.present;
        ev.fg = h.fg.data;
        ev.mtrx_identity = s.mtrx == 0;
    }
    // reference slots (decode.rs submit_frame: refresh_frame_flags)
    std::shared_ptr<const Cdf> slot_cdf;
    if (h.refresh_context) {
        slot_cdf = res.out_cdf;
    } else if (in.in_cdf) {
        slot_cdf = refs_[h.refidx[h.primary_ref_frame]].cdf;
    } else {
        auto c = std::make_shared<Cdf>();
        cdf_init_default(*c, h.quant.yac);
        slot_cdf = c;
    }
    int refpoc[7] = {0};
    if (!intra)
        for (int i = 0; i < 7; i++) refpoc[i] = in.refs[i]->hdr->frame_offset;
    int old_ids[8];
    for (int i = 0; i < 8; i++) old_ids[i] = refs_[i].pic_id;
    auto hdr_c = std::shared_ptr<const FrameHdr>(frame_hdr_);
    const int bw = ((h.width[0] + 7) >> 3) << 1, bh = ((h.height + 7) >> 3) << 1;
    for (int i = 0; i < 8; i++) {
        if (!(h.refresh_frame_flags & (1 << i))) continue;
        RefSlot &rs = refs_[i];
        rs.pic_id = ev.pic_id;
        rs.hdr = hdr_c;
        rs.cdf = slot_cdf;
        rs.segmap = res.segmap;
        rs.mvs = h.allow_intrabc ? nullptr : res.mvs;
        rs.job = job;
        rs.cdf_from_job = job && h.refresh_context;
        rs.mvs_from_job = job && !h.allow_intrabc;
        memcpy(rs.refpoc, refpoc, sizeof(refpoc));
        rs.bw = bw;
        rs.bh = bh;
        rs.showable = h.showable_frame;
    }
    release_unused(ev, old_ids);
    // the new picture itself is dead if no slot holds it and it is not shown
    bool live = false;
    for (int j = 0; j < 8; j++) live |= refs_[j].pic_id == ev.pic_id;
    if (!live) ev.release.push_back(ev.pic_id);
    out_.push_back(std::move(ev));
    return 0;
}

int Decoder::send(const uint8_t *data, size_t size) {
    // keep the bytes alive for the tiles of a frame that spans several calls
    tile_bufs_.push_back(std::make_shared<std::vector<uint8_t>>(data, data + size));
    const uint8_t *p = tile_bufs_.back()->data();
    size_t off = 0;
    while (off < size) {
        size_t used = 0;
        const int r = parse_obu(p + off, size - off, &used);
        if (r < 0) {
            if (error.empty()) error = "OBU parse error";
            return r;
        }
        if (!used) return -EINVAL;
        off += used;
    }
    if (!frame_hdr_) tile_bufs_.clear();
    return 0;
}

int Decoder::pop(DecEvent &ev) {
    if (out_.empty()) return 0;
    ev = std::move(out_.front());
    out_.pop_front();
    if (ev.job) {
        ev.job->wait();
        if (ev.job->rc < 0) {
            error = ev.job->err.empty() ? "frame decode failed" : ev.job->err;
            const int rc = ev.job->rc;
            ev.job.reset();
            return rc;
        }
        ev.job.reset();
    }
    return 1;
}

void Decoder::resolve(RefSlot &r) {
    if (!r.job) return;
    r.job->wait_result();
    if (r.cdf_from_job) r.cdf = r.job->res.out_cdf;
    r.segmap = r.job->res.segmap;
    r.mvs = r.mvs_from_job ? r.job->res.mvs : nullptr;
    r.job.reset();
    r.cdf_from_job = r.mvs_from_job = false;
}

void Decoder::resolve_all() {
    for (RefSlot &r : refs_) resolve(r);
}

Decoder::~Decoder() {
    for (auto &j : running_) j->wait();
}

}  // namespace av1
