"""Stream decode on the device: the front-end's per-frame work lists (rav1d_amd/libmi_av1dec.so,
include/mi_av1dec.h) executed by librav1d_amd.so's frame executor (mi_frame_run / mi_frame_end).

This is the host loop rav1d runs in decode.rs:4526-4550 (decode_tile_sbrow, then filter_sbrow)
with the pixel work moved to the GPU: for every decoder event, the frame's reconstruction and
in-loop filters are enqueued on one stream into device pictures; shown pictures are handed to
the caller (on the device). There is no CPU pixel path here.
"""
import ctypes

from . import MiFramePictures, check, lib
from . import frame as F
from .av1dec import Av1Decoder, stream_units


class DevicePictureSet:
    """The four pictures one frame's pass 2 writes (recon, deblocked, cdef, restored)."""

    def __init__(self, w, h, bpc, layout):
        self.frames = [F.Frame(w, h, bpc, layout) for _ in range(4)]
        self.pics = MiFramePictures()
        for i, fr in enumerate(self.frames):
            self.pics.pics[i] = fr.picture()
        self.final = 0

    def output(self):
        return self.frames[self.final]


def run_frame(ctx, fr, stream=None, refs=None):
    """Enqueue one MiDecFrame on the device; returns its DevicePictureSet (output() = the
    reference-quality picture once the stream reaches it). refs: the frame's seven reference
    pictures (Frame or None, in MiDecEvent.ref_pic order) for an inter frame."""
    ps = DevicePictureSet(fr.up_w, fr.h, fr.bpc, fr.layout)   # upscaled geometry with super-resolution
    for i, r in enumerate(refs or []):
        if r is not None:
            ps.pics.refs[i] = r.picture()
    ps.refs = [r for r in (refs or []) if r is not None]       # keep the reference tensors alive
    final = ctypes.c_int(-1)
    check(lib().mi_frame_run(ctx.h, ctypes.byref(fr), ctypes.byref(ps.pics), ctypes.byref(final),
                             F._stream_ptr(stream)), "mi_frame_run")
    ps.final = final.value
    return ps


def frame_end(ctx, stream=None):
    check(lib().mi_frame_end(ctx.h, F._stream_ptr(stream)), "mi_frame_end")


def _refs(pics, ev, key=lambda p: p):
    """The reference pictures (final Frames) of an event's frame, in ref_pic order."""
    out = []
    for r in ev.ref_pic:
        out.append(key(pics[r]).output() if r >= 0 and r in pics else None)
    return out


def decode_ivf(ctx, data, stream=None, sync_each=True, inloop_filters=14, threads=1):
    """Decode a stream (IVF, Annex B or section 5) on the device; yields the shown pictures (Frame, device planes) in
    output order. With sync_each, every frame is checked with mi_frame_end before it is shown.
    inloop_filters: Dav1dSettings.inloop_filters (rav1d_amd.av1dec.INLOOPFILTER_*). threads > 1: the
    front-end's frame and tile threads (mi_dec_set_threads)."""
    dec = Av1Decoder(threads, inloop_filters=inloop_filters)
    pics = {}
    for tu in stream_units(data):
        dec.send(tu)
        for ev in dec.events():
            if ev.frame:
                pics[ev.pic_id] = run_frame(ctx, ev.frame.contents, stream, _refs(pics, ev))
                if sync_each:
                    frame_end(ctx, stream)
            if ev.show_pic >= 0:
                yield pics[ev.show_pic].output()
            for i in range(ev.n_release):
                pics.pop(ev.release[i], None)
    frame_end(ctx, stream)


_extra_lanes = {}


def _lanes(ctx, stream, n):
    """n (context, stream) pairs for frames in flight: the caller's first, then cached extra
    contexts with their own streams (a context's calls stay on one stream)."""
    import torch
    lanes = [(ctx, stream)]
    key = id(ctx)
    extra = _extra_lanes.setdefault(key, [])
    while len(extra) < n - 1:
        from .frame import Context
        extra.append((Context(torch.cuda.current_device()), torch.cuda.Stream()))
    return lanes + extra[:n - 1]


def decode_to_muxer(ctx, data, muxer, stream=None, apply_grain=True, pipelined=True, threads=8, in_flight=2,
                    inloop_filters=14, stats=None):
    """Decode an IVF stream on the device and write every shown picture through `muxer`
    (rav1d_amd.output.Muxer): the picture leaves HBM once, via mi_output_picture into pinned
    host memory, with film grain applied in that same pass when the frame carries grain and
    apply_grain is set (Dav1dSettings.apply_grain, src/lib.rs). Returns the pictures written.

    pipelined: rav1d's frame threading on this path (src/thread_task.rs):
      * the host front-end decodes frames on `threads` worker threads (each frame's tiles on
        their own threads too), a few temporal units ahead of the device (mi_dec_set_threads);
      * frames are reconstructed `in_flight` at a time, frame k on (context, stream) k % in_flight;
        a frame whose prediction reads other pictures waits for their events first (allintra:
        80 -> 49 ms with 2 lanes; inter streams whose front-end is the bound: unchanged);
      * a shown picture goes to the muxer once its output copy has landed (an event, not a
        stream sync), one picture behind; host pictures rotate.
    Device failures of any frame are reported by the mi_frame_end calls at the end of the
    stream. Without pipelined: one frame at a time, each checked by mi_frame_end before it is
    shown, the front-end one temporal unit at a time (its tiles still on `threads` threads).

    stats: a dict to receive the per-stage breakdown: host time waiting for the
    front-end's events (front_end_ms), host time inside mi_frame_run (run_host_ms), the device
    stages of every frame from mi_ctx_timing (upload_ms / inter_ms / intra_ms / filter_ms,
    upload_bytes), the output copies into host memory (d2h_ms, HIP events) and the muxer's host
    time (mux_ms)."""
    import time

    from . import MiFrameTiming
    from .av1dec import stream_events
    from .output import HostPicture, output_picture
    import torch
    if not pipelined:
        in_flight = 1
    lanes = _lanes(ctx, stream, max(1, in_flight))
    streams = [st if st is not None else torch.cuda.current_stream() for _, st in lanes]
    if len(lanes) > 1:
        for st in streams[1:]:
            st.wait_stream(streams[0])
    pics, done_ev, n = {}, {}, 0
    hosts = [None] * (len(lanes) + 1)
    pending = []                        # (slot, event) of pictures awaiting the muxer, in order
    k = 0
    clock = time.perf_counter
    acc = dict(front_end_ms=0.0, mux_ms=0.0, d2h_ms=0.0)
    out_ev = []
    if stats is not None:
        for lctx, _ in lanes:
            check(lib().mi_ctx_set_timing(lctx.h, 1), "mi_ctx_set_timing")

    def flush(keep):
        nonlocal n
        while len(pending) > keep:
            slot, ev = pending.pop(0)
            ev.synchronize()
            t = clock()
            muxer.write(hosts[slot].pic)
            acc["mux_ms"] += (clock() - t) * 1e3
            n += 1

    slot = 0
    # (without pipelined the front-end still decodes each frame's tiles on `threads` threads,
    # but no temporal unit ahead of the one the device is given)
    events = iter(stream_events(data, threads, lookahead=None if pipelined else 0, inloop_filters=inloop_filters))
    while True:
        t = clock()
        ev = next(events, None)
        acc["front_end_ms"] += (clock() - t) * 1e3
        if ev is None:
            break
        if ev.frame:
            li = k % len(lanes)
            k += 1
            lctx, lst = lanes[li]
            for r in ev.ref_pic:          # pictures this frame's prediction reads
                if r >= 0 and r in done_ev:
                    streams[li].wait_event(done_ev[r])
            # the pictures are allocated (and zero-filled) on the lane's own stream
            with torch.cuda.stream(streams[li]):
                ps = run_frame(lctx, ev.frame.contents, lst, _refs(pics, ev, key=lambda p: p[0]))
            pics[ev.pic_id] = (ps, li)
            e = torch.cuda.Event()
            e.record(streams[li])
            done_ev[ev.pic_id] = e
            if not pipelined:
                frame_end(lctx, lst)
        if ev.show_pic >= 0:
            ps, li = pics[ev.show_pic]
            out = ps.output()
            lctx, lst = lanes[li]
            if any(p[0] == slot for p in pending):
                flush(0)
            h = hosts[slot]
            if h is None or (h.pic.w, h.pic.h, h.pic.bpc, h.pic.layout) != (out.w, out.h, out.bpc, out.layout):
                hosts[slot] = h = HostPicture(out.w, out.h, out.bpc, out.layout)
            fg = ev.fg if (ev.fg_present and apply_grain) else None
            if stats is not None:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(streams[li])
            output_picture(lctx, out, h, fg, ev.mtrx_identity, lst)
            if stats is not None:
                b.record(streams[li])
                out_ev.append((a, b))
            done = torch.cuda.Event()
            done.record(streams[li])
            pending.append((slot, done))
            flush(len(lanes) if pipelined else 0)
            slot = (slot + 1) % len(hosts)
        for i in range(ev.n_release):
            pics.pop(ev.release[i], None)
            done_ev.pop(ev.release[i], None)
    flush(0)
    for lctx, lst in lanes:
        frame_end(lctx, lst)
    if stats is not None:
        tot = dict(frames=0, run_host_ms=0.0, upload_ms=0.0, inter_ms=0.0, intra_ms=0.0, filter_ms=0.0,
                   upload_bytes=0, run_stage_ms=0.0, run_levels_ms=0.0)
        for lctx, _ in lanes:
            tm = MiFrameTiming()
            check(lib().mi_ctx_timing(lctx.h, ctypes.byref(tm)), "mi_ctx_timing")
            check(lib().mi_ctx_set_timing(lctx.h, 0), "mi_ctx_set_timing")
            tot["frames"] += tm.frames
            tot["run_host_ms"] += tm.host_ms
            tot["run_stage_ms"] += tm.stage_ms
            tot["run_levels_ms"] += tm.strips_ms
            for f in ("upload_ms", "inter_ms", "intra_ms", "filter_ms", "upload_bytes"):
                tot[f] += getattr(tm, f)
        acc["d2h_ms"] = sum(a.elapsed_time(b) for a, b in out_ev)
        stats.update(tot)
        stats.update(acc)
    return n
