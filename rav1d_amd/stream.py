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
from .av1dec import Av1Decoder, ivf_frames


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


def run_frame(ctx, fr, stream=None):
    """Enqueue one MiDecFrame on the device; returns its DevicePictureSet (output() = the
    reference-quality picture once the stream reaches it)."""
    ps = DevicePictureSet(fr.up_w, fr.h, fr.bpc, fr.layout)   # upscaled geometry with super-resolution
    final = ctypes.c_int(-1)
    check(lib().mi_frame_run(ctx.h, ctypes.byref(fr), ctypes.byref(ps.pics), ctypes.byref(final),
                             F._stream_ptr(stream)), "mi_frame_run")
    ps.final = final.value
    return ps


def frame_end(ctx, stream=None):
    check(lib().mi_frame_end(ctx.h, F._stream_ptr(stream)), "mi_frame_end")


def decode_ivf(ctx, data, stream=None, sync_each=True):
    """Decode an IVF stream on the device; yields the shown pictures (Frame, device planes) in
    output order. With sync_each, every frame is checked with mi_frame_end before it is shown."""
    dec = Av1Decoder()
    pics = {}
    for tu in ivf_frames(data):
        dec.send(tu)
        for ev in dec.events():
            if ev.frame:
                pics[ev.pic_id] = run_frame(ctx, ev.frame.contents, stream)
                if sync_each:
                    frame_end(ctx, stream)
            if ev.show_pic >= 0:
                yield pics[ev.show_pic].output()
            for i in range(ev.n_release):
                pics.pop(ev.release[i], None)
    frame_end(ctx, stream)


def decode_to_muxer(ctx, data, muxer, stream=None, apply_grain=True, pipelined=True):
    """Decode an IVF stream on the device and write every shown picture through `muxer`
    (rav1d_amd.output.Muxer): the picture leaves HBM once, via mi_output_picture into pinned
    host memory, with film grain applied in that same pass when the frame carries grain and
    apply_grain is set (Dav1dSettings.apply_grain, src/lib.rs). Returns the pictures written.

    pipelined: the host front-end parses temporal unit t + 1 while the device reconstructs
    frame t (rav1d overlaps its entropy pass with reconstruction the same way with frame
    threads, src/thread_task.rs): a shown picture is handed to the muxer once its output copy
    (an event, not a stream sync) has landed, one picture behind; two host pictures alternate.
    Device failures of any frame are reported by the mi_frame_end at the end of the stream.
    Without it every frame is checked by mi_frame_end before it is shown."""
    from .output import HostPicture, output_picture
    import torch
    dec = Av1Decoder()
    pics, n = {}, 0
    hosts = [None, None]
    pending = None                      # (slot, event) of the picture awaiting the muxer

    def flush():
        nonlocal pending, n
        if pending is None:
            return
        slot, ev = pending
        ev.synchronize()
        muxer.write(hosts[slot].pic)
        n += 1
        pending = None

    slot = 0
    for tu in ivf_frames(data):
        dec.send(tu)
        for ev in dec.events():
            if ev.frame:
                pics[ev.pic_id] = run_frame(ctx, ev.frame.contents, stream)
                if not pipelined:
                    frame_end(ctx, stream)
            if ev.show_pic >= 0:
                out = pics[ev.show_pic].output()
                h = hosts[slot]
                if h is None or (h.pic.w, h.pic.h, h.pic.bpc, h.pic.layout) != (out.w, out.h, out.bpc, out.layout):
                    if pending is not None and pending[0] == slot:
                        flush()
                    hosts[slot] = h = HostPicture(out.w, out.h, out.bpc, out.layout)
                fg = ev.fg if (ev.fg_present and apply_grain) else None
                output_picture(ctx, out, h, fg, 0, stream)
                done = torch.cuda.Event()
                done.record(stream if stream is not None else torch.cuda.current_stream())
                flush()                  # the previous picture, while this one is on the device
                pending = (slot, done)
                if not pipelined:
                    flush()
                slot ^= 1
            for i in range(ev.n_release):
                pics.pop(ev.release[i], None)
    flush()
    frame_end(ctx, stream)
    return n
