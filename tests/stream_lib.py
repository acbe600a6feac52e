"""Whole-stream decode through the front-end (rav1d_amd/libmi_av1dec.so) and the oracle's frame
driver (oracle/decode.c), hashed like the reference's md5 muxer (tools/output/md5.rs:541-637).

TEST INFRASTRUCTURE ONLY: this is the checker that pins the CPU restatement (and, through it,
the GPU path) to the reference's own MD5 vectors (tests/dav1d-test-data/**/meson.build).
"""
import ctypes
import hashlib

import numpy as np

from rav1d_amd.av1dec import MiDecFrame
from tests import oracle_lib


def _bind(o):
    if getattr(o, "_dec_bound", False):
        return o
    vp = ctypes.c_void_p
    o.oracle_decode_frame.argtypes = [ctypes.POINTER(MiDecFrame), vp, vp, vp, vp, vp]
    o.oracle_decode_frame.restype = None
    o.oracle_decode_frame_refs.argtypes = [ctypes.POINTER(MiDecFrame), vp, vp, vp, vp, vp, vp, vp, vp]
    o.oracle_decode_frame_refs.restype = None
    o._dec_bound = True
    return o


def alloc_picture(w, h, bpc, layout):
    """dav1d default-allocator geometry (src/picture.rs:98-115): 128-aligned planes."""
    aw, ah = (w + 127) & ~127, (h + 127) & ~127
    ss_hor, ss_ver = int(layout in (1, 2)), int(layout == 1)
    dt = np.uint8 if bpc == 8 else np.uint16
    planes = [np.zeros((ah, aw), dt)]
    if layout:
        planes += [np.zeros((ah >> ss_ver, aw >> ss_hor), dt) for _ in range(2)]
    return planes


def md5_update_picture(md5, planes, w, h, layout):
    """md5_write (tools/output/md5.rs:541-576): visible rows of every plane, pixel bytes LE."""
    md5.update(np.ascontiguousarray(planes[0][:h, :w]).tobytes())
    if layout:
        ss_hor, ss_ver = int(layout in (1, 2)), int(layout == 1)
        cw, ch = (w + ss_hor) >> ss_hor, (h + ss_ver) >> ss_ver
        for p in (1, 2):
            md5.update(np.ascontiguousarray(planes[p][:ch, :cw]).tobytes())


def oracle_frame(fr, refs=None):
    """Reconstruct one MiDecFrame through the oracle; returns the final planes (1 or 3).
    refs: the seven reference pictures of an inter frame, (planes, w, h) each (None: unused)."""
    o = _bind(oracle_lib.load_oracle())
    # super-resolution: every picture has the upscaled geometry (the coded width is a prefix)
    pics = [alloc_picture(fr.up_w, fr.h, fr.bpc, fr.layout) for _ in range(3)]
    for p in pics:
        while len(p) < 3:
            p.append(p[0])
    arr = [(ctypes.c_void_p * 3)(*[a.ctypes.data for a in p]) for p in pics]
    st = (ctypes.c_ssize_t * 3)(*[a.strides[0] for a in pics[0]])
    out = (ctypes.c_void_p * 3)()
    rp = (ctypes.c_void_p * 21)()
    rs = (ctypes.c_ssize_t * 14)()
    rwh = (ctypes.c_int * 14)()
    for i, r in enumerate(refs or []):
        if r is None:
            continue
        planes, w, h = r
        for p in range(3):
            a = planes[p] if p < len(planes) else planes[0]
            rp[i * 3 + p] = a.ctypes.data
        rs[i * 2] = planes[0].strides[0]
        rs[i * 2 + 1] = (planes[1] if len(planes) > 1 else planes[0]).strides[0]
        rwh[i * 2], rwh[i * 2 + 1] = w, h
    o.oracle_decode_frame_refs(ctypes.byref(fr), arr[0], arr[1], arr[2], st, rp, rs, rwh, out)
    by_addr = {a.ctypes.data: a for p in pics for a in p}
    n = 3 if fr.layout else 1
    return [by_addr[out[i]] for i in range(n)]


def decode_stream(data, recon=oracle_frame, max_frames=None, threads=1, apply_grain=False, inloop_filters=14,
                  hash_output=True):
    """Decode an IVF stream; returns (md5 hex, frames output). `recon(frame, refs) -> planes` runs
    the pixel path (refs: the reference pictures, (planes, w, h) or None, in ref_pic order).
    apply_grain: the reference CLI's --filmgrain 1 (Dav1dSettings.apply_grain, src/lib.rs): shown
    pictures that carry grain get it (the oracle's rav1d_apply_grain) before hashing (oracle by default; the GPU path in the -m gpu tests). threads > 1: the
    front-end's frame threads (mi_dec_set_threads). inloop_filters: Dav1dSettings.inloop_filters
    (mi_dec_set_inloop_filters). hash_output=False: no hashing (returns (None, frames)), the
    reference CLI's --muxer null."""
    from rav1d_amd.av1dec import stream_events
    from rav1d_amd.output import Muxer, host_picture_np
    pics = {}
    md5 = hashlib.md5()
    mux = Muxer("md5")           # the product md5 muxer (libmi_av1dec.so), checked against hashlib
    shown = 0
    for ev in stream_events(data, threads, inloop_filters=inloop_filters):
        if ev.frame:
            fr = ev.frame.contents
            refs = [None] * 7
            for i in range(7):
                r = ev.ref_pic[i]
                if r >= 0:
                    planes, w, h = pics[r][0], pics[r][1], pics[r][2]
                    refs[i] = (planes, w, h)
            pics[ev.pic_id] = (recon(fr, refs), fr.up_w, fr.h, fr.layout, fr.bpc)
        if ev.show_pic >= 0:
            planes, w, h, layout, bpc = pics[ev.show_pic]
            if apply_grain and ev.fg_present:
                planes = oracle_lib.film_grain(planes, bpc, layout, w, h, ev.fg, ev.mtrx_identity)
            if hash_output:
                md5_update_picture(md5, planes, w, h, layout)
                mux.write(host_picture_np(planes, w, h, bpc, layout))
            shown += 1
        for i in range(ev.n_release):
            pics.pop(ev.release[i], None)
        if max_frames and shown >= max_frames:
            break
    digest = mux.digest()
    mux.close()
    if not hash_output:
        return None, shown
    if shown:
        assert digest == md5.hexdigest(), "md5 muxer disagrees with hashlib"
    return digest if shown else md5.hexdigest(), shown
