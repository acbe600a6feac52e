"""Reference MD5 vectors decoded on the MI355X: front-end work lists executed by
librav1d_amd.so's frame executor (mi_frame_run: inter prediction -- MC, OBMC, warp, scaled
references, compound masks -- and inter residuals, persistent intra reconstruction incl.
inter-intra, deblocking, CDEF, loop restoration; film grain at output for the --filmgrain 1
vectors), shown pictures hashed as the md5 muxer does
(tools/output/md5.rs:541-637). Expected MD5s are the reference's (tests/golden/streams)."""
import hashlib
import json
import os

import numpy as np
import pytest

from tests.stream_lib import md5_update_picture

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "streams")
VECTORS = json.load(open(os.path.join(GOLDEN, "vectors.json")))


def _without_queue(fr):
    """A copy of a MiDecFrame without the front-end's intra queue: mi_frame_run plans it."""
    from rav1d_amd.av1dec import MiDecFrame
    c = MiDecFrame.from_buffer_copy(fr)
    c.q_intra = c.q_intra_tx = c.q_dep_start = c.q_deps = c.q_strip_start = None
    c.q_n_deps = c.q_nstrips = c.q_granules = 0
    return c


def gpu_md5(ctx, data, threads=1, plan="front-end", monkeypatch=None):
    from rav1d_amd import stream as S
    if plan == "executor":
        run = S.run_frame
        monkeypatch.setattr(S, "run_frame", lambda c, fr, *a, **k: run(c, _without_queue(fr), *a, **k))
    md5 = hashlib.md5()
    n = 0
    for pic in S.decode_ivf(ctx, data, threads=threads):
        planes = [pic.buffer_np(p) for p in range(len(pic.planes))]
        md5_update_picture(md5, planes, pic.w, pic.h, pic.layout)
        n += 1
    return md5.hexdigest(), n


@pytest.mark.gpu
@pytest.mark.parametrize("threads,plan", [(1, "front-end"), (1, "executor"), (8, "front-end")],
                         ids=["t1", "t1-own-plan", "t8"])
@pytest.mark.parametrize("v", VECTORS, ids=[v["name"] for v in VECTORS])
def test_gpu_decode_matches_reference_md5(gpu, v, threads, plan, monkeypatch):
    """threads 8: the work lists of the front-end's tile decoders (merged in tile order, intra
    dependencies inside each tile) and frame threads, through the device. The intra queue is
    the front-end's (MiDecFrame.q_*, planned on its frame threads) or, own-plan, the one
    mi_frame_run plans itself from the decode-order lists."""
    data = open(os.path.join(GOLDEN, v["file"]), "rb").read()
    if v.get("filmgrain") and (threads > 1 or plan != "front-end"):
        pytest.skip("grain vectors: covered at threads 1 (the grain path does not depend on the work lists)")
    if v.get("filmgrain"):
        # --filmgrain 1: the grain is applied on the device as the picture is output
        from rav1d_amd.output import Muxer
        from rav1d_amd.stream import decode_to_muxer
        m = Muxer("md5")
        n = decode_to_muxer(gpu, data, m, apply_grain=True, pipelined=False)
        md5 = m.digest()
        m.close()
    else:
        md5, n = gpu_md5(gpu, data, threads, plan, monkeypatch)
    assert n > 0
    assert md5 == v["md5"], f"{v['name']}: {n} frames, md5 {md5} != {v['md5']}"


@pytest.mark.gpu
def test_frame_run_rejects_malformed_work_lists(gpu):
    """Bad descriptors return -EINVAL before any device work (never a fault)."""
    import ctypes

    from rav1d_amd import lib
    from rav1d_amd.av1dec import Av1Decoder, ivf_frames
    from rav1d_amd.stream import DevicePictureSet
    v = next(x for x in VECTORS if x["name"] == "issue_320")
    dec = Av1Decoder()
    data = open(os.path.join(GOLDEN, v["file"]), "rb").read()
    for tu in ivf_frames(data):
        dec.send(tu)
        evs = [e for e in dec.events() if e.frame]
        if evs:
            break
    fr = evs[0].frame.contents
    ps = DevicePictureSet(fr.w, fr.h, fr.bpc, fr.layout)
    final = ctypes.c_int()
    L = lib()
    assert L.mi_frame_run(gpu.h, ctypes.byref(fr), ctypes.byref(ps.pics), ctypes.byref(final), None) == 0
    assert L.mi_frame_end(gpu.h, None) == 0
    from rav1d_amd import MiIntraFrame  # noqa: F401  (struct mirrors loaded)
    from rav1d_amd.av1dec import MiDecFrame
    n = fr.n_intra
    blocks = (ctypes.c_uint8 * (32 * n)).from_address(fr.intra)
    txs = (ctypes.c_uint8 * (16 * n)).from_address(fr.intra_tx)
    cases = []
    # a block outside the picture
    b = bytearray(blocks)
    b[0:2] = (4000).to_bytes(2, "little")
    cases.append(("x", b, bytes(txs)))
    # an illegal transform type (17: past WHT_WHT)
    t = bytearray(txs)
    k = 0
    t[16 * k + 10] = 17
    t[16 * k + 12:16 * k + 16] = (1).to_bytes(4, "little", signed=True)
    cases.append(("txtp", bytes(blocks), t))
    # a coefficient offset past the arena
    t = bytearray(txs)
    k = next(i for i in range(n) if int.from_bytes(bytes(txs[16 * i + 12:16 * i + 16]), "little", signed=True) >= 0)
    t[16 * k:16 * k + 4] = (fr.ncoef + 10).to_bytes(4, "little")
    cases.append(("coef_off", bytes(blocks), t))
    # the same corruptions in the front-end's queue (the arrays the kernels read when it is given)
    qb = (ctypes.c_uint8 * (32 * n)).from_address(fr.q_intra)
    qt = (ctypes.c_uint8 * (16 * n)).from_address(fr.q_intra_tx)
    b = bytearray(qb)
    b[0:2] = (4000).to_bytes(2, "little")
    cases.append(("queue x", b, bytes(qt), "q"))
    t = bytearray(qt)
    k = next(i for i in range(n) if int.from_bytes(bytes(qt[16 * i + 12:16 * i + 16]), "little", signed=True) >= 0)
    t[16 * k:16 * k + 4] = (fr.ncoef + 10).to_bytes(4, "little")
    cases.append(("queue coef_off", bytes(qb), t, "q"))
    for what, bb, tt, *kind in cases:
        bad = MiDecFrame.from_buffer_copy(fr)
        bbuf = (ctypes.c_uint8 * len(bb)).from_buffer_copy(bytes(bb))
        tbuf = (ctypes.c_uint8 * len(tt)).from_buffer_copy(bytes(tt))
        if kind:
            bad.q_intra = ctypes.addressof(bbuf)
            bad.q_intra_tx = ctypes.addressof(tbuf)
        else:
            # decode-order lists: without a queue, mi_frame_run plans (and checks) them itself
            bad.intra = ctypes.addressof(bbuf)
            bad.intra_tx = ctypes.addressof(tbuf)
            bad.q_intra = bad.q_intra_tx = bad.q_dep_start = bad.q_deps = bad.q_strip_start = None
            bad.q_n_deps = bad.q_nstrips = bad.q_granules = 0
        assert isinstance(bad, MiDecFrame)
        assert L.mi_frame_run(gpu.h, ctypes.byref(bad), ctypes.byref(ps.pics), ctypes.byref(final), None) == -22, what
    assert L.mi_frame_end(gpu.h, None) == 0
    assert np.any(ps.output().buffer_np(0))


@pytest.mark.gpu
def test_unsatisfiable_dependency_reports_eio(gpu):
    """A work list whose dependency can never be met (two blocks waiting on each other) must end
    in -EIO from mi_frame_end — the kernel's bounded wait gives up and the frame is reported as
    failed, never silently returned."""
    import ctypes

    import torch

    from rav1d_amd import TXBLOCK_DTYPE, MiIntraFrame, lib
    from rav1d_amd.frame import Frame
    pic = Frame(64, 64, 8, 1)
    blk = np.zeros(2, dtype=[("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"), ("plane", "u1"),
                             ("mode", "u1"), ("angle", "i1"), ("flags", "u1"), ("filt_idx", "u1"),
                             ("alpha", "i1"), ("tile_w", "<u2"), ("tile_h", "<u2"), ("max_w", "<u2"),
                             ("max_h", "<u2"), ("aux_off", "<u4"), ("pal_off", "<u4"), ("reserved", "<u4")])
    assert blk.dtype.itemsize == 32
    blk["w"], blk["h"], blk["x"], blk["mode"] = 4, 4, [4, 0], 0
    blk["tile_w"], blk["tile_h"], blk["max_w"], blk["max_h"] = 64, 64, 64, 64
    blk["flags"] = [1, 0]   # block 0 has a left neighbour
    tx = np.zeros(2, TXBLOCK_DTYPE)
    tx["x"], tx["eob"] = [4, 0], -1
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()  # noqa: E731
    d_blk, d_tx = dev(blk), dev(tx)
    d_ds = dev(np.array([0, 1, 2], np.int32))
    d_deps = dev(np.array([1, 0], np.int32))    # 0 waits for 1, 1 waits for 0
    d_coef = torch.zeros(64, dtype=torch.int16, device="cuda")
    d = MiIntraFrame()
    d.pic = pic.picture()
    d.blocks, d.tx, d.dep_start, d.deps = (t.data_ptr() for t in (d_blk, d_tx, d_ds, d_deps))
    d.coef, d.n = d_coef.data_ptr(), 2
    L = lib()
    assert L.mi_intra_recon(gpu.h, ctypes.byref(d), 1, 0, None) == 0
    assert L.mi_frame_end(gpu.h, None) == -5   # -EIO
    assert L.mi_frame_end(gpu.h, None) == 0    # reported once


def _superres_frames(name, n_frames, up_num, up_den, keep_lr):
    """Front-end frames of an intra vector turned into super-resolution frames: the coded
    width stays, up_w = w * up_num / up_den (a width the frame header could carry, denominator
    9..16 over 8), and the loop-restoration units are re-laid over the upscaled width (unit x
    clamped into the coded frame's units) or switched off. Yields (frame, keepalive)."""
    import ctypes

    from rav1d_amd.av1dec import Av1Decoder, MiDecFrame, ivf_frames
    v = next(x for x in VECTORS if x["name"] == name)
    dec = Av1Decoder()
    got = 0
    for tu in ivf_frames(open(os.path.join(GOLDEN, v["file"]), "rb").read()):
        dec.send(tu)
        for ev in dec.events():
            if not ev.frame or got >= n_frames:
                continue
            src = ev.frame.contents
            fr = MiDecFrame.from_buffer_copy(src)
            fr.up_w = src.w * up_num // up_den
            keep = []
            if keep_lr and src.restore_planes:
                old = np.frombuffer((ctypes.c_uint8 * (108 * src.sb128h * src.lr_sb128w)).from_address(src.lr_mask),
                                    np.uint8).reshape(src.sb128h, src.lr_sb128w, 108)
                nw = (fr.up_w + 127) >> 7
                cols = np.minimum(np.arange(nw) * src.lr_sb128w // nw, src.lr_sb128w - 1)
                new = np.ascontiguousarray(old[:, cols])
                keep.append(new)
                fr.lr_mask, fr.lr_sb128w = new.ctypes.data, nw
            else:
                fr.restore_planes = 0
            got += 1
            yield fr, (keep, ev)


@pytest.mark.gpu
@pytest.mark.parametrize("keep_lr", [False, True])
def test_superres_frames_match_oracle(gpu, keep_lr):
    """Super-resolution through the frame executor (CDEF output upscaled by mi_superres_frame,
    then LR over the upscaled width reading the upscaled deblocked picture, recon.rs:4211-4283)
    equals the oracle's frame driver on the same work lists. No intra-only reference vector
    uses super-resolution, so the frames are the allintra vector's with a widened up_w: parity
    unpinned by reference outputs, pinned to the oracle (whose resize step follows
    decode.rs:4640-4660 / mc.rs resize)."""
    import torch

    from rav1d_amd.stream import run_frame
    from tests.stream_lib import oracle_frame
    for fr, _keep in _superres_frames("av1-1-b8-02-allintra", 3, 3, 2, keep_lr):
        ps = run_frame(gpu, fr)
        torch.cuda.synchronize()
        from rav1d_amd.stream import frame_end
        frame_end(gpu)
        want = oracle_frame(fr)
        out = ps.output()
        ss_h, ss_v = int(fr.layout in (1, 2)), int(fr.layout == 1)
        for p in range(len(want)):
            h = fr.h if p == 0 else (fr.h + ss_v) >> ss_v
            w = fr.up_w if p == 0 else (fr.up_w + ss_h) >> ss_h
            got = out.buffer_np(p)[:h, :w]
            assert np.array_equal(got, want[p][:h, :w]), f"plane {p} keep_lr={keep_lr}"


class _Collect:
    """A muxer that keeps a copy of every picture handed to it (host pictures, visible area)."""

    def __init__(self):
        self.frames = []

    def write(self, pic):
        from rav1d_amd.output import HostPicture
        h = HostPicture.__new__(HostPicture)
        h.pic = pic
        self.frames.append([h.plane_np(p) for p in range(3 if pic.layout else 1)])


def _oracle_frames(data):
    """Every shown picture of the oracle's decode (visible area per plane)."""
    from rav1d_amd.av1dec import stream_events
    from tests.stream_lib import oracle_frame
    pics, out = {}, []
    for ev in stream_events(data):
        if ev.frame:
            fr = ev.frame.contents
            refs = [None if r < 0 else pics[r][:3] for r in ev.ref_pic]
            pics[ev.pic_id] = (oracle_frame(fr, refs), fr.up_w, fr.h, fr.layout)
        if ev.show_pic >= 0:
            planes, w, h, lay = pics[ev.show_pic]
            ss_hor, ss_ver = int(lay in (1, 2)), int(lay == 1)
            dims = [(w, h)] + [((w + ss_hor) >> ss_hor, (h + ss_ver) >> ss_ver)] * 2
            out.append([planes[p][:dims[p][1], :dims[p][0]] for p in range(len(planes))])
        for i in range(ev.n_release):
            pics.pop(ev.release[i], None)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["av1-1-b8-02-allintra", "00000623"])
def test_two_device_lanes_match_oracle_per_frame(gpu, name):
    """Frames alternating over two (context, stream) lanes that overlap on the device (rav1d's
    frame threads, decode_to_muxer in_flight=2), each lane's context fresh so that its
    first-use initialisation happens while the other lane's work is queued: every shown picture
    equals the oracle's. Before the fix this failed in about one run in four: the contexts'
    device words were zeroed by a null-stream hipMemset, unordered with the lanes' non-blocking
    streams, and it could land in the middle of the other lane's persistent intra launch."""
    from rav1d_amd import stream as S
    from rav1d_amd.frame import Context
    data = open(os.path.join(GOLDEN, next(v for v in VECTORS if v["name"] == name)["file"]), "rb").read()
    want = _oracle_frames(data)
    for rep in range(2):
        S._extra_lanes.clear()                     # fresh contexts and streams for the extra lane
        m = _Collect()
        n = S.decode_to_muxer(Context(0), data, m, apply_grain=False, in_flight=2)
        assert n == len(want)
        for k, (got, exp) in enumerate(zip(m.frames, want)):
            for p in range(len(exp)):
                assert np.array_equal(got[p], exp[p]), f"{name} rep {rep} frame {k} plane {p}"
