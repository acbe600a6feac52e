"""The frame executor's host-side checks (mi_frame_validate, the validation mi_frame_run runs
before enqueuing anything) accept every frame the front-end emits for the reference vectors,
and reject malformed inter descriptors. CPU only: no device call is made."""
import ctypes
import json
import os

import numpy as np
import pytest

from rav1d_amd import MCBLOCK_DTYPE, MiFramePictures, MiPicture, lib
from rav1d_amd.av1dec import MiDecFrame, stream_events
from rav1d_amd.frame import plane_geometry

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "streams")
VECTORS = json.load(open(os.path.join(GOLDEN, "vectors.json")))


def fake_picture(w, h, bpc, layout, base):
    """A picture descriptor with the default allocator's geometry and dummy plane addresses
    (the checks never dereference them)."""
    (_, ys), (_, cs), _ = plane_geometry(w, h, layout, bpc)
    p = MiPicture()
    for k in range(3):
        p.data[k] = base + k * 0x100000
    p.stride[0], p.stride[1] = ys, cs
    p.w, p.h, p.layout, p.bpc = w, h, layout, bpc
    return p


def frames_with_pictures(data, threads=1):
    """(MiDecFrame copy, MiFramePictures) of every frame of a stream, refs filled. threads > 1:
    the front-end's frame and tile threads (work lists merged from the tiles' decoders)."""
    geo = {}
    for ev in stream_events(data, threads):
        if not ev.frame:
            continue
        fr = MiDecFrame.from_buffer_copy(ev.frame.contents)
        ps = MiFramePictures()
        for k in range(4):
            ps.pics[k] = fake_picture(fr.up_w, fr.h, fr.bpc, fr.layout, 0x10000000 * (k + 1))
        for i in range(7):
            r = ev.ref_pic[i]
            if r >= 0 and r in geo:
                ps.refs[i] = fake_picture(*geo[r], 0x70000000 + r * 0x1000000)
        geo[ev.pic_id] = (fr.up_w, fr.h, fr.bpc, fr.layout)
        yield fr, ps, ev


def validate(fr, ps):
    why = ctypes.c_char_p()
    rc = lib().mi_frame_validate(ctypes.byref(fr), ctypes.byref(ps), ctypes.byref(why))
    return rc, (why.value or b"").decode()


@pytest.mark.parametrize("threads", [1, 8], ids=["t1", "t8"])
@pytest.mark.parametrize("v", VECTORS, ids=[v["name"] for v in VECTORS])
def test_front_end_frames_validate(v, threads):
    data = open(os.path.join(GOLDEN, v["file"]), "rb").read()
    n = 0
    for fr, ps, _ in frames_with_pictures(data, threads):
        rc, why = validate(fr, ps)
        assert rc == 0, f"{v['name']} frame {n}: rejected by {why}"
        n += 1
    assert n > 0


@pytest.mark.parametrize("name", ["av1-1-b8-02-allintra", "00001138"])
def test_front_end_intra_queue(name):
    """The front-end's intra queue (MiDecFrame.q_*) is a permutation of the decode-order blocks,
    its dependencies lie inside it, its strips partition it; without it the frame still
    validates (mi_frame_run plans), and a queue dependency out of range is rejected."""
    v = next(x for x in VECTORS if x["name"] == name)
    data = open(os.path.join(GOLDEN, v["file"]), "rb").read()
    checked = 0
    for fr, ps, _ in frames_with_pictures(data, 4):
        n = fr.n_intra
        if n == 0:
            continue
        assert fr.q_intra and fr.q_dep_start
        blk = np.ctypeslib.as_array((ctypes.c_uint8 * (32 * n)).from_address(fr.intra)).reshape(n, 32)
        qb = np.ctypeslib.as_array((ctypes.c_uint8 * (32 * n)).from_address(fr.q_intra)).reshape(n, 32)
        key = lambda a: sorted(map(bytes, a))
        assert key(blk) == key(qb)
        ds = np.ctypeslib.as_array((ctypes.c_int32 * (n + 1)).from_address(fr.q_dep_start))
        assert ds[0] == 0 and ds[-1] == fr.q_n_deps and (np.diff(ds) >= 0).all()
        ss = None
        if fr.q_nstrips > 1:
            ss = np.ctypeslib.as_array((ctypes.c_int32 * (fr.q_nstrips + 1)).from_address(fr.q_strip_start))
            assert ss[0] == 0 and ss[-1] == n and (np.diff(ss) >= 0).all()
        assert validate(fr, ps)[0] == 0
        c = MiDecFrame.from_buffer_copy(fr)
        c.q_intra = None
        assert validate(c, ps)[0] == 0
        if fr.q_n_deps:
            deps = (ctypes.c_int32 * fr.q_n_deps)()
            ctypes.memmove(deps, fr.q_deps, 4 * fr.q_n_deps)
            deps[0] = n
            c = MiDecFrame.from_buffer_copy(fr)
            c.q_deps = ctypes.addressof(deps)
            rc, why = validate(c, ps)
            assert rc != 0 and why
            # a dependency on a later entry of the same strip (its workers take entries in order)
            i = next(i for i in range(n) if ds[i + 1] > ds[i])
            end = n
            if fr.q_nstrips > 1:
                end = next(int(x) for x in ss[1:] if x > i)
            if i + 1 < end:
                ctypes.memmove(deps, fr.q_deps, 4 * fr.q_n_deps)
                deps[ds[i]] = i + 1
                rc, why = validate(c, ps)
                assert rc != 0 and why
        checked += 1
    assert checked > 0


def test_malformed_inter_units_are_rejected():
    v = next(x for x in VECTORS if x["name"] == "00000706")
    data = open(os.path.join(GOLDEN, v["file"]), "rb").read()
    gen = frames_with_pictures(data)      # kept alive: the frame's arrays belong to its decoder
    fr, ps = next((f, p) for f, p, _ in gen if f.n_mc > 4)
    assert validate(fr, ps)[0] == 0
    units = np.frombuffer(ctypes.string_at(fr.mc, 24 * fr.n_mc), MCBLOCK_DTYPE).copy()

    def with_units(mod):
        u = units.copy()
        mod(u)
        bad = MiDecFrame.from_buffer_copy(fr)
        keep = np.ascontiguousarray(u)
        bad.mc = keep.ctypes.data
        return validate(bad, ps)[0], keep

    def ref9(u): u["ref"][0, 0] = 9
    def w24(u): u["w"][0] = 24
    def far(u): u["x"][0] = 60000
    def filt(u): u["filter2d"][0] = 12
    def mask(u): u["comp"][0], u["ref"][0], u["mask_off"][0] = 2, (0, 1), fr.nmasks + 1
    def prep(u): u["comp"][0], u["ref"][0], u["mask_off"][0] = 6, (0, -1), fr.ntmp + 1
    cases = {"ref out of range": ref9, "width not a power of two": w24, "outside the plane": far,
             "bad filter": filt, "mask past the arena": mask, "prep past the tmp arena": prep}
    for what, mod in cases.items():
        rc, _ = with_units(mod)
        assert rc == -22, what
    # a missing reference picture for a unit's reference
    ps2 = MiFramePictures.from_buffer_copy(ps)
    r = int(units["ref"][0, 0])
    ps2.refs[r] = MiPicture()
    assert validate(fr, ps2)[0] == -22
    del gen
