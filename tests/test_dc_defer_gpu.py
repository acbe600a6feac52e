"""GPU parity: DC-only residuals deferred into the deblocking pass.

mi_itx_frame_runs(MI_ITX_DC_DEFER) records each DC-only block's constant in the context's DC
map instead of adding it; mi_deblock_frame_dc adds it to the pixels it stages. The deblocked
picture must equal the one of the plain order (itx adds every residual, then deblock), which the
oracle's itx_frame + deblock_frame produce (rav1d src/itx.rs:64-188 dc_only path, then
src/lf_apply.rs:597-834)."""
import ctypes

import numpy as np
import pytest
import torch

from rav1d_amd import ITX_DC_DEFER, ITX_KEEP_COEFS, lib
from rav1d_amd.frame import Frame, LoopFilterMeta, _stream_ptr
from rav1d_amd.synth import itx_band_order, itx_dc_runs, make_frame
from tests import oracle_lib
from tests.pipeline import pad_planes

pytestmark = pytest.mark.gpu


def _inputs(w, h, bpc, layout, seed):
    fr = make_frame(w, h, bpc, layout, seed=seed, with_fg=False)
    ah = (h + 127) & ~127
    ssv = 1 if layout == 1 else 0
    blk, _, bs = itx_band_order(fr["blocks"], [ah, ah >> ssv, ah >> ssv])
    de = itx_dc_runs(blk, bs)
    return fr, blk, bs, de


def _run(gpu, fr, blk, bs, de, defer, filter_y=None, dst_same=False):
    w, h, bpc, layout = fr["w"], fr["h"], fr["bpc"], fr["layout"]
    A = Frame(w, h, bpc, layout)
    for p, a in enumerate(fr["planes"]):
        A.set_plane_np(p, a)
    D = A if dst_same else Frame(w, h, bpc, layout)
    blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
    coef = torch.from_numpy(fr["coef"].copy()).cuda()
    lf = LoopFilterMeta(fr["lf"])
    if filter_y is not None:
        lf.s.filter_y = filter_y
    pa, pd = A.picture(), D.picture()
    bsa = (ctypes.c_uint32 * bs.size)(*[int(v) for v in bs.reshape(-1)])
    dea = (ctypes.c_uint32 * de.size)(*[int(v) for v in de.reshape(-1)])
    sp = _stream_ptr(None)
    L = lib()
    rc = L.mi_itx_frame_runs(gpu.h, ctypes.byref(pa), ctypes.c_void_p(blocks.data_ptr()), bsa, dea,
                             ctypes.c_void_p(coef.data_ptr()), ITX_KEEP_COEFS | (ITX_DC_DEFER if defer else 0), sp)
    assert rc == 0
    rc = L.mi_deblock_frame_dc(gpu.h, ctypes.byref(pa), ctypes.byref(pd), ctypes.byref(lf.s), sp)
    torch.cuda.synchronize()
    return rc, A, D


def _oracle(fr, deblock=True):
    """the plain order on the CPU, as tests/pipeline.py's oracle_pipeline: itx, then deblock"""
    w, h, bpc, layout = fr["w"], fr["h"], fr["bpc"], fr["layout"]
    A = oracle_lib.itx_frame(pad_planes(fr["planes"], w, h, bpc, layout), fr["blocks"], fr["coef"].copy(), bpc)
    return oracle_lib.deblock_frame(A, bpc, layout, w, h, fr["lf"], sb128=1) if deblock else A


@pytest.mark.parametrize("geom", [(256, 192, 8, 1), (640, 360, 10, 1), (352, 288, 12, 3), (720, 486, 10, 2),
                                  (200, 136, 10, 0), (1920, 1080, 10, 1)])
def test_deferred_dc_matches_oracle(gpu, geom):
    w, h, bpc, layout = geom
    fr, blk, bs, de = _inputs(w, h, bpc, layout, seed=w * 3 + bpc)
    assert (de > bs[:, :-1]).any(), "the frame must hold DC runs"
    rc, A, D = _run(gpu, fr, blk, bs, de, defer=True)
    assert rc == 0
    ref = _oracle(fr)
    for p in range(3 if layout else 1):
        got = D.plane_np(p)
        ph, pw = got.shape
        assert np.array_equal(got, ref[p][:ph, :pw]), f"plane {p}"


def test_deferred_dc_equals_plain_order_at_4k10(gpu):
    fr, blk, bs, de = _inputs(3840, 2160, 10, 1, seed=0x4C100001)
    rc, _, d_defer = _run(gpu, fr, blk, bs, de, defer=True)
    assert rc == 0
    rc, _, d_plain = _run(gpu, fr, blk, bs, de, defer=False)
    assert rc == 0
    for p in range(3):
        assert np.array_equal(d_defer.plane_np(p), d_plain.plane_np(p)), p


def test_deferred_dc_with_deblocking_off(gpu):
    # filter_y 0: the output is the reconstruction with the DC added, nothing filtered
    fr, blk, bs, de = _inputs(640, 360, 10, 1, seed=5)
    rc, _, D = _run(gpu, fr, blk, bs, de, defer=True, filter_y=0)
    assert rc == 0
    ref = _oracle(fr, deblock=False)
    for p in range(3):
        got = D.plane_np(p)
        ph, pw = got.shape
        assert np.array_equal(got, ref[p][:ph, :pw]), p


def test_deferred_dc_rejects_in_place_and_other_geometry(gpu):
    fr, blk, bs, de = _inputs(256, 192, 10, 1, seed=6)
    rc, _, _ = _run(gpu, fr, blk, bs, de, defer=True, dst_same=True)
    assert rc == -22
    # a pending deferral is consumed by the next deblock call; a picture of another size is refused
    rc, A, _ = _run(gpu, fr, blk, bs, de, defer=False)
    assert rc == 0
    other = Frame(320, 192, 10, 1)
    blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
    coef = torch.from_numpy(fr["coef"].copy()).cuda()
    pa = A.picture()
    L = lib()
    assert L.mi_itx_frame_runs(gpu.h, ctypes.byref(pa), ctypes.c_void_p(blocks.data_ptr()),
                               (ctypes.c_uint32 * bs.size)(*[int(v) for v in bs.reshape(-1)]),
                               (ctypes.c_uint32 * de.size)(*[int(v) for v in de.reshape(-1)]),
                               ctypes.c_void_p(coef.data_ptr()), ITX_KEEP_COEFS | ITX_DC_DEFER, _stream_ptr(None)) == 0
    lf = LoopFilterMeta(fr["lf"])
    po, pd = other.picture(), Frame(320, 192, 10, 1).picture()
    assert L.mi_deblock_frame_dc(gpu.h, ctypes.byref(po), ctypes.byref(pd), ctypes.byref(lf.s), _stream_ptr(None)) == -22
    # the DEFER flag needs the runs table
    ss = (ctypes.c_uint32 * 20)(*[0] * 20)
    assert L.mi_itx_frame(gpu.h, ctypes.byref(pa), ctypes.c_void_p(blocks.data_ptr()), ss,
                          ctypes.c_void_p(coef.data_ptr()), ITX_DC_DEFER, _stream_ptr(None)) == -22


def test_deferred_dc_under_graph_capture(gpu):
    # captured, the deferral is not taken (a tag fixed in the graph could match a previous
    # replay's entries): replaying the graph gives the plain order's picture
    fr, blk, bs, de = _inputs(640, 360, 10, 1, seed=8)
    w, h = 640, 360
    A, D = Frame(w, h, 10, 1), Frame(w, h, 10, 1)
    blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
    coef = torch.from_numpy(fr["coef"].copy()).cuda()
    lf = LoopFilterMeta(fr["lf"])
    pa, pd = A.picture(), D.picture()
    bsa = (ctypes.c_uint32 * bs.size)(*[int(v) for v in bs.reshape(-1)])
    dea = (ctypes.c_uint32 * de.size)(*[int(v) for v in de.reshape(-1)])
    L = lib()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        assert L.mi_itx_frame_runs(gpu.h, ctypes.byref(pa), ctypes.c_void_p(blocks.data_ptr()), bsa, dea,
                                   ctypes.c_void_p(coef.data_ptr()), ITX_KEEP_COEFS | ITX_DC_DEFER, _stream_ptr(s)) == 0
        assert L.mi_deblock_frame_dc(gpu.h, ctypes.byref(pa), ctypes.byref(pd), ctypes.byref(lf.s), _stream_ptr(s)) == 0
    for p, a in enumerate(fr["planes"]):
        A.set_plane_np(p, a)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    ref = _oracle(fr)
    for p in range(3):
        got = D.plane_np(p)
        ph, pw = got.shape
        assert np.array_equal(got, ref[p][:ph, :pw]), p
