"""GPU parity: batched intra prediction (mi_ipred_blocks) and the table-compatible per-call
entry (mi_dsp_intra_pred) vs the oracle's restatement of ipred_tmpl.c — every mode, block
size, directional angle with and without edge filtering / upsampling, CfL and palette, at
8/10/12 bits, bit-exact."""
import ctypes

import numpy as np
import pytest
import torch

from rav1d_amd import IPRED_CFL, IPRED_PAL, lib
from rav1d_amd.frame import Frame, _stream_ptr
from rav1d_amd.ipred_synth import make_ipred_blocks
from tests import oracle_lib

pytestmark = pytest.mark.gpu


def oracle_block(b, edges, ac, idx, bpc):
    w, h, mode, t = int(b["w"]), int(b["h"]), int(b["mode"]), int(b["edge_off"])
    if mode >= IPRED_PAL:
        return oracle_lib.pal_pred(edges[t:t + 8], idx[b["aux_off"]:b["aux_off"] + w * h], w, h, bpc)
    if mode >= IPRED_CFL:
        return oracle_lib.cfl_pred(mode - IPRED_CFL, edges, t, w, h, ac[b["aux_off"]:b["aux_off"] + w * h],
                                   int(b["alpha"]), bpc)
    return oracle_lib.intra_pred(mode, edges, t, w, h, int(b["angle"]), int(b["max_w"]), int(b["max_h"]), bpc)


def run_batch(gpu, n, bpc, seed, modes=None):
    rng = np.random.default_rng(seed)
    blocks, edges, ac, idx, rows = make_ipred_blocks(n, bpc, rng, modes=modes)
    f = Frame(4096, rows, bpc, 0)
    db = torch.from_numpy(blocks.view(np.uint8).copy()).cuda()
    de = torch.from_numpy(edges.view(np.uint8).copy()).cuda()
    da = torch.from_numpy(ac.copy()).cuda()
    di = torch.from_numpy(idx.copy()).cuda()
    rc = lib().mi_ipred_blocks(gpu.h, ctypes.byref(f.picture()), ctypes.c_void_p(db.data_ptr()), len(blocks),
                               ctypes.c_void_p(de.data_ptr()), ctypes.c_void_p(da.data_ptr()),
                               ctypes.c_void_p(di.data_ptr()), _stream_ptr(None))
    assert rc == 0
    torch.cuda.synchronize()
    out = f.plane_np(0)
    for k, b in enumerate(blocks):
        x, y, w, h = int(b["x"]), int(b["y"]), int(b["w"]), int(b["h"])
        exp = oracle_block(b, edges, ac, idx, bpc)
        got = out[y:y + h, x:x + w]
        assert np.array_equal(got, exp), f"block {k}: mode {b['mode']} {w}x{h} angle {b['angle']:#x}"


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_ipred_batch_all_modes(gpu, bpc):
    run_batch(gpu, 1500, bpc, seed=bpc)


@pytest.mark.parametrize("mode", [6, 7, 8, 13])
def test_ipred_batch_directional_and_filter(gpu, mode):
    run_batch(gpu, 800, 10, seed=100 + mode, modes=[mode])


@pytest.mark.parametrize("bpc", [8, 10])
def test_dsp_intra_pred_percall_host_pointers(gpu, bpc):
    rng = np.random.default_rng(7 + bpc)
    dt = np.uint8 if bpc == 8 else np.uint16
    for _ in range(60):
        mode = int(rng.integers(0, 14))
        w, h = [(4, 4), (8, 8), (16, 8), (8, 32), (32, 32), (64, 16)][int(rng.integers(0, 6))]
        if mode == 13:
            w, h = min(w, 32), min(h, 32)
        angle = 0
        if mode in (6, 7, 8):
            from rav1d_amd.ipred_synth import random_angle
            angle = random_angle(rng, mode) | (1 << 10)
        elif mode == 13:
            angle = int(rng.integers(0, 5))
        e = rng.integers(0, 1 << bpc, size=261).astype(dt)
        dst = np.zeros((h, 80), dt)
        rc = lib().mi_dsp_intra_pred(mode, ctypes.c_void_p(dst.ctypes.data), dst.strides[0],
                                     ctypes.c_void_p(e.ctypes.data + 130 * e.itemsize), w, h, angle, w, h,
                                     (1 << bpc) - 1)
        assert rc == 0
        exp = oracle_lib.intra_pred(mode, e, 130, w, h, angle, w, h, bpc)
        assert np.array_equal(dst[:, :w], exp), (mode, w, h, angle)
        assert not dst[:, w:].any(), "wrote outside the block"
