"""Malformed device descriptors never fault: the kernels skip records the reference could never
issue and the context reports -EINVAL (mi_ctx_device_status / mi_frame_end). The reference
fuzzes its decoder with tests/dav1d-test-data/oss-fuzz; here the descriptor layer is the
boundary, so its records are checked where they are consumed."""
import ctypes

import numpy as np
import pytest
import torch

from rav1d_amd import TXBLOCK_DTYPE, MiIntraFrame, lib
from rav1d_amd.frame import Frame

EINVAL = -22


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("bad", ["txtp", "outside", "wrong_size", "plane"])
def test_itx_frame_rejects_bad_blocks(gpu, bad):
    pic = Frame(64, 64, 10, 1)
    before = [pic.buffer_np(p) for p in range(3)]
    blk = np.zeros(2, TXBLOCK_DTYPE)
    blk["tx"], blk["eob"], blk["x"] = 1, 5, [0, 8]      # two 8x8 DCT_DCT blocks
    coef = np.zeros(2 * 64, np.int32)
    coef[0], coef[64] = 700, 700
    blk["coef_off"] = [0, 64]
    if bad == "txtp":
        blk["txtp"][1] = 16            # WHT on 8x8: no such itxfm_add slot
    elif bad == "outside":
        blk["x"][1] = 124              # 124 + 8 > the 128-px aligned plane
    elif bad == "wrong_size":
        blk["tx"][1] = 2               # a 16x16 record in the 8x8 group
    else:
        blk["plane"][1] = 3
    ss = (ctypes.c_uint32 * 20)(*([0, 0] + [2] * 18))   # both records in the 8x8 group
    d_blk, d_coef = _dev(blk), torch.from_numpy(coef).cuda()
    p = pic.picture()
    L = lib()
    assert L.mi_itx_frame(gpu.h, ctypes.byref(p), ctypes.c_void_p(d_blk.data_ptr()), ss,
                          ctypes.c_void_p(d_coef.data_ptr()), 0, None) == 0
    assert L.mi_ctx_device_status(gpu.h, None) == EINVAL
    assert L.mi_ctx_device_status(gpu.h, None) == 0          # reported once
    after = pic.buffer_np(0)
    assert np.any(after[:8, :8] != before[0][:8, :8])         # the valid block was applied
    if bad != "outside":
        assert np.array_equal(after[:, 8:], before[0][:, 8:])  # the rejected one wrote nothing


@pytest.mark.gpu
def test_intra_recon_rejects_bad_blocks(gpu):
    pic = Frame(64, 64, 8, 1)
    blk = np.zeros(3, dtype=[("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"), ("plane", "u1"),
                             ("mode", "u1"), ("angle", "i1"), ("flags", "u1"), ("filt_idx", "u1"),
                             ("alpha", "i1"), ("tile_w", "<u2"), ("tile_h", "<u2"), ("max_w", "<u2"),
                             ("max_h", "<u2"), ("aux_off", "<u4"), ("pal_off", "<u4"), ("reserved", "<u4")])
    blk["w"], blk["h"], blk["x"] = 4, 4, [0, 4, 8]
    blk["tile_w"], blk["tile_h"], blk["max_w"], blk["max_h"] = 64, 64, 64, 64
    blk["x"][1] = 200                   # outside the picture
    blk["flags"][2] = 1                 # block 2 reads block 1's column: must not hang
    tx = np.zeros(3, TXBLOCK_DTYPE)
    tx["x"], tx["eob"] = blk["x"], -1
    d_blk, d_tx = _dev(blk), _dev(tx)
    d_ds, d_deps = _dev(np.array([0, 0, 0, 1], np.int32)), _dev(np.array([1], np.int32))
    d_coef = torch.zeros(64, dtype=torch.int16, device="cuda")
    d = MiIntraFrame()
    d.pic = pic.picture()
    d.blocks, d.tx, d.dep_start, d.deps = (t.data_ptr() for t in (d_blk, d_tx, d_ds, d_deps))
    d.coef, d.n = d_coef.data_ptr(), 3
    L = lib()
    assert L.mi_intra_recon(gpu.h, ctypes.byref(d), 1, 0, None) == 0
    assert L.mi_frame_end(gpu.h, None) == EINVAL
    assert L.mi_frame_end(gpu.h, None) == 0
