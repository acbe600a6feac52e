"""GPU parity: whole-frame deblocking (all column edges, then all row edges) vs the oracle's
per-superblock-row traversal of the reference, bit-exact."""
import numpy as np
import pytest
import torch

from rav1d_amd.frame import Frame, LoopFilterMeta, deblock_frame
from tests import oracle_lib
from tests.test_oracle_lf import frame, pad_planes

pytestmark = pytest.mark.gpu


def run_gpu(gpu, planes, lf, w, h, bpc, layout, oop=False):
    f = Frame(w, h, bpc, layout)
    for p, a in enumerate(planes):
        f.set_plane_np(p, a)
    meta = LoopFilterMeta(lf)
    if oop:
        d = Frame(w, h, bpc, layout)
        for p in range(len(planes)):   # poison: every plane pixel must be written
            d.planes[p].fill_(0x5A)
        deblock_frame(gpu, f, meta, dst=d)
        torch.cuda.synchronize()
        src_after = [f.plane_np(p) for p in range(len(planes))]
        assert all(np.array_equal(s, a) for s, a in zip(src_after, planes)), "source written"
        return [d.plane_np(p) for p in range(len(planes))]
    deblock_frame(gpu, f, meta)
    torch.cuda.synchronize()
    return [f.plane_np(p) for p in range(len(planes))]


@pytest.mark.parametrize("oop", [False, True], ids=["inplace", "tiles"])
@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [1, 2, 3, 0])
@pytest.mark.parametrize("size", [(256, 192), (200, 136)])
def test_deblock_matches_oracle(gpu, bpc, layout, size, oop):
    w, h = size
    planes, lf = frame(w, h, bpc, layout, seed=bpc * 7 + layout)
    planes = planes[:1] if layout == 0 else planes
    got = run_gpu(gpu, planes, lf, w, h, bpc, layout, oop)
    ref = oracle_lib.deblock_frame(pad_planes(planes, w, h, bpc, layout), bpc, layout, w, h, lf,
                                   sb128=int(w == 256))
    for p in range(len(planes)):
        ph, pw = planes[p].shape
        assert np.array_equal(got[p], ref[p][:ph, :pw]), f"plane {p}"


@pytest.mark.parametrize("oop", [False, True], ids=["inplace", "tiles"])
@pytest.mark.parametrize("bpc", [8, 10])
def test_deblock_4k_matches_oracle(gpu, bpc, oop):
    w, h = 3840, 2160
    planes, lf = frame(w, h, bpc, 1, seed=0x4C100001)
    got = run_gpu(gpu, planes, lf, w, h, bpc, 1, oop)
    ref = oracle_lib.deblock_frame(pad_planes(planes, w, h, bpc, 1), bpc, 1, w, h, lf)
    for p in range(3):
        ph, pw = planes[p].shape
        assert np.array_equal(got[p], ref[p][:ph, :pw])
