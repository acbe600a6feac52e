"""GPU parity: whole-frame loop restoration (stripe x tile workgroups reading C and D) vs the
oracle's in-place unit/stripe algorithm with line buffer and column backups, bit-exact."""
import numpy as np
import pytest
import torch

from rav1d_amd.frame import Frame, LrMeta, lr_frame
from rav1d_amd.synth import make_lr_meta
from tests import oracle_lib
from tests.test_oracle_lf import pad_planes
from tests.test_oracle_lr import planes_for

pytestmark = pytest.mark.gpu


def to_frame(planes, w, h, bpc, layout):
    f = Frame(w, h, bpc, layout)
    for p, a in enumerate(planes):
        f.set_plane_np(p, a)
    return f


def run_case(gpu, w, h, bpc, layout, seed, sb128, unit_log2=None, ordered=False):
    rng = np.random.default_rng(seed)
    c = planes_for(w, h, bpc, layout, rng)
    d = planes_for(w, h, bpc, layout, rng)
    lr = make_lr_meta(w, h, layout, rng, sb128=sb128, unit_log2=unit_log2)
    fc, fd = to_frame(c, w, h, bpc, layout), to_frame(d, w, h, bpc, layout)
    fo = Frame(w, h, bpc, layout)
    lr_frame(gpu, fc, fd, fo, LrMeta(lr, geometry=(w, h, layout) if ordered else None))
    torch.cuda.synchronize()
    ref = oracle_lib.lr_frame(pad_planes(c, w, h, bpc, layout), pad_planes(d, w, h, bpc, layout),
                              bpc, layout, w, h, lr)
    for p in range(len(c)):
        ph, pw = c[p].shape
        assert np.array_equal(fo.plane_np(p), ref[p][:ph, :pw]), f"plane {p}"


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [1, 2, 3, 0])
@pytest.mark.parametrize("geom", [(256, 200, 1, None), (200, 150, 0, (6, 5)), (330, 260, 0, (7, 6))])
def test_lr_matches_oracle(gpu, bpc, layout, geom):
    w, h, sb128, ul = geom
    if ul is not None and layout != 1:
        ul = (ul[0], ul[0])
    run_case(gpu, w, h, bpc, layout, seed=bpc * 31 + layout + w, sb128=sb128, unit_log2=ul)


@pytest.mark.parametrize("bpc", [8, 10])
def test_lr_1080p_matches_oracle(gpu, bpc):
    run_case(gpu, 1920, 1080, bpc, 1, seed=0x4C1, sb128=1)


@pytest.mark.parametrize("layout", [1, 3])
def test_lr_tile_order_matches_oracle(gpu, layout):
    """The workgroups in mi_lr_tile_order's order (longest tiles first): the same pixels."""
    run_case(gpu, 330, 260, 10, layout, seed=0x7E + layout, sb128=0, unit_log2=(6, 5) if layout == 1 else (6, 6),
             ordered=True)
    run_case(gpu, 1920, 1080, 10, layout, seed=0x7F + layout, sb128=1, ordered=True)
