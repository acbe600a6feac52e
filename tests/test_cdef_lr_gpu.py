"""GPU parity: fused CDEF + loop restoration (mi_cdef_lr_frame: one workgroup per stripe x 64
luma columns, the CDEF output kept in LDS) vs the oracle's CDEF then loop restoration, and vs
the two-kernel device path (mi_cdef_frame, mi_lr_frame), bit-exact."""
import numpy as np
import pytest
import torch

from rav1d_amd.frame import CdefMeta, Frame, LrMeta, cdef_frame, cdef_lr_frame, lr_frame
from rav1d_amd.synth import add_cdef_meta, make_lr_meta
from tests import oracle_lib
from tests.test_oracle_lf import frame, pad_planes

pytestmark = pytest.mark.gpu


def to_frame(planes, w, h, bpc, layout):
    f = Frame(w, h, bpc, layout)
    for p, a in enumerate(planes):
        f.set_plane_np(p, a)
    return f


def run_case(gpu, w, h, bpc, layout, seed, unit_log2=None, restore_planes=None, cdef_off=False):
    planes, lf = frame(w, h, bpc, layout, seed)
    planes = planes[:1] if layout == 0 else planes
    rng = np.random.default_rng(seed + 99)
    cd = add_cdef_meta(lf, rng)
    if cdef_off:
        cd["y_strength"][:] = 0
        cd["uv_strength"][:] = 0
    # (a 64-px luma unit exists only with 64x64 superblocks: lr_unit_shift, obu.rs)
    sb128 = 0 if unit_log2 is not None and unit_log2[0] == 6 else 1
    lr = make_lr_meta(w, h, layout, rng, sb128=sb128, unit_log2=unit_log2)
    if restore_planes is not None:
        lr["restore_planes"] = restore_planes
    cm, lm = CdefMeta(lf["masks"], cd), LrMeta(lr)
    d = to_frame(planes, w, h, bpc, layout)
    fused = Frame(w, h, bpc, layout)
    cdef_lr_frame(gpu, d, fused, cm, lm)
    c, two = Frame(w, h, bpc, layout), Frame(w, h, bpc, layout)
    cdef_frame(gpu, d, c, cm)
    lr_frame(gpu, c, d, two, lm)
    torch.cuda.synchronize()
    ref_c = oracle_lib.cdef_frame(pad_planes(planes, w, h, bpc, layout), bpc, layout, w, h, lf["masks"], cd)
    cc = [ref_c[p][:a.shape[0], :a.shape[1]] for p, a in enumerate(planes)]
    ref = oracle_lib.lr_frame(pad_planes(cc, w, h, bpc, layout), pad_planes(planes, w, h, bpc, layout),
                              bpc, layout, w, h, lr)
    def where(x, y):
        bad = np.argwhere(x != y)
        return f"{len(bad)} px differ, first (row, col) {bad[:6].tolist()}"

    for p, a in enumerate(planes):
        ph, pw = a.shape
        got = fused.plane_np(p)
        r = ref[p][:ph, :pw]
        assert np.array_equal(two.plane_np(p), r), f"plane {p}: two-kernel path vs oracle: {where(two.plane_np(p), r)}"
        assert np.array_equal(got, r), f"plane {p}: fused vs oracle: {where(got, r)}"
        assert np.array_equal(d.plane_np(p), a), "the deblocked picture must stay untouched"


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [1, 2, 3, 0])
@pytest.mark.parametrize("size", [(256, 192), (200, 134), (330, 260)])
def test_cdef_lr_matches_oracle(gpu, bpc, layout, size):
    run_case(gpu, size[0], size[1], bpc, layout, seed=bpc * 7 + layout * 3 + size[1])


@pytest.mark.parametrize("layout", [1, 3])
def test_cdef_lr_partial_planes(gpu, layout):
    """Loop restoration on luma only: the chroma planes are the CDEF output."""
    run_case(gpu, 264, 136, 10, layout, seed=0xC1 + layout, restore_planes=1)


def test_cdef_lr_without_cdef_strengths(gpu):
    """Every CDEF strength zero: the window is D itself."""
    run_case(gpu, 200, 150, 8, 1, seed=0xC2, cdef_off=True)


@pytest.mark.parametrize("unit_log2", [(6, 5), (8, 7)])
def test_cdef_lr_unit_sizes(gpu, unit_log2):
    run_case(gpu, 392, 264, 10, 1, seed=0xC3 + unit_log2[0], unit_log2=unit_log2)


@pytest.mark.parametrize("bpc", [8, 10])
def test_cdef_lr_1080p_matches_oracle(gpu, bpc):
    run_case(gpu, 1920, 1080, bpc, 1, seed=0xCD1F)
