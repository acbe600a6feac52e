"""GPU parity: film grain (parallel-LFSR/wavefront-AR prep + per-pixel apply) vs the oracle's
rav1d_apply_grain, bit-exact."""
import numpy as np
import pytest
import torch

from rav1d_amd.frame import Frame, film_grain_frame
from rav1d_amd.synth import make_fg_params
from tests import oracle_lib
from tests.test_lr_gpu import to_frame
from tests.test_oracle_lf import pad_planes
from tests.test_oracle_lr import planes_for

pytestmark = pytest.mark.gpu


def run_case(gpu, w, h, bpc, layout, seed, is_id=0, **over):
    rng = np.random.default_rng(seed)
    planes = planes_for(w, h, bpc, layout, rng)
    fg = make_fg_params(rng, layout)
    fg.update(over)
    src = to_frame(planes, w, h, bpc, layout)
    dst = Frame(w, h, bpc, layout)
    film_grain_frame(gpu, src, dst, fg, is_id)
    torch.cuda.synchronize()
    ref = oracle_lib.film_grain(pad_planes(planes, w, h, bpc, layout), bpc, layout, w, h, fg, is_id)
    for p in range(len(planes)):
        ph, pw = planes[p].shape
        assert np.array_equal(dst.plane_np(p), ref[p][:ph, :pw]), f"plane {p}"
        assert np.array_equal(src.plane_np(p), planes[p])


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [1, 2, 3, 0])
@pytest.mark.parametrize("size", [(256, 160), (201, 133)])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_film_grain_matches_oracle(gpu, bpc, layout, size, seed):
    run_case(gpu, size[0], size[1], bpc, layout, seed=seed * 100 + bpc + layout, is_id=seed == 2)


@pytest.mark.parametrize("lag", [0, 1, 2, 3])
def test_film_grain_ar_lags(gpu, lag):
    run_case(gpu, 160, 96, 10, 1, seed=77 + lag, ar_coeff_lag=lag, overlap_flag=1)


def test_film_grain_8k_matches_oracle(gpu):
    run_case(gpu, 7680, 4320, 10, 1, seed=0xF6000001)
