"""End-to-end GPU parity: one frame through the whole device pipeline (bench.Pipeline:
itx -> deblock -> CDEF -> LR -> film grain, with the film-grain prep on a side stream) vs
the oracle pipeline, every intermediate picture bit-exact."""
import numpy as np
import pytest
import torch

from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame
from tests.pipeline import oracle_pipeline

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("geom", [(1920, 1080, 10, 1), (640, 360, 8, 1), (352, 288, 12, 3), (3840, 2160, 10, 1)])
def test_pipeline_matches_oracle(gpu, geom):
    import bench
    w, h, bpc, layout = geom
    fr = make_frame(w, h, bpc, layout, seed=w + bpc)
    pipe = bench.Pipeline(gpu, fr)
    pipe.step(torch.cuda.current_stream())
    torch.cuda.synchronize()
    ref = oracle_pipeline(fr)
    for name, pic in (("recon_deblocked", pipe.A), ("cdef", pipe.B), ("lr", pipe.O), ("out", pipe.G)):
        for p in range(3 if layout else 1):
            got = pic.plane_np(p)
            ph, pw = got.shape
            assert np.array_equal(got, ref[name][p][:ph, :pw]), f"{name} plane {p}"
