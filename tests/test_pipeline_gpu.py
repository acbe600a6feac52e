"""End-to-end GPU parity: one frame through the whole device pipeline (bench.Pipeline:
[MC ->] itx -> deblock -> CDEF -> LR [-> film grain, prep on a side stream]) vs the oracle
pipeline, every intermediate picture bit-exact."""
import numpy as np
import pytest
import torch

from rav1d_amd.synth import make_frame
from tests.pipeline import oracle_pipeline

pytestmark = pytest.mark.gpu

# (w, h, bpc, layout, inter frame with MC, film grain)
GEOMS = [(1920, 1080, 10, 1, False, True), (640, 360, 8, 1, False, True), (352, 288, 12, 3, False, True),
         (1920, 1080, 10, 1, True, False), (720, 486, 8, 2, True, True), (3840, 2160, 10, 1, True, False)]


@pytest.mark.parametrize("geom", GEOMS)
def test_pipeline_matches_oracle(gpu, geom):
    import bench
    w, h, bpc, layout, mc, fg = geom
    fr = make_frame(w, h, bpc, layout, seed=w + bpc, with_fg=fg, with_mc=mc)
    pipe = bench.Pipeline(gpu, fr)
    pipe.step(torch.cuda.current_stream())
    torch.cuda.synchronize()
    ref = oracle_pipeline(fr)
    stages = [("recon_deblocked", pipe.D), ("cdef", pipe.B), ("lr", pipe.O)]
    if fg:
        stages.append(("out", pipe.G))
    for name, pic in stages:
        for p in range(3 if layout else 1):
            got = pic.plane_np(p)
            ph, pw = got.shape
            assert np.array_equal(got, ref[name][p][:ph, :pw]), f"{name} plane {p}"
