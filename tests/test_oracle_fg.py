"""CPU checks of the film-grain oracle (oracle/filmgrain.c)."""
import os
import re

import numpy as np
import pytest

from rav1d_amd.synth import make_fg_params
from tests import oracle_lib
from tests.test_oracle_lf import pad_planes
from tests.test_oracle_lr import planes_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_TABLES = "/root/reference/src/tables.c"


@pytest.mark.skipif(not os.path.exists(REF_TABLES), reason="reference not mounted")
def test_gaussian_table_matches_reference():
    txt = open(REF_TABLES).read()
    i = txt.index("dav1d_gaussian_sequence[2048]")
    body = txt[txt.index("{", i) + 1: txt.index("};", i)]
    ref = [int(v) for v in re.findall(r"-?\d+", body)]
    ours = open(os.path.join(ROOT, "rav1d_amd", "csrc", "tables", "gaussian_sequence.inc")).read()
    ours = [int(v) for v in re.findall(r"-?\d+", ours.split("\n", 1)[1])]
    assert ref == ours and len(ours) == 2048


def test_grain_template_statistics():
    """White Gaussian template (lag 0): zero-mean, spread ~ the gaussian table / 2^shift."""
    rng = np.random.default_rng(1)
    fg = make_fg_params(rng)
    fg.update(ar_coeff_lag=0, grain_scale_shift=0)
    g = oracle_lib.fg_grain_y(fg, 8).astype(np.float64)
    assert abs(g.mean()) < 3 and 20 < g.std() < 40 and g.min() >= -128 and g.max() <= 127


def test_zero_scaling_is_copy():
    w, h, bpc, layout = 100, 70, 10, 1
    rng = np.random.default_rng(2)
    planes = pad_planes(planes_for(w, h, bpc, layout, rng), w, h, bpc, layout)
    fg = make_fg_params(rng)
    fg.update(y_points=[(0, 0), (255, 0)], num_y_points=2, clip_to_restricted_range=0,
              chroma_scaling_from_luma=0, num_uv_points=[0, 0], uv_points=[[], []])
    out = oracle_lib.film_grain(planes, bpc, layout, w, h, fg)
    for p in range(3):
        assert np.array_equal(out[p], planes[p])


def test_per_call_strips_compose_the_frame():
    """oracle_fg_32x32xn (the fgy_32x32xn table slot) over every 32-row strip of the luma plane,
    with the frame's own template and scaling LUT, reproduces oracle_fg_apply's luma plane."""
    import ctypes
    from rav1d_amd.frame import film_grain_data
    w, h, bpc, layout = 150, 90, 10, 1
    rng = np.random.default_rng(3)
    planes = pad_planes(planes_for(w, h, bpc, layout, rng), w, h, bpc, layout)
    fg = make_fg_params(rng, layout)
    fg.update(overlap_flag=1)
    ref = oracle_lib.film_grain(planes, bpc, layout, w, h, fg)
    o = oracle_lib.load_oracle()
    VP, I = ctypes.c_void_p, ctypes.c_int
    o.oracle_fg_generate_scaling.argtypes = [I, VP, I, VP]
    o.oracle_fg_generate_scaling.restype = None
    o.oracle_fg_32x32xn.argtypes = [I, I, VP, VP, ctypes.c_ssize_t, VP, I, VP, VP, I, I, VP, ctypes.c_ssize_t, I, I]
    o.oracle_fg_32x32xn.restype = None
    lut = np.zeros((74, 82), np.int16)
    lut[:73] = oracle_lib.fg_grain_y(fg, bpc)
    pts = np.zeros((14, 2), np.uint8)
    pts[:fg["num_y_points"]] = fg["y_points"]
    scl = np.zeros(4096, np.uint8)
    o.oracle_fg_generate_scaling(bpc, oracle_lib.ptr(pts), fg["num_y_points"], oracle_lib.ptr(scl))
    d = film_grain_data(fg)
    src = np.ascontiguousarray(planes[0])
    out = src.copy()
    for row in range((h + 31) // 32):
        bh = min(32, h - 32 * row)
        off = row * 32 * src.shape[1]
        o.oracle_fg_32x32xn(0, layout, ctypes.c_void_p(out.ctypes.data + 2 * off),
                            ctypes.c_void_p(src.ctypes.data + 2 * off), src.strides[0], ctypes.byref(d), w,
                            oracle_lib.ptr(scl), oracle_lib.ptr(lut), bh, row, None, 0, 0, (1 << bpc) - 1)
    assert np.array_equal(out[:h, :w], ref[0][:h, :w])


TABLES = {"dr_intra_derivative": 44, "filter_intra_taps": 320, "mc_subpel_filters": 720, "mc_warp_filter": 1544,
          "obmc_masks": 64, "resize_filter": 512, "sm_weights": 128}


@pytest.mark.skipif(not os.path.exists(REF_TABLES), reason="reference not mounted")
@pytest.mark.parametrize("name", sorted(TABLES))
def test_kernel_tables_match_reference(name):
    """Every constant table the HIP kernels and the oracle compile in equals the reference's
    dav1d_<name> (src/tables.c; the generic-C layout of the filter-intra F() macro,
    tables.c:753-757), parsed by tools/gen_tables.py, value for value."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_tables
    txt = open(REF_TABLES).read()
    key = next(k for k in re.findall(r"dav1d_" + name + r"\[[^=]*", txt))
    fn = gen_tables.filter_intra if name == "filter_intra_taps" else gen_tables.numbers
    ref = fn(gen_tables.body_of(txt, key.strip()))
    ours = open(os.path.join(ROOT, "rav1d_amd", "csrc", "tables", f"{name}.inc")).read()
    ours = [int(v) for v in re.findall(r"-?\d+", re.sub(r"/\*.*?\*/", "", ours, flags=re.S))]
    assert len(ref) == TABLES[name] and ref == ours


@pytest.mark.skipif(not os.path.exists(REF_TABLES), reason="reference not mounted")
def test_sgr_params_match_reference():
    """k_sgr_params in lr.hip (and the per-call tests' copy) equal dav1d_sgr_params."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_tables
    ref = gen_tables.numbers(gen_tables.body_of(open(REF_TABLES).read(), "dav1d_sgr_params[16][2]"))
    src = open(os.path.join(ROOT, "rav1d_amd", "csrc", "lr.hip")).read()
    i = src.index("k_sgr_params[16][2] = {")
    ours = [int(v) for v in re.findall(r"-?\d+", src[i + len("k_sgr_params[16][2] = {"): src.index("};", i)])]
    assert ref == ours and len(ours) == 32
    from tests.test_dsp_calls_gpu import _SGR
    assert [v for pr in _SGR for v in pr] == ref
