"""Debug: per-call generate_grain_uv vs the oracle, print mismatch positions."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from rav1d_amd import lib
from rav1d_amd.frame import film_grain_data, Context
from rav1d_amd.synth import make_fg_params
from tests.test_dsp_calls_gpu import _fg_sigs, _o, _entry, P
ctx = Context(0)
o = _fg_sigs(_o())
for bpc in (10,):
    rng = np.random.default_rng(1000 + bpc)
    bdmax = (1 << bpc) - 1
    for it in range(6):
        layout = int(rng.integers(1, 4))
        fg = make_fg_params(rng, layout)
        d = film_grain_data(fg)
        ref_y = np.zeros((73, 82), np.int16)
        o.oracle_fg_generate_grain_y(P(ref_y), ctypes.byref(d), bdmax)
        got_y = np.zeros((74, 82), _entry(bpc))
        assert lib().mi_dsp_fg_generate_grain_y(P(got_y), ctypes.byref(d), bdmax) == 0
        sx, sy = int(layout != 3), int(layout == 1)
        print("it", it, "layout", layout, "lag", fg["ar_coeff_lag"], "y ok", np.array_equal(got_y[:73].astype(np.int16), ref_y), "ny", fg["num_y_points"])
        for uv in (0, 1):
            fill = int(rng.integers(-100, 100))
            ref = np.full((74, 82), fill, np.int16)
            o.oracle_fg_generate_grain_uv(P(ref), P(ref_y), ctypes.byref(d), uv, sx, sy, bdmax)
            got = np.full((74, 82), fill, _entry(bpc))
            assert lib().mi_dsp_fg_generate_grain_uv(layout, P(got), P(got_y), ctypes.byref(d), uv, bdmax) == 0
            bad = np.argwhere(got.astype(np.int16) != ref)
            print("  uv", uv, "bad", len(bad), bad[:6].tolist(), flush=True)
