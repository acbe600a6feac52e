"""CPU checks of the CDEF oracle (oracle/cdef.c)."""
import ctypes

import numpy as np

from rav1d_amd.synth import add_cdef_meta
from tests import oracle_lib
from tests.oracle_lib import load_oracle, ptr
from tests.test_oracle_lf import frame, pad_planes


def find_dir(block, bpc):
    o = load_oracle()
    o.oracle_cdef_find_dir.restype = ctypes.c_int
    o.oracle_cdef_find_dir.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p, ctypes.c_int]
    b = np.ascontiguousarray(block)
    var = np.zeros(1, np.uint32)
    d = o.oracle_cdef_find_dir(ptr(b), b.strides[0], ptr(var), (1 << bpc) - 1)
    return d, int(var[0])


def test_find_dir_on_oriented_lines():
    # a pattern constant along one orientation must be detected as that direction class
    yy, xx = np.mgrid[0:8, 0:8]
    horiz = np.where(yy % 2 == 0, 200, 40).astype(np.uint8)     # rows constant
    vert = np.where(xx % 2 == 0, 200, 40).astype(np.uint8)      # columns constant
    dh, vh = find_dir(horiz, 8)
    dv, vv = find_dir(vert, 8)
    assert dh == 2 and dv == 6 and vh > 0 and vv > 0
    flat = np.full((8, 8), 128, np.uint8)
    assert find_dir(flat, 8) == (0, 0)


def test_zero_strength_frame_is_copy():
    w, h, bpc = 128, 64, 10
    planes, lf = frame(w, h, bpc, 1, 1)
    cd = add_cdef_meta(lf, np.random.default_rng(0))
    cd["y_strength"][:] = 0
    cd["uv_strength"][:] = 0
    src = pad_planes(planes, w, h, bpc, 1)
    out = oracle_lib.cdef_frame(src, bpc, 1, w, h, lf["masks"], cd)
    for p in range(3):
        assert np.array_equal(out[p], src[p])


def test_cdef_changes_textured_frame():
    w, h, bpc = 128, 128, 8
    planes, lf = frame(w, h, bpc, 1, 2)
    cd = add_cdef_meta(lf, np.random.default_rng(1), skip_frac=0.0, idx_unset_frac=0.0)
    cd["y_strength"][:] = 63
    src = pad_planes(planes, w, h, bpc, 1)
    out = oracle_lib.cdef_frame(src, bpc, 1, w, h, lf["masks"], cd)
    assert not np.array_equal(out[0], src[0])
    # output stays within the pixel range
    assert out[0].max() <= 255
