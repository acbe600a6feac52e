"""mi_lr_tile_order / mi_cdef_tile_order (host): permutations of the loop-restoration and CDEF
workgroups with the costliest first. CPU only."""
import ctypes

import numpy as np
import pytest

from rav1d_amd import MiCdef, MiLr, lib
from rav1d_amd.synth import RESTORATION_NONE, RESTORATION_WIENER, add_cdef_meta, make_lr_meta
from tests.test_oracle_lf import frame


def order_of(w, h, layout, lr):
    m = np.ascontiguousarray(lr["lr_mask"])
    s = MiLr()
    s.sb128w = m.shape[1]
    s.restore_planes = lr["restore_planes"]
    s.unit_size_log2[0], s.unit_size_log2[1] = lr["unit_size_log2"]
    cap = 4096
    buf = (ctypes.c_int32 * cap)()
    n = lib().mi_lr_tile_order(m.ctypes.data_as(ctypes.c_void_p), w, h, layout, ctypes.byref(s), buf, cap)
    return np.array(buf[:n]) if n >= 0 else n


@pytest.mark.parametrize("layout", [0, 1, 2, 3])
@pytest.mark.parametrize("size", [(330, 260), (1920, 1080)])
def test_order_is_a_permutation(layout, size):
    w, h = size
    lr = make_lr_meta(w, h, layout, np.random.default_rng(w + layout), sb128=1)
    o = order_of(w, h, layout, lr)
    assert isinstance(o, np.ndarray) and len(o) > 0
    assert np.array_equal(np.sort(o), np.arange(len(o)))


def test_order_puts_copies_last():
    """Wiener / self-guided tiles before the copy tiles (RESTORATION_NONE)."""
    w, h = 640, 360
    lr = make_lr_meta(w, h, 0, np.random.default_rng(7), sb128=0, unit_log2=(6, 6))
    u = lr["lr_mask"]["lr"]
    u["type"][:] = RESTORATION_NONE
    # one Wiener unit: the 64x64 at x = 320, y = 0 (128x128 superblock 2, quadrant 1), which
    # stripe 0's tile 5 alone uses
    u["type"][0, 2, 0, 1] = RESTORATION_WIENER
    o = order_of(w, h, 0, lr)
    assert o[0] == 5 and np.array_equal(o[1:6], [0, 1, 2, 3, 4]), o[:8]


def test_order_rejects_small_capacity():
    lr = make_lr_meta(330, 260, 1, np.random.default_rng(1), sb128=1)
    m = np.ascontiguousarray(lr["lr_mask"])
    s = MiLr()
    s.sb128w = m.shape[1]
    s.restore_planes = lr["restore_planes"]
    s.unit_size_log2[0], s.unit_size_log2[1] = lr["unit_size_log2"]
    buf = (ctypes.c_int32 * 4)()
    assert lib().mi_lr_tile_order(m.ctypes.data_as(ctypes.c_void_p), 330, 260, 1, ctypes.byref(s), buf, 4) < 0


def cdef_order_of(w, h, layout, lf, cd):
    m = np.ascontiguousarray(lf["masks"])
    s = MiCdef()
    s.sb128w = m.shape[1]
    s.y_strength[:] = [int(v) for v in cd["y_strength"]]
    s.uv_strength[:] = [int(v) for v in cd["uv_strength"]]
    buf = (ctypes.c_int32 * 4096)()
    n = lib().mi_cdef_tile_order(m.ctypes.data_as(ctypes.c_void_p), w, h, layout, ctypes.byref(s), buf, 4096)
    return np.array(buf[:n]) if n >= 0 else n


@pytest.mark.parametrize("layout", [0, 1])
def test_cdef_order_is_a_permutation_costliest_first(layout):
    w, h = 330, 200
    _, lf = frame(w, h, 8, layout, 5)
    cd = add_cdef_meta(lf, np.random.default_rng(6))
    o = cdef_order_of(w, h, layout, lf, cd)
    assert isinstance(o, np.ndarray) and np.array_equal(np.sort(o), np.arange(len(o)))
    # a unit with cdef_idx -1 (nothing to filter) never precedes one with a primary strength
    m = lf["masks"]
    tx = (w + 63) // 64

    def prim(t):
        x, y = t % tx, t // tx
        idx = int(m[y >> 1, x >> 1]["cdef_idx"][(y & 1) * 2 + (x & 1)])
        return idx >= 0 and (cd["y_strength"][idx] >> 2 or (layout and cd["uv_strength"][idx] >> 2))

    def none(t):
        x, y = t % tx, t // tx
        return int(m[y >> 1, x >> 1]["cdef_idx"][(y & 1) * 2 + (x & 1)]) < 0

    last_prim = max((i for i, t in enumerate(o) if prim(t)), default=-1)
    first_none = min((i for i, t in enumerate(o) if none(t)), default=len(o))
    assert last_prim < first_none


def test_cdef_order_deals_each_class_to_xcds_in_runs():
    """Within a cost class, the units workgroup b % 8 == x takes (XCD x) are one increasing,
    contiguous run of that class's units in picture order, and the runs follow XCD order."""
    w, h = 1920, 1080
    _, lf = frame(w, h, 8, 1, 11)
    cd = add_cdef_meta(lf, np.random.default_rng(12))
    o = cdef_order_of(w, h, 1, lf, cd)
    assert isinstance(o, np.ndarray) and np.array_equal(np.sort(o), np.arange(len(o)))
    m = lf["masks"]
    tx = (w + 63) // 64

    def cls(t):   # (mi_cdef_tile_order's classes: 2 a primary strength, 1 secondary only, 0 none)
        x, y = t % tx, t // tx
        sb = m[y >> 1, x >> 1]
        idx = int(sb["cdef_idx"][(y & 1) * 2 + (x & 1)])
        if idx < 0:
            return 0
        yl, uvl = int(cd["y_strength"][idx]), int(cd["uv_strength"][idx])
        if not yl and not uvl:
            return 0
        rows = sb["noskip_mask"][8 * (y & 1):8 * (y & 1) + 8]
        if not any(((int(r[1]) << 16 | int(r[0])) >> (16 * (x & 1))) & 0xffff for r in rows):
            return 0
        return 2 if (yl >> 2 or uvl >> 2) else 1

    c = np.array([cls(int(t)) for t in o])
    assert np.all(np.diff(c) <= 0), "classes costliest first"
    for k in np.unique(c):
        pos = np.nonzero(c == k)[0]
        items = sorted(int(t) for t in o[pos])   # the class's units in picture order
        runs = [[int(o[p]) for p in pos if p % 8 == x] for x in range(8)]
        flat = [t for r in runs for t in r]
        assert flat == items, "XCD x holds the x-th contiguous run of the class"
