"""Oracle self-checks for motion compensation (CPU only): the C restatement (oracle/mc.c) is
compared with an independent numpy restatement of mc_tmpl.c's put/prep arithmetic, and
its edge emulation with clamped indexing. Parity against the reference itself is unpinned
(DESIGN.md §Oracle): the reference ships no per-function vectors for this path."""
import ctypes

import numpy as np
import pytest

from tests import oracle_lib
from tests.oracle_lib import load_oracle, ptr

SUBPEL = None


def subpel():
    global SUBPEL
    if SUBPEL is None:
        import os
        txt = open(os.path.join(oracle_lib.ROOT, "rav1d_amd", "csrc", "tables", "mc_subpel_filters.inc")).read()
        vals = [int(v) for v in txt.split("*/", 1)[1].replace(",", " ").split()]
        SUBPEL = np.array(vals, np.int64).reshape(6, 15, 8)
    return SUBPEL


F2D_H = [0, 0, 0, 2, 2, 2, 1, 1, 1]
F2D_V = [0, 1, 2, 0, 1, 2, 0, 1, 2]


def np_mc(src, x0, y0, w, h, mx, my, f2d, bpc, prep):
    """numpy restatement of put/prep_8tap_c and put/prep_bilin_c (mc_tmpl.c) on a padded src
    with the block's top-left at (x0, y0)."""
    ib = 4 if bpc == 8 else 14 - bpc
    bias = 0 if bpc == 8 else 8192
    bdmax = (1 << bpc) - 1
    s = src.astype(np.int64)
    rnd = lambda v, sh: (v + ((1 << sh) >> 1)) >> sh
    if f2d == 9:
        SH = 4
        fh = np.array([0, 0, 0, 16 - mx, mx, 0, 0, 0]) if mx else None
        fv = np.array([0, 0, 0, 16 - my, my, 0, 0, 0]) if my else None
    else:
        SH = 6
        th, tv = F2D_H[f2d], F2D_V[f2d]
        fh = (subpel()[th if w > 4 else 3 + (th & 1)][mx - 1]) if mx else None
        fv = (subpel()[tv if h > 4 else 3 + (tv & 1)][my - 1]) if my else None

    def hsum(rows):   # rows: absolute row indices -> (len(rows), w)
        return sum(fh[k] * s[rows][:, x0 - 3 + k:x0 - 3 + k + w] for k in range(8))

    if fh is not None and fv is not None:
        mid = rnd(hsum(np.arange(y0 - 3, y0 + h + 4)), SH - ib)
        v = sum(fv[k] * mid[k:k + h] for k in range(8))
        return rnd(v, SH) - bias if prep else np.clip(rnd(v, SH + ib), 0, bdmax)
    if fh is not None:
        px = rnd(hsum(np.arange(y0, y0 + h)), SH - ib)
        return px - bias if prep else np.clip((px + ((1 << ib) >> 1)) >> ib, 0, bdmax)
    if fv is not None:
        v = sum(fv[k] * s[y0 - 3 + k:y0 - 3 + k + h, x0:x0 + w] for k in range(8))
        return rnd(v, SH - ib) - bias if prep else np.clip(rnd(v, SH), 0, bdmax)
    v = s[y0:y0 + h, x0:x0 + w]
    return (v << ib) - bias if prep else v


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_oracle_put_prep_match_numpy(bpc):
    o = load_oracle()
    oracle_lib._mc_sigs(o)
    rng = np.random.default_rng(bpc)
    dt = np.uint8 if bpc == 8 else np.uint16
    src = rng.integers(0, 1 << bpc, size=(160, 160)).astype(dt)
    for case in range(160):
        w, h = [(2, 2), (4, 4), (4, 8), (8, 4), (8, 8), (16, 8), (32, 32), (64, 16), (128, 128), (4, 16)][case % 10]
        w, h = min(w, 128), min(h, 128)
        f2d = int(rng.integers(0, 10))
        mx = int(rng.integers(0, 16)) * (case % 4 != 0)
        my = int(rng.integers(0, 16)) * (case % 3 != 0)
        x0, y0 = 8, 8
        sp = src[y0:, x0:]
        ss = src.strides[0]
        exp_put = np_mc(src, x0, y0, w, h, mx, my, f2d, bpc, False)
        exp_prep = np_mc(src, x0, y0, w, h, mx, my, f2d, bpc, True)
        dst = np.zeros((h, w), dt)
        o.oracle_mc_put(f2d, ptr(dst), dst.strides[0], ctypes.c_void_p(sp.ctypes.data), ss, w, h, mx, my, bpc)
        tmp = np.zeros((h, w), np.int16)
        o.oracle_mc_prep(f2d, ptr(tmp), ctypes.c_void_p(sp.ctypes.data), ss, w, h, mx, my, bpc)
        assert np.array_equal(dst.astype(np.int64), exp_put), (case, w, h, f2d, mx, my)
        assert np.array_equal(tmp.astype(np.int64), exp_prep), (case, w, h, f2d, mx, my)


def test_oracle_emu_edge_is_clamping():
    o = load_oracle()
    oracle_lib._mc_sigs(o)
    rng = np.random.default_rng(7)
    ref = rng.integers(0, 1024, size=(40, 50)).astype(np.uint16)
    for _ in range(200):
        bw, bh = int(rng.integers(1, 30)), int(rng.integers(1, 30))
        x, y = int(rng.integers(-bw + 1, 50)), int(rng.integers(-bh + 1, 40))
        dst = np.zeros((bh, 64), np.uint16)
        o.oracle_mc_emu_edge(bw, bh, 50, 40, x, y, ptr(dst), dst.strides[0], ptr(ref), ref.strides[0], 10)
        ys = np.clip(np.arange(y, y + bh), 0, 39)
        xs = np.clip(np.arange(x, x + bw), 0, 49)
        assert np.array_equal(dst[:, :bw], ref[np.ix_(ys, xs)])


def test_oracle_w_mask_420_is_rounded_quad_average():
    o = load_oracle()
    oracle_lib._mc_sigs(o)
    rng = np.random.default_rng(3)
    w, h = 16, 8
    t1 = rng.integers(-8000, 30000, size=(h, w)).astype(np.int16)
    t2 = rng.integers(-8000, 30000, size=(h, w)).astype(np.int16)
    dst = np.zeros((h, w), np.uint16)
    for sign in (0, 1):
        m420 = np.zeros((h // 2) * (w // 2), np.uint8)
        o.oracle_mc_w_mask(ptr(dst), dst.strides[0], ptr(t1), ptr(t2), w, h, ptr(m420), sign, 1, 1, 10)
        m444 = np.zeros(h * w, np.uint8)
        o.oracle_mc_w_mask(ptr(dst), dst.strides[0], ptr(t1), ptr(t2), w, h, ptr(m444), sign, 0, 0, 10)
        full = m444.reshape(h, w).astype(np.int64)
        assert full.min() >= 38 and full.max() <= 64
        quad = full[0::2, 0::2] + full[0::2, 1::2] + full[1::2, 0::2] + full[1::2, 1::2]
        assert np.array_equal(m420.reshape(h // 2, w // 2), (quad + 2 - sign) >> 2)


def test_oracle_mc_frame_integer_copy():
    """Zero sub-pel, single reference: the prediction is the displaced reference block."""
    from rav1d_amd import MCBLOCK_DTYPE
    rng = np.random.default_rng(5)
    w, h = 64, 48
    ref = rng.integers(0, 1024, size=(128, 128)).astype(np.uint16)
    cur = np.zeros((128, 128), np.uint16)
    u = np.zeros(2, MCBLOCK_DTYPE)
    u[0] = (8, 8, 16, 16, 0, 0, (16, 0), (-24, 0), (0, -1), 0, 0, 0)    # mv (+2, -3) px
    u[1] = (32, 16, 8, 8, 0, 3, (-80, 0), (8, 0), (0, -1), 0, 0, 0)     # mv (-10, +1) px
    out, _ = oracle_lib.mc_frame([cur], [[ref]], 10, 0, w, h, u, np.zeros(1, np.uint8))
    assert np.array_equal(out[0][8:24, 8:24], ref[5:21, 10:26])
    assert np.array_equal(out[0][16:24, 32:40], ref[17:25, 22:30])


def test_oracle_ext_paths_preserve_flat_pictures():
    """Invariants of the scaled, warp and resize restatements: every filter bank sums to its
    unit gain, so a flat reference predicts / upscales to the same flat value (any phase,
    any step), at every bit depth."""
    from rav1d_amd import MCBLOCK_DTYPE, MC_PREP, WARP_DTYPE
    rng = np.random.default_rng(9)
    for bpc in (8, 10, 12):
        dt = np.uint8 if bpc == 8 else np.uint16
        v = int(rng.integers(0, 1 << bpc))
        ref = np.full((128, 256), v, dt)
        cur = np.zeros((128, 256), dt)
        # scaled: 1.5x reference, random phases / filters, put
        u = np.zeros(4, MCBLOCK_DTYPE)
        for k in range(4):
            u[k] = (16 * k, 8, 16, 8, 0, k * 2 + 1, (int(rng.integers(-99, 99)), 0), (int(rng.integers(-99, 99)), 0),
                    (0, -1), 0, 0, 0)
        out, _ = oracle_lib.mc_scaled_frame([cur], [[ref]], [(240, 96)], bpc, 0, 160, 64, u, np.zeros(1, np.int16))
        assert (out[0][8:16, :64] == v).all()
        # warp: random shear parameters
        wb = np.zeros(3, WARP_DTYPE)
        for k in range(3):
            abcd = [int(x) for x in rng.integers(-900, 900, size=4)]
            wb[k] = (8 * k, 0, 0, 0, 0, 0, 20 + k, 9, int(rng.integers(0, 1 << 16)) & ~63,
                     int(rng.integers(0, 1 << 16)) & ~63, abcd, 0, 8, 0)
        out, _ = oracle_lib.mc_warp_frame([cur], [[ref]], bpc, 0, 160, 64, wb, np.zeros(1, np.int16))
        assert (out[0][0:8, 0:24] == v).all()
        # super-resolution 100 -> 160 luma
        up = oracle_lib.superres_frame([ref], [cur], bpc, 0, 100, 160, 32)
        assert (up[0][:32, :160] == v).all()
