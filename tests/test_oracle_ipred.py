"""Oracle self-checks for intra prediction (CPU only): oracle/ipred.c against an independent
numpy restatement of ipred_tmpl.c for the non-directional modes and CfL / palette, and
structural properties of the directional modes. Parity with the reference is unpinned
(DESIGN.md §Oracle)."""
import numpy as np
import pytest

from tests import oracle_lib

SMW = None


def sm_weights():
    global SMW
    if SMW is None:
        import os
        txt = open(os.path.join(oracle_lib.ROOT, "rav1d_amd", "csrc", "tables", "sm_weights.inc")).read()
        SMW = np.array([int(v) for v in txt.split("*/", 1)[1].replace(",", " ").split()], np.int64)
    return SMW


def np_pred(mode, e, t, w, h, bpc):
    top = e[t + 1:t + 1 + w].astype(np.int64)
    left = e[t - h:t][::-1].astype(np.int64)       # left[i] = topleft[-(1+i)]
    c = int(e[t])
    X, Y = np.meshgrid(np.arange(w), np.arange(h))
    if mode == 1:
        return np.broadcast_to(top, (h, w))
    if mode == 2:
        return np.broadcast_to(left[:, None], (h, w))
    if mode == 12:
        T, L = top[X], left[Y]
        base = L + T - c
        ld, td, tld = abs(L - base), abs(T - base), abs(c - base)
        return np.where((ld <= td) & (ld <= tld), L, np.where(td <= tld, T, c))
    sw = sm_weights()
    right, bottom = int(e[t + w]), int(e[t - h])
    wv, wh = sw[h + Y], sw[w + X]
    if mode == 9:
        return (wv * top[X] + (256 - wv) * bottom + wh * left[Y] + (256 - wh) * right + 256) >> 9
    if mode == 10:
        return (wv * top[X] + (256 - wv) * bottom + 128) >> 8
    if mode == 11:
        return (wh * left[Y] + (256 - wh) * right + 128) >> 8
    if mode in (0, 3, 4):
        tsum, lsum = int(top.sum()), int(left.sum())
        if mode == 4:
            return np.full((h, w), (tsum + (w >> 1)) >> int(np.log2(w)))
        if mode == 3:
            return np.full((h, w), (lsum + (h >> 1)) >> int(np.log2(h)))
        dc = (tsum + lsum + ((w + h) >> 1)) >> ((w + h) & -(w + h)).bit_length() - 1
        if w != h:
            q = w > 2 * h or h > 2 * w
            dc = (dc * ((0x3334 if q else 0x5556) if bpc == 8 else (0x6667 if q else 0xAAAB))) >> (16 if bpc == 8 else 17)
        return np.full((h, w), dc)
    if mode == 5:
        return np.full((h, w), 128 if bpc == 8 else (1 << (bpc - 1)))
    raise ValueError(mode)


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_oracle_nondirectional_match_numpy(bpc):
    rng = np.random.default_rng(bpc)
    for _ in range(300):
        w, h = [4, 8, 16, 32, 64][rng.integers(0, 5)], [4, 8, 16, 32, 64][rng.integers(0, 5)]
        if max(w, h) > 4 * min(w, h):
            continue
        mode = int(rng.choice([0, 1, 2, 3, 4, 5, 9, 10, 11, 12]))
        e = rng.integers(0, 1 << bpc, size=2 * 130 + 1)
        got = oracle_lib.intra_pred(mode, e, 130, w, h, 0, w, h, bpc)
        assert np.array_equal(got.astype(np.int64), np_pred(mode, e, 130, w, h, bpc)), (mode, w, h)


def test_oracle_z1_45_degrees_is_diagonal_copy():
    """Z1 at 45 degrees without edge filtering: dst[y][x] = top[x + y + 1] (dx = 64)."""
    rng = np.random.default_rng(1)
    e = rng.integers(0, 1024, size=261)
    got = oracle_lib.intra_pred(6, e, 130, 8, 8, 45, 8, 8, 10)
    top = e[131:]
    exp = np.array([[top[min(x + y + 1, 8 + 8 - 1)] for x in range(8)] for y in range(8)])
    assert np.array_equal(got, exp)


def test_oracle_cfl_and_palette():
    rng = np.random.default_rng(2)
    e = rng.integers(0, 1024, size=261)
    ac = rng.integers(-2000, 2000, size=64).astype(np.int16)
    for mode, alpha in ((0, 5), (3, -7), (4, 16), (5, -16)):
        got = oracle_lib.cfl_pred(mode, e, 130, 8, 8, ac, alpha, 10).astype(np.int64)
        dc = int(np_pred(mode, e, 130, 8, 8, 10)[0, 0])
        diff = alpha * ac.astype(np.int64).reshape(8, 8)
        exp = np.clip(dc + np.sign(diff) * ((abs(diff) + 32) >> 6), 0, 1023)
        assert np.array_equal(got, exp)
    pal = rng.integers(0, 1024, size=8)
    idx = rng.integers(0, 8, size=32).astype(np.uint8)
    assert np.array_equal(oracle_lib.pal_pred(pal, idx, 8, 4, 10), pal[idx].reshape(4, 8))


@pytest.mark.parametrize("bpc", [8, 10])
def test_oracle_intra_block_copy(bpc):
    """MI_INTRA_IBC in the oracle: an integer luma displacement copies the source rectangle; a
    half-pel chroma phase (odd luma displacement, 4:2:0) averages neighbours as put_bilin does."""
    from rav1d_amd import INTRA_DTYPE
    rng = np.random.default_rng(5 + bpc)
    dt = np.uint8 if bpc == 8 else np.uint16
    luma = rng.integers(0, 1 << bpc, size=(64, 64)).astype(dt)
    chroma = rng.integers(0, 1 << bpc, size=(32, 32)).astype(dt)
    mv = lambda lx, ly: (lx * 8 & 0xFFFF) | ((ly * 8 & 0xFFFF) << 16)  # noqa: E731
    blk = np.zeros(2, INTRA_DTYPE)
    blk[0] = (32, 32, 16, 8, 0, 96, 0, 0, 0, 0, 64, 64, 64, 64, 0, 0, mv(-20, -24))
    blk[1] = (16, 16, 8, 8, 1, 96, 0, 0, 3, 0, 32, 32, 32, 32, 0, 0, mv(-9, -20))
    z = np.zeros(1, np.int16)
    out = oracle_lib.intra_blocks([luma, chroma, chroma.copy()], bpc, blk, z, np.zeros(1, np.uint8), np.zeros(8, dt))
    assert np.array_equal(out[0][32:40, 32:48], luma[8:16, 12:28])
    # chroma: x offset floor(-9 / 2) = -5 with phase 8/16, y offset -10 exactly (source and
    # destination disjoint, as the block-copy constraints guarantee)
    src = chroma.astype(np.int64)
    a, b = src[6:14, 11:19], src[6:14, 12:20]
    ib = 4 if bpc == 8 else 14 - bpc
    px = (16 * a + 8 * (b - a) + ((1 << (4 - ib)) >> 1)) >> (4 - ib)
    exp = np.clip((px + ((1 << ib) >> 1)) >> ib, 0, (1 << bpc) - 1)
    assert np.array_equal(out[1][16:24, 16:24].astype(np.int64), exp)


@pytest.mark.parametrize("bpc", [8, 10])
def test_oracle_intra_block_copy_edge(bpc):
    """A half-pel chroma block copy whose source ends at the reference area's right / bottom
    border (max_w x max_h = f.bw*4 >> ss_hor by f.bh*4 >> ss_ver): the tap past the border reads
    the replicated last column / row (emu_edge, recon.rs:2052-2083), not the padding."""
    from rav1d_amd import INTRA_DTYPE
    rng = np.random.default_rng(17 + bpc)
    dt = np.uint8 if bpc == 8 else np.uint16
    luma = rng.integers(0, 1 << bpc, size=(64, 64)).astype(dt)
    chroma = rng.integers(0, 1 << bpc, size=(32, 48)).astype(dt)   # 8 columns of padding beyond max_w=40
    mv = lambda lx, ly: (lx * 8 & 0xFFFF) | ((ly * 8 & 0xFFFF) << 16)  # noqa: E731
    blk = np.zeros(1, INTRA_DTYPE)
    # chroma 8x8 at (32, 24) in a 40x32 area; luma mv (-1, -1): offset (-1, -1), phases 8/16
    blk[0] = (32, 24, 8, 8, 1, 96, 0, 0, 3, 0, 40, 32, 40, 32, 0, 0, mv(-1, -1))
    z = np.zeros(1, np.int16)
    out = oracle_lib.intra_blocks([luma, chroma, chroma.copy()], bpc, blk, z, np.zeros(1, np.uint8), np.zeros(8, dt))
    src = chroma.astype(np.int64)[:32, :40]
    src = np.pad(src, ((0, 1), (0, 1)), mode="edge")
    ib = 4 if bpc == 8 else 14 - bpc
    rnd = lambda v, s: (v + ((1 << s) >> 1)) >> s  # noqa: E731
    a, b = src[23:32, 31:39], src[23:32, 32:40]
    hm = rnd(16 * a + 8 * (b - a), 4 - ib)
    v = rnd(16 * hm[:-1] + 8 * (hm[1:] - hm[:-1]), 4 + ib)
    exp = np.clip(v, 0, (1 << bpc) - 1)
    assert np.array_equal(out[1][24:32, 32:40].astype(np.int64), exp)
