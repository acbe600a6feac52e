"""Seeded intra-prediction block sets (per-block modes, sizes, angles, edge buffers) for the
batched intra entry's parity tests and benchmark (luma modes
uniform over the 13 intra modes with angle deltas in [-3, 3], CfL for chroma)."""
import numpy as np

from . import IPRED_CFL, IPRED_DTYPE, IPRED_PAL

# AV1 directional base angles of the 8 directional luma modes (V, H, D45, D135, D113, D157,
# D203, D67), each with 7 deltas of 3 degrees
BASE_ANGLES = [90, 180, 45, 135, 113, 157, 203, 67]
EDGE_SPAN = 2 * 128 + 4          # per-block edge region (topleft at +130)
SIZES = [(4, 4), (4, 8), (8, 4), (8, 8), (8, 16), (16, 8), (16, 16), (16, 32), (32, 16), (32, 32), (32, 64),
         (64, 32), (64, 64), (4, 16), (16, 4), (8, 32), (32, 8), (16, 64), (64, 16)]


def random_angle(rng, kind):
    while True:
        a = BASE_ANGLES[int(rng.integers(0, 8))] + 3 * int(rng.integers(-3, 4))
        if kind == 6 and 0 < a < 90:
            return a
        if kind == 7 and 90 < a < 180:
            return a
        if kind == 8 and a > 180:
            return a


def make_ipred_blocks(n, bpc, rng, sizes=SIZES, modes=None, plane_w=4096):
    """n blocks laid out left to right in 64-row bands of a destination plane (no overlap)."""
    bdmax = (1 << bpc) - 1
    recs, edges, ac, idx = [], [], [], []
    x = y = 0
    for k in range(n):
        w, h = sizes[int(rng.integers(0, len(sizes)))]
        mode = int(rng.choice(modes)) if modes is not None else int(rng.integers(0, 16))
        angle = 0
        if mode in (6, 7, 8):
            angle = random_angle(rng, mode) | (int(rng.integers(0, 2)) << 9) | (int(rng.integers(0, 2)) << 10)
        elif mode == 13:
            if w > 32 or h > 32:
                w, h = min(w, 32), min(h, 32)
            angle = int(rng.integers(0, 5))
        elif mode == 14:
            mode = IPRED_CFL + int(rng.choice([0, 3, 4, 5]))
        elif mode == 15:
            mode = IPRED_PAL
        if x + w > plane_w:
            x, y = 0, y + 64
        e = rng.integers(0, bdmax + 1, size=EDGE_SPAN)
        aux = 0
        if mode >= IPRED_PAL:
            aux = sum(len(i) for i in idx)
            idx.append(rng.integers(0, 8, size=w * h).astype(np.uint8))
        elif mode >= IPRED_CFL:
            aux = sum(len(a) for a in ac)
            ac.append(rng.integers(-(bdmax << 3), (bdmax << 3) + 1, size=w * h).astype(np.int16))
        recs.append((k * EDGE_SPAN + 130, aux, x, y, w, h, 0, mode, angle,
                     int(rng.integers(1, 3 * w + 1)), int(rng.integers(1, 3 * h + 1)),
                     int(rng.integers(-16, 17)) if mode >= IPRED_CFL else 0, 0))
        edges.append(e)
        x += w
    blocks = np.array(recs, dtype=IPRED_DTYPE)
    dt = np.uint8 if bpc == 8 else np.uint16
    return (blocks, np.concatenate(edges).astype(dt),
            np.concatenate(ac) if ac else np.zeros(1, np.int16),
            np.concatenate(idx) if idx else np.zeros(1, np.uint8), y + 64)
