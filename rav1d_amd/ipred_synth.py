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


def make_intra_frame(w, h, bpc, layout, rng, sb=64, min_bs=8, tx_split=0.5, pal_frac=0.05, cfl_frac=0.4,
                     filter_frac=0.1, ii_frac=0.0, edge_filter=None, cfl_dev_frac=0.5, ibc_frac=0.05):
    """A whole intra frame as MiIntraBlock transform blocks in decode order (blocks in quadtree
    z-order, luma then U then V per block, transform blocks raster within a block), with the
    edge-availability flags a decoder would pass (top-right / bottom-left only where those
    pixels are already decoded) and each block's dependency level (1 + the deepest level among
    the blocks owning any pixel its edges may read). Returns dict(blocks (decode order),
    order (indices sorted by level), level_start, ac, idx, pal, deps (per block, decode-order
    indices of those owners)). Single tile; w, h multiples
    of 64. A cfl_dev_frac share of the CfL blocks up to 32x32 take MI_INTRA_CFL_AC (the AC is
    computed on the device from the reconstructed luma; its owners join the dependencies), with
    random cfl_ac padding."""
    from . import (INTRA_BOTTOM_LEFT, INTRA_DTYPE, INTRA_EDGE_FILTER, INTRA_HAVE_LEFT, INTRA_HAVE_TOP, INTRA_II,
                   INTRA_SMOOTH_NB, INTRA_TOP_RIGHT)
    from .synth import partition_blocks
    ss_h = 1 if layout in (1, 2) else 0
    ss_v = 1 if layout == 1 else 0
    nplanes = 3 if layout else 1
    dims = [(w, h)] + [((w + ss_h) >> ss_h, (h + ss_v) >> ss_v)] * (nplanes - 1)
    owner = [np.full((ph, pw), -1, np.int64) for pw, ph in dims]
    level_of, dep_lists = [], []
    if edge_filter is None:
        edge_filter = int(rng.integers(0, 2))
    recs, ac, idx, pal = [], [], [], []
    n_ac = n_idx = n_pal = 0
    dt = np.uint8 if bpc == 8 else np.uint16
    for (bx, by, bw, bh) in partition_blocks(w, h, rng, sb=sb, min_bs=min_bs):
        for pl in range(nplanes):
            sh, sv = (ss_h, ss_v) if pl else (0, 0)
            pw, ph = dims[pl]
            px, py, pbw, pbh = bx >> sh, by >> sv, bw >> sh, bh >> sv
            tw = pbw // 2 if pbw >= 8 and rng.random() < tx_split else pbw
            th = pbh // 2 if pbh >= 8 and rng.random() < tx_split else pbh
            tw, th = min(tw, 64), min(th, 64)
            if tw * 4 < th:
                th = tw * 4
            if th * 4 < tw:
                tw = th * 4
            for ty in range(py, py + pbh, th):
                for tx in range(px, px + pbw, tw):
                    if tx >= pw or ty >= ph:
                        continue
                    own = owner[pl]
                    flags = (INTRA_HAVE_LEFT if tx > 0 else 0) | (INTRA_HAVE_TOP if ty > 0 else 0)
                    flags |= INTRA_EDGE_FILTER if edge_filter else 0
                    flags |= INTRA_SMOOTH_NB if rng.random() < 0.3 else 0
                    if ty > 0 and tx + tw < pw and (own[ty - 1, tx + tw:min(tx + 2 * tw, pw)] >= 0).all() \
                            and rng.random() < 0.85:
                        flags |= INTRA_TOP_RIGHT
                    if tx > 0 and ty + th < ph and (own[ty + th:min(ty + 2 * th, ph), tx - 1] >= 0).all() \
                            and rng.random() < 0.85:
                        flags |= INTRA_BOTTOM_LEFT
                    # CfL with the AC from the reconstructed luma (decided before the dependencies)
                    r = rng.random()
                    cfl_dev = bool(pl and pal_frac <= r < pal_frac + cfl_frac and tw <= 32 and th <= 32
                                   and rng.random() < cfl_dev_frac)
                    reserved = 0
                    # intra block copy: a luma-integer displacement up / left onto pixels already
                    # reconstructed (half-pel in subsampled chroma for odd displacements)
                    ibc = None
                    if not cfl_dev and rng.random() < ibc_frac:
                        for t_ in range(8):
                            lx, lyd = -int(rng.integers(0, 65)), -int(rng.integers(0, 65))
                            if t_ & 1:
                                # a source hugging the right / bottom border: the half-pel chroma
                                # tap reads one column / row past the reference area (emu_edge)
                                lx, lyd = (-int(rng.integers(0, 2)), lyd) if t_ & 2 else (lx, -int(rng.integers(0, 2)))
                            mvx, mvy = 8 * lx, 8 * lyd
                            sx, sy = tx + (mvx >> (3 + sh)), ty + (mvy >> (3 + sv))
                            mxp = (mvx & (15 >> (1 - sh))) << (1 - sh)
                            myp = (mvy & (15 >> (1 - sv))) << (1 - sv)
                            ex, ey = min(sx + tw + (mxp > 0), pw), min(sy + th + (myp > 0), ph)
                            if sx >= 0 and sy >= 0 and sx + tw <= pw and sy + th <= ph and \
                                    (own[sy:ey, sx:ex] >= 0).all():
                                ibc = (mvx, mvy, own[sy:ey, sx:ex].ravel())
                                break
                    # dependency level from every pixel the edge may read
                    deps = []
                    if ibc is not None:
                        deps.append(ibc[2])
                    if cfl_dev:
                        wp = int(rng.integers(0, tw // 4)) if rng.random() < 0.3 else 0
                        hp = int(rng.integers(0, th // 4)) if rng.random() < 0.3 else 0
                        reserved = wp | (hp << 8) | (ss_h << 16) | (ss_v << 17)
                        flags |= 128
                        ly0, lx0 = ty << ss_v, tx << ss_h
                        ly1 = ly0 + ((th - 4 * hp) << ss_v)
                        lx1 = lx0 + ((tw - 4 * wp) << ss_h)
                        deps.append(owner[0][ly0:ly1, lx0:lx1].ravel())
                    if tx > 0:
                        deps.append(own[ty:min(ty + 2 * th, ph), tx - 1])
                    if ty > 0:
                        deps.append(own[ty - 1, max(tx - 1, 0):min(tx + 2 * tw, pw)])
                    lv = 0
                    dep_ids = np.unique(np.concatenate(deps)) if deps else np.zeros(0, np.int64)
                    dep_ids = dep_ids[dep_ids >= 0]
                    if dep_ids.size:
                        lv = 1 + max(level_of[i] for i in dep_ids)
                    dep_lists.append(dep_ids)
                    mode, angle, filt, alpha, aux, poff = 0, 0, 0, 0, 0, 0
                    if ibc is not None:
                        mode, filt = 96, sh | (sv << 1)
                        reserved = (ibc[0] & 0xFFFF) | ((ibc[1] & 0xFFFF) << 16)
                        flags &= ~INTRA_II
                    elif r < pal_frac:
                        mode = 64
                        pal.append(rng.integers(0, 1 << bpc, size=8).astype(dt))
                        poff, n_pal = n_pal, n_pal + 8
                        idx.append(rng.integers(0, 8, size=tw * th).astype(np.uint8))
                        aux, n_idx = n_idx, n_idx + tw * th
                    elif pl and r < pal_frac + cfl_frac:
                        mode = 32
                        alpha = int(rng.integers(-16, 17))
                        ac.append(rng.integers(-400, 401, size=tw * th).astype(np.int16))
                        aux, n_ac = n_ac, n_ac + tw * th
                    elif tw <= 32 and th <= 32 and r < pal_frac + cfl_frac + filter_frac:
                        mode, filt = 13, int(rng.integers(0, 5))
                    else:
                        mode = int(rng.integers(0, 13))
                        if 1 <= mode <= 8:
                            angle = int(rng.integers(-3, 4))
                        if mode in (0, 1, 2, 9) and rng.random() < ii_frac:
                            flags |= INTRA_II
                            idx.append(rng.integers(0, 65, size=tw * th).astype(np.uint8))
                            aux, n_idx = n_idx, n_idx + tw * th
                    k = len(recs)
                    # intrabc: max_w / max_h = the reference area mc() clamps to (the plane)
                    mw, mh = (pw, ph) if mode == 96 else (pw - tx, ph - ty)
                    recs.append((tx, ty, tw, th, pl, mode, angle, flags, filt, alpha, pw, ph, mw, mh,
                                 aux, poff, reserved))
                    level_of.append(lv)
                    own[ty:ty + th, tx:tx + tw] = k
    blocks = np.array(recs, dtype=INTRA_DTYPE)
    lv = np.array(level_of, np.int64)
    order = np.argsort(lv, kind="stable")
    level_start = np.searchsorted(lv[order], np.arange(lv.max() + 2)).astype(np.int64)
    cat = lambda xs, d: np.concatenate(xs) if xs else np.zeros(1, d)  # noqa: E731
    return dict(blocks=blocks, order=order, level_start=level_start, ac=cat(ac, np.int16), idx=cat(idx, np.uint8),
                pal=cat(pal, dt), deps=dep_lists)
