"""Seeded synthetic frame descriptors (the pass-1 outputs the GPU path consumes).

There is no CPU front-end yet, so tests and the benchmark feed the
DSP path with descriptors drawn from the distributions of SURVEY.md §8(d): transform-size
histogram of a real 4K intra frame, types uniform over each size's legal set, eob regimes
DC-only 60 % / partial 30 % / full 10 %, coefficient magnitudes inside the dequantiser's
range (|c| <= (128 << bpc) - 1, rav1d src/recon.rs decode_coefs clamp). Everything is a pure
function of (geometry, seed), so the same inputs regenerate bit-identically anywhere.
"""
import numpy as np

from . import TXBLOCK_DTYPE, N_RECT_TX_SIZES

# RectTxfmSize (rav1d src/levels.rs:46-82): (w, h)
TX_DIMS = [(4, 4), (8, 8), (16, 16), (32, 32), (64, 64), (4, 8), (8, 4), (8, 16), (16, 8),
           (16, 32), (32, 16), (32, 64), (64, 32), (4, 16), (16, 4), (8, 32), (32, 8),
           (16, 64), (64, 16)]
TX_BY_DIMS = {d: i for i, d in enumerate(TX_DIMS)}


def tx_types(tx):
    """Legal TxfmType values per size (rav1d src/itx.rs:400-457)."""
    w, h = TX_DIMS[tx]
    m = max(w, h)
    if m == 64:
        return [0]
    if m == 32:
        return [0, 9]
    if w == 16 and h == 16:
        return list(range(12))
    return list(range(16))


# Per square region size: weights of (stop with square, stop with rect tiles, split).
_REGION_P = {64: (0.06, 0.10, 0.84), 32: (0.10, 0.30, 0.60), 16: (0.18, 0.10, 0.72),
             8: (0.40, 0.06, 0.54), 4: (1.0, 0.0, 0.0)}


def _rects_in(s):
    out = []
    for (w, h) in TX_DIMS:
        if w != h and max(w, h) == s:
            out.append((w, h))
    return out


def tile_plane(pw, ph, rng, sb=64):
    """Tile a pw x ph plane with transform blocks; returns list of (x, y, tx)."""
    blocks = []

    def rec(x, y, s):
        if x >= pw or y >= ph:
            return
        fits = x + s <= pw and y + s <= ph
        p_sq, p_rect, p_split = _REGION_P[s]
        rects = _rects_in(s)
        if s == 4:
            if fits:
                blocks.append((x, y, 0))
            return
        r = rng.random()
        if fits and r < p_sq:
            blocks.append((x, y, TX_BY_DIMS[(s, s)]))
            return
        if fits and rects and r < p_sq + p_rect:
            w, h = rects[rng.integers(len(rects))]
            for yy in range(y, y + s, h):
                for xx in range(x, x + s, w):
                    blocks.append((xx, yy, TX_BY_DIMS[(w, h)]))
            return
        h2 = s // 2
        for dy in (0, h2):
            for dx in (0, h2):
                rec(x + dx, y + dy, h2)

    for y in range(0, ph, sb):
        for x in range(0, pw, sb):
            rec(x, y, sb)
    return blocks


def make_coefs(rng, tx, txtp, eob_regime, bpc):
    """Column-major (height min(h,32)) coefficients for one block + its eob."""
    w, h = TX_DIMS[tx]
    sw, sh = min(w, 32), min(h, 32)
    cf_max = (128 << bpc) - 1
    c = np.zeros((sw, sh), dtype=np.int64)       # c[x, y] -> arena[y + x*sh]
    amp = (1 << bpc) * 4
    if eob_regime == 0:                          # DC only
        c[0, 0] = int(rng.normal(0, amp))
        eob = 0
    else:
        if eob_regime == 1:                      # partial: low-frequency corner
            nx, ny = int(rng.integers(1, sw + 1)), int(rng.integers(1, sh + 1))
            nx, ny = max(1, nx // 2), max(1, ny // 2)
        else:
            nx, ny = sw, sh
        xs = np.arange(nx)[:, None]
        ys = np.arange(ny)[None, :]
        decay = 1.0 / (1.0 + 0.7 * (xs + ys))
        vals = rng.normal(0, 1, size=(nx, ny)) * amp * decay
        vals[rng.random((nx, ny)) < 0.35] = 0
        c[:nx, :ny] = np.rint(vals).astype(np.int64)
        eob = int(rng.integers(1, nx * ny + 1)) if nx * ny > 1 else int(rng.integers(0, 2))
    c = np.clip(c, -cf_max - 1, cf_max)
    return c.reshape(-1), eob   # reshape of (sw, sh) row-major == y + x*sh order


def make_texture(rng, w, h, bpc):
    bdmax = (1 << bpc) - 1
    yy, xx = np.mgrid[0:h, 0:w]
    base = (np.sin(xx / 37.0) + np.cos(yy / 23.0)) * 0.25 + 0.5
    noise = rng.integers(-64, 65, size=(h, w)) * (bdmax / 1023.0)
    return np.clip(base * bdmax + noise, 0, bdmax).astype(np.uint16 if bpc > 8 else np.uint8)


def make_itx_frame(w, h, bpc=10, layout=1, seed=0x1D1C0001, dc_frac=0.6, full_frac=0.1,
                   with_wht=False):
    """Synthetic frame for the itx stage.

    Returns dict(blocks=structured array sorted by size/type (device order),
    size_start=20 offsets, coef=arena (int16/int32, decode order), planes=[Y,U,V] numpy
    prediction planes, w, h, bpc, layout).
    """
    rng = np.random.default_rng(seed)
    ss_hor = 1 if layout in (1, 2) else 0
    ss_ver = 1 if layout == 1 else 0
    cw, ch = (w + ss_hor) >> ss_hor, (h + ss_ver) >> ss_ver
    plane_dims = [(w, h), (cw, ch), (cw, ch)] if layout != 0 else [(w, h)]
    recs = []
    coef_chunks = []
    off = 0
    for p, (pw, ph) in enumerate(plane_dims):
        sb = 64 if p == 0 else 64 >> ss_hor
        for (x, y, tx) in tile_plane(pw, ph, rng, sb=sb):
            r = rng.random()
            if with_wht and tx == 0 and rng.random() < 0.1:
                txtp, regime = 16, 2
            elif r < dc_frac:
                txtp, regime = 0, 0
            else:
                types = tx_types(tx)
                txtp = types[int(rng.integers(len(types)))]
                regime = 2 if rng.random() < full_frac / (1 - dc_frac) else 1
            c, eob = make_coefs(rng, tx, txtp, regime, bpc)
            if txtp == 16:
                c = np.clip(c // 64, -(1 << (bpc + 2)), (1 << (bpc + 2)))
            recs.append((off, x, y, p, tx, txtp, 0, eob))
            coef_chunks.append(c)
            off += c.size
    blocks = np.array(recs, dtype=TXBLOCK_DTYPE)
    cdt = np.int16 if bpc == 8 else np.int32
    coef = np.concatenate(coef_chunks).astype(cdt)
    order = np.lexsort((blocks["coef_off"], blocks["eob"] > 0, blocks["txtp"], blocks["tx"]))
    blocks = blocks[order]
    size_start = np.searchsorted(blocks["tx"], np.arange(N_RECT_TX_SIZES + 1)).astype(np.uint32)
    planes = [make_texture(rng, pw, ph, bpc) for (pw, ph) in plane_dims]
    return dict(blocks=blocks, size_start=size_start, coef=coef, planes=planes, w=w, h=h,
                bpc=bpc, layout=layout)


def itx_algorithmic_bytes(blocks, bpc, zero_coefs=True):
    """sum over blocks of coefB*n_coef (+ the zeroing write) + 2*pixB*w*h,
    plus the 16-byte descriptor."""
    pxb = 1 if bpc == 8 else 2
    cb = 2 if bpc == 8 else 4
    dims = np.array(TX_DIMS)
    w = dims[blocks["tx"], 0]
    h = dims[blocks["tx"], 1]
    ncoef = np.minimum(w, 32) * np.minimum(h, 32)
    dconly = (blocks["txtp"] == 0) & (blocks["eob"] < 1)
    ncoef = np.where(dconly, 1, ncoef)
    per = cb * ncoef * (2 if zero_coefs else 1) + 2 * pxb * w * h + 16
    return int(per.sum())
