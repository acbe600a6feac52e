"""Seeded synthetic frame descriptors (the pass-1 outputs the GPU path consumes).

There is no CPU front-end yet, so tests and the benchmark feed the
DSP path with descriptors drawn from the distributions of SURVEY.md §8(d): transform-size
histogram of a real 4K intra frame, types uniform over each size's legal set, eob regimes
DC-only 60 % / partial 30 % / full 10 %, coefficient magnitudes inside the dequantiser's
range (|c| <= (128 << bpc) - 1, rav1d src/recon.rs decode_coefs clamp). Everything is a pure
function of (geometry, seed), so the same inputs regenerate bit-identically anywhere.
"""

import numpy as np

from . import MC_NCLASS, MCBLOCK_DTYPE, TXBLOCK_DTYPE, N_RECT_TX_SIZES

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
                   with_wht=False, packed=False):
    """Synthetic frame for the itx stage (packed: non-DC blocks as pack_coefs stores them).

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
            flags = 0
            if txtp == 0 and eob < 1:
                c = c.reshape(-1)[:1]     # a DC-only block keeps its DC alone (as the front-end stores it)
            elif packed:
                c, flags = pack_coefs(c, tx, bpc > 8)
                if flags and off % 4:
                    coef_chunks.append(np.zeros(4 - off % 4, dtype=c.dtype))
                    off += 4 - off % 4
            recs.append((off, x, y, p, tx, txtp, flags, eob))
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


def itx_device_order(blocks):
    """mi_itx_frame order: grouped by tx size (required); inside a size DC-only blocks first,
    then by plane and raster position (neighbouring blocks of a workgroup share pixel lines:
    4K10 itx 46.4 -> 43.5 us against type order). Returns (blocks, size_start)."""
    dc = (blocks["txtp"] == 0) & (blocks["eob"] < 1)
    order = np.lexsort((blocks["x"], blocks["y"], blocks["plane"], ~dc, blocks["tx"]))
    blocks = blocks[order]
    return blocks, np.searchsorted(blocks["tx"], np.arange(N_RECT_TX_SIZES + 1)).astype(np.uint32)


ITX_BANDS = 8


def itx_band_order(blocks, plane_heights):
    """mi_itx_frame_banded order: grouped by tx size, inside a size by picture band (band q =
    plane rows [q*h/8, (q+1)*h/8) of the block's plane, h = the 128-aligned plane height),
    then as itx_device_order. Returns (blocks, size_start, band_start[19][9])."""
    ph = np.asarray(plane_heights, np.int64)
    band = np.minimum(blocks["y"].astype(np.int64) * ITX_BANDS // ph[blocks["plane"]], ITX_BANDS - 1)
    dc = (blocks["txtp"] == 0) & (blocks["eob"] < 1)
    order = np.lexsort((blocks["x"], blocks["y"], blocks["plane"], ~dc, band, blocks["tx"]))
    blocks = blocks[order]
    band = band[order]
    key = blocks["tx"].astype(np.int64) * ITX_BANDS + band
    band_start = np.searchsorted(key, np.arange(N_RECT_TX_SIZES * ITX_BANDS + 1)).astype(np.uint32)
    bs = np.empty((N_RECT_TX_SIZES, ITX_BANDS + 1), np.uint32)
    for t in range(N_RECT_TX_SIZES):
        bs[t] = band_start[t * ITX_BANDS:(t + 1) * ITX_BANDS + 1]
    size_start = np.searchsorted(blocks["tx"], np.arange(N_RECT_TX_SIZES + 1)).astype(np.uint32)
    return blocks, size_start, bs


def itx_dc_runs(blocks, band_start):
    """dc_end[19][8] for mi_itx_frame_runs: the end of the DC-only run (DCT_DCT, eob < 1) that
    begins each (size, band) range of blocks in itx_band_order's order (DC-only blocks first)."""
    dc = (blocks["txtp"] == 0) & (blocks["eob"] < 1)
    dc_end = np.empty((N_RECT_TX_SIZES, ITX_BANDS), np.uint32)
    for t in range(N_RECT_TX_SIZES):
        for q in range(ITX_BANDS):
            lo, hi = int(band_start[t][q]), int(band_start[t][q + 1])
            n = int(dc[lo:hi].sum())
            assert dc[lo:lo + n].all(), "DC-only blocks must lead their band"
            dc_end[t][q] = lo + n
    return dc_end


def itx_algorithmic_bytes(blocks, bpc, zero_coefs=True, dc_defer=False):
    """sum over blocks of coefB*n_coef (+ the zeroing write) + 2*pixB*w*h,
    plus the 16-byte descriptor (n_coef: the stored coefficients, a packed block's corner). dc_defer (MI_ITX_DC_DEFER): a DC-only block writes its 4-byte
    DC-map entry per 4x4 unit instead of reading and writing its pixels."""
    pxb = 1 if bpc == 8 else 2
    cb = 2 if bpc == 8 else 4
    dims = np.array(TX_DIMS)
    w = dims[blocks["tx"], 0]
    h = dims[blocks["tx"], 1]
    ncoef = np.minimum(w, 32) * np.minimum(h, 32)
    fl = blocks["flags"].astype(np.int64)
    ncoef = np.where(fl & 0x80, (((fl >> 3) & 7) * 4 + 4) * ((fl & 7) * 4 + 4), ncoef)   # MI_TX_PACKED
    ncoef = np.where(fl & 0x40, ncoef // 2, ncoef)                                       # MI_TX_I16
    dconly = (blocks["txtp"] == 0) & (blocks["eob"] < 1)
    ncoef = np.where(dconly, 1, ncoef)
    pix = 2 * pxb * w * h
    if dc_defer:
        pix = np.where(dconly, 4 * (w // 4) * (h // 4), pix)
    per = cb * ncoef * (2 if zero_coefs else 1) + pix + 16
    return int(per.sum())


def dc_map_bytes(w, h, layout):
    """Bytes of the deferred-DC map (one 4-byte entry per 4x4 unit of the 128-aligned planes,
    rav1d_amd/csrc/common.h dc_map_geom): what mi_deblock_frame_dc reads on top of the picture."""
    aw, ah = (w + 127) & ~127, (h + 127) & ~127
    sh = 1 if layout in (1, 2) else 0
    sv = 1 if layout == 1 else 0
    n = (aw >> 2) * (ah >> 2)
    if layout:
        n += 2 * ((aw >> sh) >> 2) * ((ah >> sv) >> 2)
    return 4 * n


# ---------------------------------------------------------------------------------------
# Deblocking metadata (Av1Filter masks + level map), derived from a transform tiling the way
# rav1d's lf_mask builds them (src/lf_mask.rs:130-378): an edge at every transform-block
# boundary, filter-width index = min over the two sides of log2(tx extent / 4 px), capped at
# 2 (luma: 4/8/16) or 1 (chroma: 4/6).
# ---------------------------------------------------------------------------------------

AV1FILTER_DTYPE = np.dtype([("filter_y", "<u2", (2, 32, 3, 2)), ("filter_uv", "<u2", (2, 32, 2, 2)),
                            ("cdef_idx", "i1", (4,)), ("noskip_mask", "<u2", (16, 2))])
assert AV1FILTER_DTYPE.itemsize == 1348


def calc_eih(sharp):
    """Av1FilterLUT e/i for a sharpness (rav1d src/lf_mask.rs:608-626)."""
    e = np.zeros(64, np.uint8)
    i = np.zeros(64, np.uint8)
    for level in range(64):
        limit = level
        if sharp > 0:
            limit >>= (sharp + 3) >> 2
            limit = min(limit, 9 - sharp)
        limit = max(limit, 1)
        i[level] = limit
        e[level] = 2 * (level + 2) + limit
    return e, i


def _unit_maps(blocks, nux, nuy):
    lw = np.zeros((nuy, nux), np.int8)
    lh = np.zeros((nuy, nux), np.int8)
    sx = np.zeros((nuy, nux), bool)
    sy = np.zeros((nuy, nux), bool)
    bid = np.full((nuy, nux), -1, np.int32)
    for i, (x, y, tx) in enumerate(blocks):
        w, h = TX_DIMS[tx]
        x4, y4, w4, h4 = x >> 2, y >> 2, w >> 2, h >> 2
        lw[y4:y4 + h4, x4:x4 + w4] = int(w4).bit_length() - 1
        lh[y4:y4 + h4, x4:x4 + w4] = int(h4).bit_length() - 1
        sx[y4:y4 + h4, x4] = True
        sy[y4, x4:x4 + w4] = True
        bid[y4:y4 + h4, x4:x4 + w4] = i
    return lw, lh, sx, sy, bid


def make_lf_meta(tilings, w, h, layout, rng, sharpness=None, zero_level_frac=0.08):
    """Returns dict(level=(rows, b4_stride, 4) u8, masks=Av1Filter[sb128h, sb128w], lim_e, lim_i,
    b4_stride, sb128w, filter_y, filter_uv)."""
    ss_hor = 1 if layout in (1, 2) else 0
    ss_ver = 1 if layout == 1 else 0
    w4, h4 = (w + 3) >> 2, (h + 3) >> 2
    sb128w, sb128h = (w + 127) >> 7, (h + 127) >> 7
    b4_stride = sb128w * 32
    level = np.zeros((sb128h * 32, b4_stride, 4), np.uint8)
    masks = np.zeros((sb128h, sb128w), AV1FILTER_DTYPE)
    fy = np.zeros((sb128h, sb128w, 2, 32, 3, 2), np.uint16)
    fuv = np.zeros((sb128h, sb128w, 2, 32, 2, 2), np.uint16)
    for p, blocks in enumerate(tilings):
        luma = p == 0
        sh, sv = (0, 0) if luma else (ss_hor, ss_ver)
        nux, nuy = (w4 + sh) >> sh, (h4 + sv) >> sv
        lw, lh, sx, sy, bid = _unit_maps(blocks, nux, nuy)
        cap = 2 if luma else 1
        lwc, lhc = np.minimum(lw, cap), np.minimum(lh, cap)
        # per-block levels: slots (0, 1) for luma col/row edges, slot 1+p for chroma
        nb = len(blocks)
        lv = rng.integers(1, 64, size=(nb, 2)).astype(np.uint8)
        lv[rng.random((nb, 2)) < zero_level_frac] = 0
        valid = bid >= 0
        if luma:
            level[:nuy, :nux, 0][valid] = lv[bid[valid], 0]
            level[:nuy, :nux, 1][valid] = lv[bid[valid], 1]
        else:
            level[:nuy, :nux, 1 + p][valid] = lv[bid[valid], 0]
        csw, csh = 32 >> sh, 32 >> sv
        # column edges
        uy, ux = np.nonzero(sx & valid)
        left = np.where(ux > 0, lwc[uy, np.maximum(ux - 1, 0)], lwc[uy, ux])
        k = np.minimum(left, lwc[uy, ux]).astype(np.int64)
        X, x, Y, yy = ux // csw, ux % csw, uy // csh, uy % csh
        hb = 16 >> sv
        half, bit = yy // hb, yy % hb
        tgt = fy if luma else fuv
        flat = tgt.reshape(-1)
        shp = tgt.shape  # (sbh, sbw, 2, 32, K, 2)
        idx = np.ravel_multi_index((Y, X, np.zeros_like(Y), x, k, half), shp)
        np.bitwise_or.at(flat, idx, (1 << bit).astype(np.uint16))
        # row edges
        uy, ux = np.nonzero(sy & valid)
        up = np.where(uy > 0, lhc[np.maximum(uy - 1, 0), ux], lhc[uy, ux])
        k = np.minimum(up, lhc[uy, ux]).astype(np.int64)
        X, xx, Y, y = ux // csw, ux % csw, uy // csh, uy % csh
        hb = 16 >> sh
        half, bit = xx // hb, xx % hb
        idx = np.ravel_multi_index((Y, X, np.ones_like(Y), y, k, half), shp)
        np.bitwise_or.at(flat, idx, (1 << bit).astype(np.uint16))
    masks["filter_y"] = fy
    masks["filter_uv"] = fuv
    if sharpness is None:
        sharpness = int(rng.integers(0, 8))
    e, i = calc_eih(sharpness)
    return dict(level=level, masks=masks, lim_e=e, lim_i=i, b4_stride=b4_stride, sb128w=sb128w,
                filter_y=1, filter_uv=1 if layout != 0 else 0, sharpness=sharpness)


def make_tilings(w, h, layout, rng):
    ss_hor = 1 if layout in (1, 2) else 0
    ss_ver = 1 if layout == 1 else 0
    cw, ch = (w + ss_hor) >> ss_hor, (h + ss_ver) >> ss_ver
    out = [tile_plane(w, h, rng, sb=64)]
    if layout != 0:
        t = tile_plane(cw, ch, rng, sb=64 >> ss_hor)
        out += [t, t]
    return out


def make_mixed_texture(rng, w, h, bpc):
    """Blocky content mixing flat and textured 8x8 regions so every deblock branch fires."""
    bdmax = (1 << bpc) - 1
    base = make_texture(rng, w, h, bpc).astype(np.int64)
    amp = np.array([0, 1, 3, 8, 40]) * (bdmax // 255 + 1)
    tiles = rng.integers(0, len(amp), size=((h + 7) // 8, (w + 7) // 8))
    a = np.kron(amp[tiles], np.ones((8, 8), np.int64))[:h, :w]
    offs = np.kron(rng.integers(-20, 21, size=tiles.shape) * (bdmax // 255 + 1), np.ones((8, 8), np.int64))[:h, :w]
    smooth = (np.arange(w)[None, :] // 16 + np.arange(h)[:, None] // 16) * (bdmax // 255 + 1)
    noise = rng.integers(-1, 2, size=(h, w)) * a + rng.integers(0, 2, size=(h, w)) * (a > 0)
    img = np.where(a == 0, (bdmax // 2 + smooth % 7) + offs, base + offs + noise)
    return np.clip(img, 0, bdmax).astype(np.uint16 if bpc > 8 else np.uint8)


def add_cdef_meta(lf, rng, skip_frac=0.2, idx_unset_frac=0.1):
    """Fill cdef_idx / noskip_mask of an Av1Filter array in place and draw frame CDEF params
    within the ranges the bitstream allows (rav1d src/obu.rs cdef params: damping 3..6,
    strengths 6 bits each)."""
    m = lf["masks"]
    sbh, sbw = m.shape
    idx = rng.integers(0, 8, size=(sbh, sbw, 4)).astype(np.int8)
    idx[rng.random((sbh, sbw, 4)) < idx_unset_frac] = -1
    m["cdef_idx"] = idx
    bits = (rng.random((sbh, sbw, 16, 2, 16)) >= skip_frac)
    weights = (1 << np.arange(16)).astype(np.uint32)
    m["noskip_mask"] = (bits * weights).sum(-1).astype(np.uint16)
    ys = rng.integers(0, 64, size=8).astype(np.uint8)
    uvs = rng.integers(0, 64, size=8).astype(np.uint8)
    ys[rng.random(8) < 0.15] = 0
    uvs[rng.random(8) < 0.15] = 0
    return dict(damping=int(rng.integers(3, 7)), y_strength=ys, uv_strength=uvs)


# ---------------------------------------------------------------------------------------
# Loop-restoration units (Av1Restoration per 128x128: lr[3 planes][4 units]), with the
# parameter ranges read_restoration_info can code (rav1d src/decode.rs:3786-3838).
# ---------------------------------------------------------------------------------------

RESTUNIT_DTYPE = np.dtype([("type", "u1"), ("filter_h", "i1", (3,)), ("filter_v", "i1", (3,)),
                           ("sgr_weights", "i1", (2,))])
AV1RESTORATION_DTYPE = np.dtype([("lr", RESTUNIT_DTYPE, (3, 4))])
assert AV1RESTORATION_DTYPE.itemsize == 108
RESTORATION_NONE, RESTORATION_SWITCHABLE, RESTORATION_WIENER, RESTORATION_SGRPROJ = 0, 1, 2, 3

SGR_PARAMS = [(140, 3236), (112, 2158), (93, 1618), (80, 1438), (70, 1295), (58, 1177), (47, 1079),
              (37, 996), (30, 925), (25, 863), (0, 2589), (0, 1618), (0, 1177), (0, 925), (56, 0),
              (22, 0)]


def make_lr_meta(w, h, layout, rng, sb128=1, unit_log2=None, p_none=0.2, p_wiener=0.4):
    sbw, sbh = (w + 127) >> 7, (h + 127) >> 7
    m = np.zeros((sbh, sbw), AV1RESTORATION_DTYPE)
    u = m["lr"]  # (sbh, sbw, 3, 4)
    shape = u.shape
    r = rng.random(shape)
    typ = np.where(r < p_none, RESTORATION_NONE,
                   np.where(r < p_none + p_wiener, RESTORATION_WIENER,
                            RESTORATION_SGRPROJ + rng.integers(0, 16, size=shape)))
    u["type"] = typ
    fh = np.stack([rng.integers(-5, 11, size=shape), rng.integers(-23, 9, size=shape),
                   rng.integers(-17, 47, size=shape)], -1)
    fv = np.stack([rng.integers(-5, 11, size=shape), rng.integers(-23, 9, size=shape),
                   rng.integers(-17, 47, size=shape)], -1)
    fh[:, :, 1:, :, 0] = 0   # chroma wiener is 5-tap
    fv[:, :, 1:, :, 0] = 0
    u["filter_h"] = fh
    u["filter_v"] = fv
    sidx = np.clip(typ - RESTORATION_SGRPROJ, 0, 15)
    s0 = np.array([p[0] for p in SGR_PARAMS])[sidx]
    s1 = np.array([p[1] for p in SGR_PARAMS])[sidx]
    w0 = np.where(s0 == 0, 0, rng.integers(-96, 32, size=shape))
    w1 = np.where(s1 == 0, 95, rng.integers(-32, 96, size=shape))
    u["sgr_weights"] = np.stack([w0, w1], -1)
    m["lr"] = u
    if unit_log2 is None:
        ly = int(rng.integers(6 + sb128, 9))
        lc = max(5, ly - int(rng.integers(0, 2))) if layout == 1 else ly
        unit_log2 = (ly, lc)
    return dict(lr_mask=m, unit_size_log2=tuple(unit_log2), restore_planes=7 if layout else 1,
                sb128=sb128)


def _points(rng, nmax):
    n = int(rng.integers(0, nmax + 1))
    xs = np.sort(rng.choice(256, size=n, replace=False)) if n else np.zeros(0, int)
    return [(int(x), int(rng.integers(0, 256))) for x in xs]


def make_fg_params(rng, layout=1, force_y=True):
    """Random but codable Dav1dFilmGrainData (ranges of rav1d src/obu.rs parse_film_grain)."""
    yp = _points(rng, 14)
    if force_y and not yp:
        yp = [(0, 40), (255, 90)]
    csfl = int(layout != 0 and rng.random() < 0.25)
    uvp = [[], []] if (csfl or layout == 0) else [_points(rng, 10), _points(rng, 10)]
    lag = int(rng.integers(0, 4))
    ncy = 2 * lag * (lag + 1)
    small = lambda n: [int(v) for v in np.clip(rng.normal(0, 20, size=n), -128, 127)]
    return dict(seed=int(rng.integers(0, 1 << 16)), num_y_points=len(yp), y_points=yp,
                chroma_scaling_from_luma=csfl, num_uv_points=[len(uvp[0]), len(uvp[1])], uv_points=uvp,
                scaling_shift=int(rng.integers(8, 12)), ar_coeff_lag=lag,
                ar_coeffs_y=small(ncy) + [0] * (24 - ncy),
                ar_coeffs_uv=[small(ncy + 1) + [0] * (28 - ncy - 1) for _ in range(2)],
                ar_coeff_shift=int(rng.integers(6, 10)), grain_scale_shift=int(rng.integers(0, 4)),
                uv_mult=[int(rng.integers(-128, 128)) for _ in range(2)],
                uv_luma_mult=[int(rng.integers(-128, 128)) for _ in range(2)],
                uv_offset=[int(rng.integers(-256, 256)) for _ in range(2)],
                overlap_flag=int(rng.random() < 0.7), clip_to_restricted_range=int(rng.random() < 0.5))


def pack_coefs(c, tx, hbd=False):
    """The front-end's packed form of one block's dense coefficients (rav1d_amd/host/decode.cpp
    store_coefs, MI_TX_PACKED in include/mi_av1dsp.h): the corner of whole 4 x 4 groups holding
    every non-zero coefficient, row-major, for every block of more than 16 coefficients; hbd
    (10/12-bit, int32 arena): as int16 pairs when the corner fits (MI_TX_I16), then 4x4 blocks
    too.
    Returns (arena entries, flags); the caller starts a packed block on a 4-entry boundary."""
    w, h = TX_DIMS[tx]
    sw, sh = min(w, 32), min(h, 32)
    d = c.reshape(sw, sh)      # d[x, y]
    if sw * sh <= 16 and not (hbd and c.min() >= -32768 and c.max() <= 32767):
        return c, 0            # a 4x4 block is packed only as int16
    nzx, nzy = np.nonzero(d)
    cw = (int(nzx.max()) // 4 + 1) * 4 if nzx.size else 4
    ch = (int(nzy.max()) // 4 + 1) * 4 if nzy.size else 4
    corner = np.ascontiguousarray(d[:cw, :ch].T).reshape(-1)
    flags = 0x80 | ((cw // 4 - 1) << 3) | (ch // 4 - 1)
    if hbd and corner.min() >= -32768 and corner.max() <= 32767:
        # MI_TX_I16: int16 coefficients in the int32 arena, two per entry (little-endian)
        return corner.astype(np.int16).view(np.int32).astype(np.int64), flags | 0x40
    return corner, flags


def itx_blocks_from_tilings(tilings, bpc, rng, dc_frac=0.6, full_frac=0.1, packed=False):
    """packed: non-DC blocks stored as the front-end stores them (pack_coefs)."""
    recs, chunks, off = [], [], 0
    for p, blocks in enumerate(tilings):
        for (x, y, tx) in blocks:
            if rng.random() < dc_frac:
                txtp, regime = 0, 0
            else:
                types = tx_types(tx)
                txtp = types[int(rng.integers(len(types)))]
                regime = 2 if rng.random() < full_frac / (1 - dc_frac) else 1
            c, eob = make_coefs(rng, tx, txtp, regime, bpc)
            flags = 0
            if txtp == 0 and eob < 1:
                c = c.reshape(-1)[:1]     # a DC-only block keeps its DC alone (as the front-end stores it)
            elif packed:
                c, flags = pack_coefs(c, tx, bpc > 8)
                if flags and off % 4:
                    chunks.append(np.zeros(4 - off % 4, dtype=c.dtype))
                    off += 4 - off % 4
            recs.append((off, x, y, p, tx, txtp, flags, eob))
            chunks.append(c)
            off += c.size
    blocks = np.array(recs, dtype=TXBLOCK_DTYPE)
    coef = np.concatenate(chunks).astype(np.int16 if bpc == 8 else np.int32)
    blocks, size_start = itx_device_order(blocks)
    return blocks, size_start, coef


def make_frame(w, h, bpc=10, layout=1, seed=0x4C100001, sb128=1, with_fg=True, with_mc=False, nrefs=2,
               mv_mode="uniform", packed=False):
    """One synthetic frame's worth of post-entropy descriptors for every implemented stage,
    all derived from one transform tiling: prediction planes, itx blocks + coefficient arena,
    deblock masks/levels, CDEF indices/strengths, LR units, film-grain parameters.
    packed: the coefficient arena in the front-end's packed form (pack_coefs).
    with_mc: an inter frame — `nrefs` textured reference
    pictures and MC units whose prediction replaces the resident prediction planes."""
    rng = np.random.default_rng(seed)
    til = make_tilings(w, h, layout, rng)
    blocks, size_start, coef = itx_blocks_from_tilings(til, bpc, rng, packed=packed)
    lf = make_lf_meta(til, w, h, layout, rng)
    cd = add_cdef_meta(lf, rng)
    lr = make_lr_meta(w, h, layout, rng, sb128=sb128)
    ss_h = 1 if layout in (1, 2) else 0
    ss_v = 1 if layout == 1 else 0
    planes = [make_mixed_texture(rng, w, h, bpc)]
    if layout:
        planes += [make_mixed_texture(rng, (w + ss_h) >> ss_h, (h + ss_v) >> ss_v, bpc) for _ in range(2)]
    fg = make_fg_params(rng, layout) if with_fg else None
    fr = dict(w=w, h=h, bpc=bpc, layout=layout, planes=planes, blocks=blocks, size_start=size_start,
              coef=coef, lf=lf, cdef=cd, lr=lr, fg=fg, refs=None, mc=None)
    if with_mc:
        cw, ch = (w + ss_h) >> ss_h, (h + ss_v) >> ss_v
        fr["refs"] = [[make_texture(rng, w, h, bpc)] +
                      ([make_texture(rng, cw, ch, bpc) for _ in range(2)] if layout else [])
                      for _ in range(nrefs)]
        fr["mc"] = make_mc_units(w, h, layout, rng, nrefs=nrefs, mv_mode=mv_mode)
    return fr


def frame_bytes(w, h, bpc, layout=1):
    pxb = 1 if bpc == 8 else 2
    ss_h = 1 if layout in (1, 2) else 0
    ss_v = 1 if layout == 1 else 0
    c = ((w + ss_h) >> ss_h) * ((h + ss_v) >> ss_v) if layout else 0
    return (w * h + 2 * c) * pxb


# ---- motion compensation -------------------------------------

def partition_blocks(w, h, rng, sb=64, min_bs=8, p_split=0.55):
    """Quadtree partition of the frame into AV1-shaped inter blocks (square, 2:1 / 1:2 and
    4:1 / 1:4 as the PARTITION_H/V/H4/V4 shapes give), (x, y, bw, bh) luma pixels. Only
    blocks whose top-left lies inside the frame are emitted (as the reference decodes)."""
    out = []

    def rec(x, y, s):
        if x >= w or y >= h:
            return
        if s > min_bs and rng.random() < p_split:
            for dy in (0, s // 2):
                for dx in (0, s // 2):
                    rec(x + dx, y + dy, s // 2)
            return
        r = rng.random()
        if r < 0.6 or s < 16:
            out.append((x, y, s, s))
        elif r < 0.75:
            out.extend([(x, y, s, s // 2), (x, y + s // 2, s, s // 2)])
        elif r < 0.9:
            out.extend([(x, y, s // 2, s), (x + s // 2, y, s // 2, s)])
        elif r < 0.95 and s >= 32:
            out.extend([(x, y + k * s // 4, s, s // 4) for k in range(4)])
        elif s >= 32:
            out.extend([(x + k * s // 4, y, s // 4, s) for k in range(4)])
        else:
            out.append((x, y, s, s))

    for y in range(0, h, sb):
        for x in range(0, w, sb):
            rec(x, y, sb)
    return [b for b in out if b[0] < w and b[1] < h]


def _mc_record(x, y, bw, bh, plane, f2d, mvs, refs, comp, param, mask_off):
    return (x, y, bw, bh, plane, f2d, (mvs[0][0], mvs[1][0]), (mvs[0][1], mvs[1][1]), refs, comp, param, mask_off)


def make_mc_units(w, h, layout, rng, nrefs=2, compound_frac=0.3, mv_px=64, sb=64, min_bs=8, blocks=None,
                  mv_mode="uniform", mv_noise_px=2):
    """Inter prediction units for one frame: every block predicted from one reference (put)
    or two (compound: avg / w_avg / mask / seg, uniformly), filters uniform over the nine
    8-tap pairs and bilinear. MVs at 1/8 pel: mv_mode "uniform" draws each block's MVs
    uniformly in +-mv_px (the worst case for reference reuse);
    "coherent" gives every 64x64 superblock one motion per reference (uniform in +-mv_px) and
    each block that motion plus noise uniform in +-mv_noise_px, as real streams' spatially
    correlated motion fields look. Returns (units bucketed by plane group and shape class,
    class_start[2 * MC_NCLASS + 1], mask buffer)."""
    ss_h = 1 if layout in (1, 2) else 0
    ss_v = 1 if layout == 1 else 0
    seg_h, seg_v = (ss_h, ss_v) if layout else (0, 0)
    if blocks is None:
        blocks = partition_blocks(w, h, rng, sb=sb, min_bs=min_bs)
    luma, chroma, masks, moff = [], [], [], 0
    sb_mv = {}
    for (x, y, bw, bh) in blocks:
        f2d = int(rng.integers(0, 10))
        if mv_mode == "coherent":
            key = (x // 64, y // 64)
            if key not in sb_mv:
                sb_mv[key] = [(int(rng.integers(-8 * mv_px, 8 * mv_px + 1)), int(rng.integers(-8 * mv_px, 8 * mv_px + 1)))
                              for _ in range(2)]
            n8 = 8 * mv_noise_px
            mvs = [(m[0] + int(rng.integers(-n8, n8 + 1)), m[1] + int(rng.integers(-n8, n8 + 1))) for m in sb_mv[key]]
        else:
            mvs = [(int(rng.integers(-8 * mv_px, 8 * mv_px + 1)), int(rng.integers(-8 * mv_px, 8 * mv_px + 1)))
                   for _ in range(2)]
        cmp_ = nrefs > 1 and rng.random() < compound_frac
        if cmp_:
            r = rng.choice(nrefs, 2, replace=False)
            refs = (int(r[0]), int(r[1]))
            comp = int(rng.integers(0, 4))
            param = int(rng.integers(1, 16)) if comp == 1 else (int(rng.integers(0, 2)) << 7)
        else:
            refs, comp, param = (int(rng.integers(0, nrefs)), -1), 0, 0
        loff = 0
        if cmp_ and comp == 2:
            masks.append(rng.integers(0, 65, size=bw * bh).astype(np.uint8))
            loff, moff = moff, moff + bw * bh
        elif cmp_ and comp == 3:
            n = (bw >> seg_h) * (bh >> seg_v)
            masks.append(np.zeros(n, np.uint8))
            loff, moff = moff, moff + n
        luma.append(_mc_record(x, y, bw, bh, 0, f2d, mvs, refs, comp, param, loff))
        if layout:
            cw, ch = bw >> ss_h, bh >> ss_v
            ccomp, coff = comp, loff
            if cmp_ and comp == 2:          # chroma wedge: its own mask at chroma resolution
                masks.append(rng.integers(0, 65, size=cw * ch).astype(np.uint8))
                coff, moff = moff, moff + cw * ch
            cparam = param
            if cmp_ and comp == 3:          # chroma of SEG: mask() with the luma-written mask
                ccomp = 2
                cparam = param | MI_MC_AFTER_SEG   # (mi_mc_frame_sync waits for the SEG unit)
            for pl in (1, 2):
                chroma.append(_mc_record(x >> ss_h, y >> ss_v, cw, ch, pl, f2d, mvs, refs, ccomp, cparam, coff))
    units, class_start = mc_sort_units(np.array(luma + chroma, dtype=MCBLOCK_DTYPE))
    mask_buf = np.concatenate(masks) if masks else np.zeros(1, np.uint8)
    if mask_buf.size == 0:
        mask_buf = np.zeros(1, np.uint8)
    return units, class_start, mask_buf


MI_MC_AFTER_SEG = 0x40   # include/mi_av1dsp.h: a chroma MASK unit reading a SEG mask of the call


def mc_sync_ok(units):
    """Whether mi_mc_frame_sync may run `units`: every SEG and MASK mask offset a multiple of
    16 and every SEG unit at least 8 wide (a mask row of at least 4 bytes)."""
    cmp_ = units["ref"][:, 1] >= 0
    seg = cmp_ & (units["comp"] == 3)
    msk = cmp_ & ((units["comp"] == 2) | seg)
    return bool(((units["mask_off"][msk] % 16) == 0).all() and (units["w"][seg] >= 8).all() and (units["h"][seg] >= 8).all())


def mc_class_of(units):
    """Shape class log2(w) * 8 + log2(h) of each unit (include/mi_av1dsp.h MI_MC_NCLASS)."""
    return (np.log2(units["w"]).astype(np.int64) * 8 + np.log2(units["h"]).astype(np.int64))


def mc_sort_units(units):
    """Bucket units by (plane group, shape class) as mi_mc_frame requires: returns the
    stably sorted units and class_start[2 * MC_NCLASS + 1]."""
    grp = (units["plane"] > 0).astype(np.int64)
    key = grp * MC_NCLASS + mc_class_of(units)
    # within a class, units in 64-row picture bands (mi_mc_frame deals a class's waves to the
    # XCDs in 8 contiguous chunks: each XCD then predicts one region of the picture), inside a
    # band grouped by compound type / single-reference destination: waves stay uniform
    sub = units["comp"].astype(np.int64) + 16 * (units["ref"][:, 1] < 0)
    order = np.lexsort((sub, units["y"].astype(np.int64) >> 6, key))
    cs = np.searchsorted(key[order], np.arange(2 * MC_NCLASS + 1)).astype(np.uint32)
    return units[order], cs


def mc_split_one_grid(units):
    """Split a frame's units for mi_mc_frame_ex(MI_MC_ONE_GRID): (a) luma and every chroma unit
    that reads no mask written in the same call, one grid; (b) the chroma MASK compound units
    (chroma of SEG blocks, and wedges, which cannot be told apart from the record), a second
    call. Returns (units_a, class_start_a, units_b, class_start_b)."""
    later = (units["plane"] > 0) & (units["ref"][:, 1] >= 0) & (units["comp"] == 2)   # MI_MC_MASK
    ua, ca = mc_sort_units(units[~later])
    ub, cb = mc_sort_units(units[later])
    return ua, ca, ub, cb


def make_mc_grid_units(pw, ph, uw, uh, plane, rng, nrefs=2, compound_frac=0.5, mv_px=24):
    """A plane tiled with uw x uh units (any size 2..128, including the 4-tap w/h <= 4 cases),
    for kernel-shape coverage. Compound only where uw, uh >= 8 (as AV1); no SEG/MASK here.
    Returns (units, class_start)."""
    recs = []
    for y in range(0, ph, uh):
        for x in range(0, pw, uw):
            f2d = int(rng.integers(0, 10))
            mvs = [(int(rng.integers(-8 * mv_px, 8 * mv_px + 1)), int(rng.integers(-8 * mv_px, 8 * mv_px + 1)))
                   for _ in range(2)]
            if uw >= 8 and uh >= 8 and rng.random() < compound_frac:
                r = rng.choice(nrefs, 2, replace=False)
                comp = int(rng.integers(0, 2))
                recs.append(_mc_record(x, y, uw, uh, plane, f2d, mvs, (int(r[0]), int(r[1])), comp,
                                       int(rng.integers(1, 16)) if comp else 0, 0))
            else:
                recs.append(_mc_record(x, y, uw, uh, plane, f2d, mvs, (int(rng.integers(0, nrefs)), -1), 0, 0, 0))
    return mc_sort_units(np.array(recs, dtype=MCBLOCK_DTYPE))


def mc_algorithmic_bytes(units, bpc):
    """per unit, pixB * [sum over refs (w+7)(h+7) + w*h] (+ mask bytes)."""
    pxb = 1 if bpc == 8 else 2
    w = units["w"].astype(np.int64)
    h = units["h"].astype(np.int64)
    nref = 1 + (units["ref"][:, 1] >= 0)
    return int((pxb * (nref * (w + 7) * (h + 7) + w * h)).sum())
