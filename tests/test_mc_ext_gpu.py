"""GPU parity for the less frequent inter paths, each against the oracle's restatement:
OBMC laps (mi_mc_frame with MI_MC_OBMC_H / _V units, blend_h / blend_v), prep into the tmp
arena (MI_MC_PREP), scaled references (mi_mc_scaled), warped motion (mi_mc_warp: warp8x8 /
warp8x8t), the compound combine from intermediates (mi_mc_combine), super-resolution
(mi_superres_frame: mc.resize) and inter-intra blending (mi_ipred_blocks with MI_IPRED_II).
Bit-exact over whole allocated planes."""
import ctypes

import numpy as np
import pytest
import torch

from rav1d_amd import (COMBINE_DTYPE, IPRED_DTYPE, IPRED_II, MC_OBMC_H, MC_OBMC_V, MC_PREP, MCBLOCK_DTYPE,
                       WARP_DTYPE, frame as F)
from rav1d_amd.frame import Frame, McMeta, mc_combine, mc_frame, mc_scaled, mc_warp, superres_frame
from rav1d_amd.synth import _mc_record, make_mc_grid_units, make_texture, mc_sort_units
from tests import oracle_lib

pytestmark = pytest.mark.gpu


def textured(w, h, bpc, layout, rng):
    f = Frame(w, h, bpc, layout)
    for p in range(len(f.planes)):
        pw, ph = f.dims(p)
        f.set_plane_np(p, make_texture(rng, pw, ph, bpc))
    return f


def randomised(w, h, bpc, layout, rng):
    f = Frame(w, h, bpc, layout)
    for p in range(len(f.planes)):
        f.set_buffer_np(p, rng.integers(0, 1 << bpc, size=f.buffer_np(p).shape))
    return f


def planes(f):
    return [f.buffer_np(p) for p in range(len(f.planes))]


def assert_planes(got_frame, exp, what):
    for p, e in enumerate(exp):
        g = got_frame.buffer_np(p)
        if not np.array_equal(g, e):
            bad = np.argwhere(g != e)
            raise AssertionError(f"{what} plane {p}: {len(bad)} mismatches, first at {bad[0]}: "
                                 f"got {g[tuple(bad[0])]} exp {e[tuple(bad[0])]}")


def rand_mv(rng, px):
    return int(rng.integers(-8 * px, 8 * px + 1)), int(rng.integers(-8 * px, 8 * px + 1))


def obmc_units(w, h, layout, rng, nrefs, bs=16):
    """OBMC laps of a bs x bs luma block grid, following obmc()'s geometry (recon.rs:2205-2309):
    above laps (neighbour widths 8..64) and left laps (neighbour heights 8..64), all planes."""
    ss_h = 1 if layout in (1, 2) else 0
    ss_v = 1 if layout == 1 else 0
    above, left = [], []
    b4 = bs // 4
    for by in range(0, h, bs):
        for bx in range(0, w, bs):
            planes_ = [(0, 4, 4)] + ([(1, 4 >> ss_h, 4 >> ss_v), (2, 4 >> ss_h, 4 >> ss_v)] if layout else [])
            if by > 0:
                x4 = 0
                while x4 < b4:
                    # neighbour widths aligned to their own size (as block positions in AV1 are)
                    step4 = int(rng.choice([s for s in (2, 4, 8, 16) if ((bx >> 2) + x4) % s == 0]))
                    ow4, oh4 = min(step4, b4), min(b4, 16) >> 1
                    f2d, mv, r = int(rng.integers(0, 10)), rand_mv(rng, 20), int(rng.integers(0, nrefs))
                    for pl, hm, vm in planes_:
                        if pl and b4 * hm + b4 * vm < 16:
                            continue
                        hp = (((oh4 * 3 + 3) >> 2) * vm)
                        hu = 1 << (hp - 1).bit_length()
                        above.append(_mc_record((bx >> (ss_h if pl else 0)) + x4 * hm, by >> (ss_v if pl else 0),
                                                ow4 * hm, hu, pl, f2d, [mv, (0, 0)], (r, -1), MC_OBMC_H, vm * oh4, 0))
                    x4 += step4
            if bx > 0:
                y4 = 0
                while y4 < b4:
                    step4 = int(rng.choice([s for s in (2, 4, 8, 16) if ((by >> 2) + y4) % s == 0]))
                    ow4, oh4 = min(b4, 16) >> 1, min(step4, b4)
                    f2d, mv, r = int(rng.integers(0, 10)), rand_mv(rng, 20), int(rng.integers(0, nrefs))
                    for pl, hm, vm in planes_:
                        if pl and b4 * hm + b4 * vm < 16:
                            continue
                        left.append(_mc_record(bx >> (ss_h if pl else 0), (by >> (ss_v if pl else 0)) + y4 * vm,
                                               ow4 * hm, oh4 * vm, pl, f2d, [mv, (0, 0)], (r, -1), MC_OBMC_V, 0, 0))
                    y4 += step4
    return [mc_sort_units(np.array(u, dtype=MCBLOCK_DTYPE)) for u in (above, left)]


@pytest.mark.parametrize("bpc", [8, 10])
@pytest.mark.parametrize("layout", [1, 2, 3])
@pytest.mark.parametrize("bs", [16, 32])
def test_obmc_laps(gpu, bpc, layout, bs):
    w, h = 192, 128
    rng = np.random.default_rng(bpc * 5 + layout + bs)
    refs = [textured(w, h, bpc, layout, rng) for _ in range(2)]
    cur = randomised(w, h, bpc, layout, rng)
    init = planes(cur)
    (ua, ca), (ul, cl) = obmc_units(w, h, layout, rng, 2, bs)
    z = np.zeros(1, np.uint8)
    mc_frame(gpu, cur, refs, McMeta(ua, ca, z))
    mc_frame(gpu, cur, refs, McMeta(ul, cl, z))
    torch.cuda.synchronize()
    rp = [planes(r) for r in refs]
    exp, _ = oracle_lib.mc_frame(init, rp, bpc, layout, w, h, ua, z)
    exp, _ = oracle_lib.mc_frame(exp, rp, bpc, layout, w, h, ul, z)
    assert_planes(cur, exp, "obmc")


def test_prep_into_tmp(gpu):
    """MI_MC_PREP units write the mct intermediate (int16) at mask_off with pitch w."""
    w, h, bpc, layout = 128, 96, 10, 1
    rng = np.random.default_rng(5)
    refs = [textured(w, h, bpc, layout, rng) for _ in range(2)]
    cur = randomised(w, h, bpc, layout, rng)
    units, cs = make_mc_grid_units(w, h, 16, 8, 0, rng, compound_frac=0.0)
    units["comp"] = MC_PREP
    units["mask_off"] = np.arange(len(units), dtype=np.uint32) * 128
    units, cs = mc_sort_units(units)
    tmp = torch.zeros(len(units) * 128, dtype=torch.int16, device="cuda")
    mc_frame(gpu, cur, refs, McMeta(units, cs, np.zeros(1, np.uint8)), tmp=tmp)
    torch.cuda.synchronize()
    _, _, exp_tmp = oracle_lib.mc_frame(planes(cur), [planes(r) for r in refs], bpc, layout, w, h, units,
                                        np.zeros(1, np.uint8), tmp=np.zeros(len(units) * 128, np.int16))
    assert np.array_equal(tmp.cpu().numpy(), exp_tmp)


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("ref_scale", [(1.5, 1.5), (0.75, 0.625), (2.0, 1.25)])
def test_scaled_refs(gpu, bpc, ref_scale):
    w, h, layout = 160, 96, 1
    rng = np.random.default_rng(bpc + int(ref_scale[0] * 8))
    rw, rh = int(w * ref_scale[0]), int(h * ref_scale[1])
    refs = [textured(rw, rh, bpc, layout, rng) for _ in range(2)]
    cur = randomised(w, h, bpc, layout, rng)
    recs, off = [], 0
    for (uw, uh) in [(8, 8), (16, 8), (4, 4), (32, 16), (64, 64), (2, 4)]:
        for pl in (0, 1, 2):
            pw, ph = (w, h) if pl == 0 else (w // 2, h // 2)
            if uw > pw or uh > ph:
                continue
            for _ in range(6):
                x = int(rng.integers(0, pw // uw)) * uw
                y = int(rng.integers(0, ph // uh)) * uh
                prep = rng.random() < 0.4
                recs.append(_mc_record(x, y, uw, uh, pl, int(rng.integers(0, 10)), [rand_mv(rng, 30), (0, 0)],
                                       (int(rng.integers(0, 2)), -1), MC_PREP if prep else 0, 0, off if prep else 0))
                off += uw * uh if prep else 0
    # puts may overlap: keep the last writer only by making put rectangles disjoint per plane
    units = np.array(recs, dtype=MCBLOCK_DTYPE)
    keep, seen = [], set()
    for i, u in enumerate(units):
        key = (int(u["plane"]), int(u["x"]) // 64, int(u["y"]) // 64)
        if u["comp"] == MC_PREP or key not in seen:
            keep.append(i)
            if u["comp"] != MC_PREP:
                seen.add(key)
    units = units[keep]
    tmp = torch.zeros(max(off, 1), dtype=torch.int16, device="cuda")
    init = planes(cur)
    mc_scaled(gpu, cur, refs, units, tmp)
    torch.cuda.synchronize()
    exp, exp_tmp = oracle_lib.mc_scaled_frame(init, [planes(r) for r in refs], [(rw, rh)] * 2, bpc, layout, w, h,
                                              units, np.zeros(max(off, 1), np.int16))
    assert_planes(cur, exp, "scaled")
    assert np.array_equal(tmp.cpu().numpy(), exp_tmp)


def warp_blocks(pw, ph, plane, rng, n, prep_frac=0.5):
    recs, off = [], 0
    cells = rng.permutation((pw // 8) * (ph // 8))[:n]
    for c in cells:
        x, y = int(c % (pw // 8)) * 8, int(c // (pw // 8)) * 8
        abcd = [int(v) for v in rng.integers(-1024, 1025, size=4)]
        mvx, mvy = int(rng.integers(0, 1 << 16)), int(rng.integers(0, 1 << 16))
        mx = (mvx - abcd[0] * 4 - abcd[1] * 7) & ~0x3f
        my = (mvy - abcd[2] * 4 - abcd[3] * 4) & ~0x3f
        dx = x + int(rng.integers(-24, 25)) - 4
        dy = y + int(rng.integers(-24, 25)) - 4
        prep = int(rng.random() < prep_frac)
        recs.append((x, y, plane, int(rng.integers(0, 2)), prep, 0, dx, dy, mx, my, abcd, off if prep else 0, 8, 0))
        off += 64 if prep else 0
    return np.array(recs, dtype=WARP_DTYPE), off


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [1, 3])
def test_warp(gpu, bpc, layout):
    w, h = 128, 96
    rng = np.random.default_rng(bpc * 3 + layout)
    refs = [textured(w, h, bpc, layout, rng) for _ in range(2)]
    cur = randomised(w, h, bpc, layout, rng)
    blocks, offs = [], 0
    for pl in (0, 1, 2):
        pw, ph = cur.dims(pl)
        b, n = warp_blocks(pw, ph, pl, rng, 40)
        b["tmp_off"] += offs
        blocks.append(b)
        offs += n
    blocks = np.concatenate(blocks)
    tmp = torch.zeros(max(offs, 1), dtype=torch.int16, device="cuda")
    init = planes(cur)
    mc_warp(gpu, cur, refs, blocks, tmp)
    torch.cuda.synchronize()
    exp, exp_tmp = oracle_lib.mc_warp_frame(init, [planes(r) for r in refs], bpc, layout, w, h, blocks,
                                            np.zeros(max(offs, 1), np.int16))
    assert_planes(cur, exp, "warp")
    assert np.array_equal(tmp.cpu().numpy(), exp_tmp)


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
def test_combine(gpu, bpc, layout):
    w, h = 128, 64
    rng = np.random.default_rng(bpc * 11 + layout)
    cur = randomised(w, h, bpc, layout, rng)
    ss_h = 1 if layout in (1, 2) else 0
    ss_v = 1 if layout == 1 else 0
    msh, msv = (ss_h, ss_v) if layout else (0, 0)
    recs, toff, moff, masks = [], 0, 0, []
    lo, hi = (-(1 << 12), 1 << 12) if bpc == 8 else (-8192, (1 << 14) - 8192)
    for by in range(0, h, 16):
        for bx in range(0, w, 16):
            comp = int(rng.integers(0, 4))
            uw, uh = 16, 16
            param = int(rng.integers(1, 16)) if comp == 1 else int(rng.integers(0, 2)) << 7
            mo = moff
            if comp == 2:
                masks.append(rng.integers(0, 65, size=uw * uh).astype(np.uint8))
                moff += uw * uh
            elif comp == 3:
                masks.append(np.zeros((uw >> msh) * (uh >> msv), np.uint8))
                moff += (uw >> msh) * (uh >> msv)
            recs.append((bx, by, uw, uh, 0, comp, param, (0, 0, 0), (toff, toff + uw * uh), mo))
            toff += 2 * uw * uh
    units = np.array(recs, dtype=COMBINE_DTYPE)
    tmp_np = rng.integers(lo, hi, size=toff).astype(np.int16)
    masks_np = np.concatenate(masks) if masks else np.zeros(1, np.uint8)
    tmp = torch.from_numpy(tmp_np).cuda()
    mdev = torch.from_numpy(masks_np.copy()).cuda()
    init = planes(cur)
    mc_combine(gpu, cur, units, tmp, mdev)
    torch.cuda.synchronize()
    exp, exp_m = oracle_lib.mc_combine_frame(init, bpc, layout, units, tmp_np, masks_np)
    assert_planes(cur, exp, "combine")
    assert np.array_equal(mdev.cpu().numpy(), exp_m)


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
@pytest.mark.parametrize("widths", [(200, 300), (128, 256), (347, 401)])
def test_superres(gpu, bpc, layout, widths):
    sw, dw = widths
    h = 40
    rng = np.random.default_rng(bpc + layout + sw)
    src = textured(sw, h, bpc, layout, rng)
    dst = randomised(dw, h, bpc, layout, rng)
    init = planes(dst)
    superres_frame(gpu, src, dst)
    torch.cuda.synchronize()
    exp = oracle_lib.superres_frame(planes(src), init, bpc, layout, sw, dw, h)
    assert_planes(dst, exp, "superres")


@pytest.mark.parametrize("bpc", [8, 10])
def test_interintra_blend(gpu, bpc):
    """MI_IPRED_II: intra prediction blended into the inter pixels (mc.blend) with the mask."""
    from rav1d_amd.ipred_synth import EDGE_SPAN
    w, h, layout = 128, 128, 1
    rng = np.random.default_rng(77 + bpc)
    cur = randomised(w, h, bpc, layout, rng)
    dt = np.uint8 if bpc == 8 else np.uint16
    recs, edges, masks = [], [], []
    moff = 0
    sizes = [(8, 8), (16, 16), (32, 32), (8, 32), (32, 8), (16, 8)]
    y = 0
    for i, (bw, bh) in enumerate(sizes):
        mode = [0, 1, 2, 9, 3, 4][i]           # II_DC (incl. LEFT/TOP), II_V, II_H, II_SMOOTH
        e = rng.integers(0, 1 << bpc, size=EDGE_SPAN).astype(dt)
        edges.append(e)
        m = rng.integers(0, 65, size=bw * bh).astype(np.uint8)
        masks.append(m)
        recs.append((i * EDGE_SPAN + EDGE_SPAN // 2, moff, 0, y, bw, bh, 0, mode | IPRED_II, 0, 0, 0, 0, 0))
        moff += bw * bh
        y += bh if y + bh + 32 <= h else 0
        if y + bh > h:
            y = 0
    # place blocks on disjoint rows of x = 0.. (one column of blocks, wrapped into columns)
    xs, ys, cx, cy = [], [], 0, 0
    for (bw, bh) in sizes:
        if cy + bh > h:
            cx, cy = cx + 32, 0
        xs.append(cx)
        ys.append(cy)
        cy += bh
    blocks = np.array(recs, dtype=IPRED_DTYPE)
    blocks["x"], blocks["y"] = xs, ys
    edges_np = np.concatenate(edges)
    idx_np = np.concatenate(masks)
    init = planes(cur)[0].copy()
    b_dev = torch.from_numpy(blocks.view(np.uint8).copy()).cuda()
    e_dev = torch.from_numpy(edges_np.view(np.uint8).copy()).cuda()
    i_dev = torch.from_numpy(idx_np.copy()).cuda()
    F.check(F.lib().mi_ipred_blocks(gpu.h, ctypes.byref(cur.picture()), ctypes.c_void_p(b_dev.data_ptr()), len(blocks),
                                    ctypes.c_void_p(e_dev.data_ptr()), None, ctypes.c_void_p(i_dev.data_ptr()), None),
            "mi_ipred_blocks")
    torch.cuda.synchronize()
    exp = init.copy()
    for k, b in enumerate(blocks):
        bw, bh, x0, y0 = int(b["w"]), int(b["h"]), int(b["x"]), int(b["y"])
        pred = oracle_lib.intra_pred(int(b["mode"]) & 127, edges_np, int(b["edge_off"]), bw, bh, 0, 0, 0, bpc)
        exp[y0:y0 + bh, x0:x0 + bw] = oracle_lib.mc_blend(exp[y0:y0 + bh, x0:x0 + bw], pred, masks[k], bpc)
    got = cur.buffer_np(0)
    assert np.array_equal(got, exp)
