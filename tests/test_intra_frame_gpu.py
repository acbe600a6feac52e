"""GPU parity: a whole intra frame through mi_intra_blocks (device-side edge gathering, one
launch per dependency level) against the oracle's sequential recon_b_intra step
(prepare_intra_edges + intra_pred / cfl_pred / pal_pred per transform block, decode order).
Bit-exact over the whole allocated planes."""
import ctypes

import numpy as np
import pytest
import torch

from rav1d_amd import frame as F
from rav1d_amd.frame import Frame
from rav1d_amd.ipred_synth import make_intra_frame
from tests import oracle_lib

pytestmark = pytest.mark.gpu


def run_intra_frame(ctx, cur, fr, stream=None):
    """Upload the blocks in level order and launch one mi_intra_blocks per level."""
    blocks = fr["blocks"][fr["order"]]
    dev = torch.from_numpy(np.ascontiguousarray(blocks).view(np.uint8).copy()).cuda()
    ac = torch.from_numpy(fr["ac"].copy()).cuda()
    idx = torch.from_numpy(fr["idx"].copy()).cuda()
    pal = torch.from_numpy(fr["pal"].view(np.uint8).copy()).cuda()
    pic = cur.picture()
    ls = fr["level_start"]
    sp = F._stream_ptr(stream)
    for lv in range(len(ls) - 1):
        a, b = int(ls[lv]), int(ls[lv + 1])
        if b > a:
            F.check(F.lib().mi_intra_blocks(ctx.h, ctypes.byref(pic), ctypes.c_void_p(dev.data_ptr() + 32 * a), b - a,
                                            ctypes.c_void_p(ac.data_ptr()), ctypes.c_void_p(idx.data_ptr()),
                                            ctypes.c_void_p(pal.data_ptr()), sp), "mi_intra_blocks")
    return dev, ac, idx, pal


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
def test_intra_frame_matches_oracle(gpu, bpc, layout):
    w, h = 256, 192
    rng = np.random.default_rng(bpc * 13 + layout)
    fr = make_intra_frame(w, h, bpc, layout, rng, ii_frac=0.2)
    cur = Frame(w, h, bpc, layout)
    for p in range(len(cur.planes)):
        cur.set_buffer_np(p, rng.integers(0, 1 << bpc, size=cur.buffer_np(p).shape))
    init = [cur.buffer_np(p) for p in range(len(cur.planes))]
    run_intra_frame(gpu, cur, fr)
    torch.cuda.synchronize()
    exp = oracle_lib.intra_blocks(init, bpc, fr["blocks"], fr["ac"], fr["idx"], fr["pal"])
    for p in range(len(cur.planes)):
        got = cur.buffer_np(p)
        if not np.array_equal(got, exp[p]):
            bad = np.argwhere(got != exp[p])
            raise AssertionError(f"plane {p}: {len(bad)} mismatches, first at {bad[0]}: got {got[tuple(bad[0])]} "
                                 f"exp {exp[p][tuple(bad[0])]}")


@pytest.mark.parametrize("sb,min_bs", [(64, 8), (128, 16)])
def test_intra_frame_block_mix(gpu, sb, min_bs):
    """Large transform blocks (64x64, 4:1 shapes) and deep dependency chains."""
    w, h, bpc, layout = 384, 256, 10, 1
    rng = np.random.default_rng(sb + min_bs)
    fr = make_intra_frame(w, h, bpc, layout, rng, sb=sb, min_bs=min_bs, tx_split=0.3)
    cur = Frame(w, h, bpc, layout)
    init = [cur.buffer_np(p) for p in range(len(cur.planes))]
    run_intra_frame(gpu, cur, fr)
    torch.cuda.synchronize()
    exp = oracle_lib.intra_blocks(init, bpc, fr["blocks"], fr["ac"], fr["idx"], fr["pal"])
    for p in range(len(cur.planes)):
        assert np.array_equal(cur.buffer_np(p), exp[p]), f"plane {p}"


@pytest.mark.parametrize("bpc,layout", [(8, 1), (10, 1), (12, 3), (8, 0)])
def test_intra_recon_with_residuals(gpu, bpc, layout):
    """Full intra reconstruction (IntraFrame: per level, prediction then itx residual) vs the
    oracle's interleaved per-block predict + itxfm_add in decode order."""
    from rav1d_amd.intra import IntraFrame, make_intra_residuals
    w, h = 192, 128
    rng = np.random.default_rng(bpc * 31 + layout)
    fr = make_intra_residuals(make_intra_frame(w, h, bpc, layout, rng), bpc, rng)
    cur = Frame(w, h, bpc, layout)
    init = [cur.buffer_np(p) for p in range(len(cur.planes))]
    IntraFrame(gpu, fr).step(cur.picture())
    torch.cuda.synchronize()
    exp = [p.copy() for p in init]
    for k in range(len(fr["blocks"])):
        exp = oracle_lib.intra_blocks(exp, bpc, fr["blocks"][k:k + 1], fr["ac"], fr["idx"], fr["pal"])
        t = fr["tx_blocks"][fr["tx_of_block"][k]:fr["tx_of_block"][k] + 1]
        exp = oracle_lib.itx_frame(exp, t, fr["coef"].copy(), bpc)
    for p in range(len(cur.planes)):
        got = cur.buffer_np(p)
        if not np.array_equal(got, exp[p]):
            bad = np.argwhere(got != exp[p])
            raise AssertionError(f"plane {p}: {len(bad)} mismatches, first at {bad[0]}")


def _oracle_recon(init, fr, bpc):
    exp = [p.copy() for p in init]
    for k in range(len(fr["blocks"])):
        exp = oracle_lib.intra_blocks(exp, bpc, fr["blocks"][k:k + 1], fr["ac"], fr["idx"], fr["pal"])
        t = fr["tx_blocks"][fr["tx_of_block"][k]:fr["tx_of_block"][k] + 1]
        exp = oracle_lib.itx_frame(exp, t, fr["coef"].copy(), bpc)
    return exp


@pytest.mark.parametrize("bpc,layout,ii,granules", [(8, 1, 0.0, False), (10, 1, 0.2, False), (12, 3, 0.0, False),
                                                   (8, 0, 0.0, False), (10, 2, 0.1, False), (8, 1, 0.0, True),
                                                   (10, 1, 0.0, True), (12, 3, 0.0, True), (8, 0, 0.0, True),
                                                   (10, 2, 0.0, True)])
def test_intra_recon_fused(gpu, bpc, layout, ii, granules):
    """The persistent fused path (mi_intra_recon: one launch, per-block dependency waits,
    prediction + residual per block) vs the oracle's interleaved decode-order recon; granules:
    MI_IR_EDGE_GRANULES (edges handed over as tagged records; intra-only frames)."""
    from rav1d_amd.intra import IntraFrame, device_status, make_intra_residuals
    w, h = 256, 192
    rng = np.random.default_rng(bpc * 37 + layout)
    fr = make_intra_residuals(make_intra_frame(w, h, bpc, layout, rng, ii_frac=ii), bpc, rng)
    cur = Frame(w, h, bpc, layout)
    for p in range(len(cur.planes)):
        cur.set_buffer_np(p, rng.integers(0, 1 << bpc, size=cur.buffer_np(p).shape))
    init = [cur.buffer_np(p) for p in range(len(cur.planes))]
    intra = IntraFrame(gpu, fr)
    for rep in range(2):   # a second launch (new epoch) over the same buffers must give the same result
        for p in range(len(cur.planes)):
            cur.set_buffer_np(p, init[p])
        intra.recon(cur.picture(), granules=granules)
        device_status(gpu)
        exp = _oracle_recon(init, fr, bpc)
        for p in range(len(cur.planes)):
            got = cur.buffer_np(p)
            if not np.array_equal(got, exp[p]):
                bad = np.argwhere(got != exp[p])
                raise AssertionError(f"rep {rep} plane {p}: {len(bad)} mismatches, first at {bad[0]}")


@pytest.mark.parametrize("nframes,granules", [(8, False), (19, False), (19, True)])
def test_intra_recon_fused_multi_frame(gpu, nframes, granules):
    """Several different frames in one launch (frame f on XCD f % 8; 19 frames: XCDs serving
    two and three frames), large blocks and deep chains, coefficients zeroed after use (the
    itxfm_add contract)."""
    from rav1d_amd.intra import IntraFrame, device_status, intra_recon, make_intra_residuals
    w, h, bpc, layout = 320, 192, 10, 1
    frames, curs, inits, frs = [], [], [], []
    for f in range(nframes):
        rng = np.random.default_rng(1000 + f)
        fr = make_intra_residuals(make_intra_frame(w, h, bpc, layout, rng, sb=64 if f % 2 else 128,
                                                   min_bs=8 if f % 2 else 16, tx_split=0.3), bpc, rng)
        cur = Frame(w, h, bpc, layout)
        inits.append([cur.buffer_np(p) for p in range(len(cur.planes))])
        frs.append(fr)
        frames.append(IntraFrame(gpu, fr))
        curs.append(cur)
    intra_recon(gpu, [(frames[f], curs[f].picture()) for f in range(nframes)], keep_coefs=False, granules=granules)
    device_status(gpu)
    for f in range(nframes):
        exp = _oracle_recon(inits[f], frs[f], bpc)
        for p in range(3):
            assert np.array_equal(curs[f].buffer_np(p), exp[p]), f"frame {f} plane {p}"
        assert int(torch.count_nonzero(frames[f].coef)) == 0, f"frame {f}: coefficients not zeroed"


@pytest.mark.parametrize("granules", [False, True])
def test_intra_recon_bench_1080p8(gpu, granules):
    """The exact workload bench.py times for configs[1]: 1080p 8-bit 4:2:0 intra frames from the
    four bench descriptor seeds (0x1A7A0001 + k), cycled through a 24-frame batch in one
    persistent launch, coefficients zeroed as consumed (itxfm_add contract). Every frame is
    compared with the oracle's decode-order reconstruction, and the device status must be 0."""
    from rav1d_amd.intra import IntraFrame, device_status, intra_recon, make_intra_residuals
    w, h, bpc, nframes, ndesc = 1920, 1080, 8, 24, 4
    frs = []
    for k in range(ndesc):
        rng = np.random.default_rng(0x1A7A0001 + k)
        frs.append(make_intra_residuals(make_intra_frame(w, h, bpc, 1, rng), bpc, rng))
    intras = [IntraFrame(gpu, frs[f % ndesc]) for f in range(nframes)]   # one coefficient arena per frame
    curs = [Frame(w, h, bpc, 1) for _ in range(nframes)]
    init = [curs[0].buffer_np(p) for p in range(3)]
    intra_recon(gpu, [(intras[f], curs[f].picture()) for f in range(nframes)], keep_coefs=False, granules=granules)
    device_status(gpu)
    for k in range(ndesc):
        fr = frs[k]
        exp, arena = oracle_lib.intra_recon(init, bpc, fr["blocks"], fr["tx_blocks"][fr["tx_of_block"]], fr["ac"],
                                            fr["idx"], fr["pal"], fr["coef"])
        assert not arena.any()
        for f in range(k, nframes, ndesc):
            for p in range(3):
                got = curs[f].buffer_np(p)
                if not np.array_equal(got, exp[p]):
                    bad = np.argwhere(got != exp[p])
                    raise AssertionError(f"frame {f} plane {p}: {len(bad)} mismatches, first at {bad[0]}")
            assert int(torch.count_nonzero(intras[f].coef)) == 0, f"frame {f}: coefficients not zeroed"


@pytest.mark.parametrize("bpc,layout", [(8, 1), (10, 2), (12, 3)])
def test_intra_recon_block_copy_heavy(gpu, bpc, layout):
    """Intra block copy at a high rate, with sources hugging the right / bottom border (the
    half-pel chroma tap past the reference area replicates its border, as emu_edge): both the
    per-level and the persistent path against the oracle, and the frame must hold block copies
    with both chroma phases non-zero."""
    from rav1d_amd.intra import IntraFrame, device_status, make_intra_residuals
    w, h = 256, 192
    rng = np.random.default_rng(4242 + bpc + layout)
    fr = make_intra_residuals(make_intra_frame(w, h, bpc, layout, rng, ibc_frac=0.6, cfl_dev_frac=0.2), bpc, rng)
    b = fr["blocks"]
    ibc = b[b["mode"] == 96]
    assert len(ibc) > 20
    if layout != 3:
        mvx = (ibc["reserved"] & 0xFFFF).astype(np.int16)
        assert ((ibc["plane"] > 0) & ((mvx & 15) != 0)).any(), "no half-pel chroma block copy"
    init_cur = Frame(w, h, bpc, layout)
    init = [init_cur.buffer_np(p) for p in range(len(init_cur.planes))]
    exp, _ = oracle_lib.intra_recon(init, bpc, b, fr["tx_blocks"][fr["tx_of_block"]], fr["ac"], fr["idx"], fr["pal"],
                                    fr["coef"])
    intra = IntraFrame(gpu, fr)
    for fused in (False, True, "granules"):
        cur = Frame(w, h, bpc, layout)
        if fused:
            intra.recon(cur.picture(), granules=fused == "granules")
            device_status(gpu)
        else:
            intra.step(cur.picture())
            torch.cuda.synchronize()
        for p in range(len(cur.planes)):
            got = cur.buffer_np(p)
            if not np.array_equal(got, exp[p]):
                bad = np.argwhere(got != exp[p])
                raise AssertionError(f"fused={fused} plane {p}: {len(bad)} mismatches, first at {bad[0]}")


@pytest.mark.parametrize("granules", [False, True])
def test_intra_recon_12bit_identity32_saturates(gpu, granules):
    """12 bpc identity transforms on 32-point columns with every coefficient at the row clip:
    the column pass's identity32 (x4, unclipped, itx_1d.rs:1106-1121) drives (c + 8) >> 4 to
    +32768, one past int16. The fused kernel keeps the residual in int16 LDS,
    so it must saturate rather than wrap (a wrapped +32768 turns a pixel that clips to 4095
    into 0: Argon 12-bit test15549_5522_4902). Negative blocks reach -32768 exactly."""
    from rav1d_amd.intra import IntraFrame, device_status, make_intra_residuals
    from rav1d_amd.synth import TX_DIMS
    w, h, bpc, layout = 256, 192, 12, 3
    rng = np.random.default_rng(0x12B1D)
    fr = make_intra_residuals(make_intra_frame(w, h, bpc, layout, rng, sb=64, min_bs=8, tx_split=0.2), bpc, rng)
    cf_max = (128 << bpc) - 1
    tb, coef = fr["tx_blocks"], fr["coef"]
    hit = set()
    for k in range(len(tb)):
        tw, th = TX_DIMS[int(tb[k]["tx"])]
        if th != 32 or tw < 8 or tw > 32:   # (64-wide sizes take DCT_DCT only)
            continue
        n = min(tw, 32) * 32
        off = int(tb[k]["coef_off"])
        sign = 1 if k % 3 else -1
        coef[off:off + n] = sign * cf_max
        tb[k]["txtp"] = 9          # IDTX
        tb[k]["eob"] = n - 1
        hit.add((tw, th))
    assert {(32, 32), (8, 32), (16, 32)} <= hit, f"sizes covered: {sorted(hit)}"
    cur = Frame(w, h, bpc, layout)
    for p in range(len(cur.planes)):
        cur.set_buffer_np(p, rng.integers(0, 1 << bpc, size=cur.buffer_np(p).shape))
    init = [cur.buffer_np(p) for p in range(len(cur.planes))]
    IntraFrame(gpu, fr).recon(cur.picture(), granules=granules)
    device_status(gpu)
    exp = _oracle_recon(init, fr, bpc)
    for p in range(len(cur.planes)):
        got = cur.buffer_np(p)
        if not np.array_equal(got, exp[p]):
            bad = np.argwhere(got != exp[p])
            raise AssertionError(f"plane {p}: {len(bad)} mismatches, first at {bad[0]}: got {got[tuple(bad[0])]} "
                                 f"exp {exp[p][tuple(bad[0])]}")
