"""GPU parity: frame-batched motion compensation (mi_mc_frame) vs the oracle's restatement
of recon mc() + compound dispatch, bit-exact over the whole allocated planes (units may
extend past the visible frame into the aligned area, as in the reference) and the SEG masks."""
import numpy as np
import pytest
import torch

from rav1d_amd import lib
from rav1d_amd.frame import Frame, McMeta, McSplitMeta, _stream_ptr, mc_frame, mc_frame_one_grid, mc_frame_sync
from rav1d_amd.synth import make_mc_grid_units, make_mc_units, make_texture, mc_sync_ok
from tests import oracle_lib

pytestmark = pytest.mark.gpu


def make_refs(w, h, bpc, layout, n, rng):
    refs = []
    for _ in range(n):
        f = Frame(w, h, bpc, layout)
        for p in range(len(f.planes)):
            pw, ph = f.dims(p)
            f.set_plane_np(p, make_texture(rng, pw, ph, bpc))
        refs.append(f)
    return refs


def run_case(gpu, w, h, bpc, layout, units, class_start, masks, refs, rng, one_grid=False, sync=False):
    cur = Frame(w, h, bpc, layout)
    init = [rng.integers(0, 1 << bpc, size=cur.buffer_np(p).shape) for p in range(len(cur.planes))]
    for p, a in enumerate(init):
        cur.set_buffer_np(p, a)
    if sync:
        # mi_mc_frame_sync: one grid, chroma units of SEG blocks wait for their mask in-launch
        meta = McMeta(units, class_start, masks)
        mc_frame_sync(gpu, cur, refs, meta)
        assert lib().mi_mc_sync_status(gpu.h, _stream_ptr(None)) == 0, "hand-off wait timed out"
    elif one_grid:
        # mi_mc_frame_ex(MI_MC_ONE_GRID) + the chroma MASK units in a second call
        meta = McSplitMeta(units, masks)
        mc_frame_one_grid(gpu, cur, refs, meta)
    else:
        meta = McMeta(units, class_start, masks)
        mc_frame(gpu, cur, refs, meta)
    torch.cuda.synchronize()
    ref_np = [[r.buffer_np(p) for p in range(len(r.planes))] for r in refs]
    dt = np.uint8 if bpc == 8 else np.uint16
    exp, exp_masks = oracle_lib.mc_frame([a.astype(dt) for a in init], ref_np, bpc, layout, w, h, units, masks)
    for p in range(len(cur.planes)):
        got = cur.buffer_np(p)
        if not np.array_equal(got, exp[p]):
            bad = np.argwhere(got != exp[p])
            raise AssertionError(f"plane {p}: {len(bad)} mismatches, first at {bad[0]}: "
                                 f"got {got[tuple(bad[0])]} exp {exp[p][tuple(bad[0])]}")
    assert np.array_equal(meta.masks.cpu().numpy(), exp_masks), "seg masks"


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [1, 2, 3, 0])
@pytest.mark.parametrize("size", [(256, 192), (200, 134)])
def test_mc_frame_matches_oracle(gpu, bpc, layout, size):
    w, h = size
    rng = np.random.default_rng(bpc * 7 + layout * 3 + w)
    refs = make_refs(w, h, bpc, layout, 3, rng)
    units, ps, masks = make_mc_units(w, h, layout, rng, nrefs=3, compound_frac=0.5, mv_px=40)
    run_case(gpu, w, h, bpc, layout, units, ps, masks, refs, rng)


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [1, 2, 3, 0])
def test_mc_frame_one_grid_matches_oracle(gpu, bpc, layout):
    w, h = 256, 192
    rng = np.random.default_rng(bpc * 5 + layout * 11 + 1)
    refs = make_refs(w, h, bpc, layout, 3, rng)
    units, ps, masks = make_mc_units(w, h, layout, rng, nrefs=3, compound_frac=0.5, mv_px=40)
    if layout:
        assert ((units["plane"] > 0) & (units["comp"] == 2) & (units["ref"][:, 1] >= 0)).any()
    run_case(gpu, w, h, bpc, layout, units, ps, masks, refs, rng, one_grid=True)


def test_mc_frame_ex_rejects_unknown_flags(gpu):
    from rav1d_amd import lib
    from rav1d_amd import MiPicture
    import ctypes
    cur = Frame(64, 64, 8, 1)
    cs = (ctypes.c_uint32 * 129)()
    rc = lib().mi_mc_frame_ex(gpu.h, ctypes.byref(cur.picture()), (MiPicture * 1)(cur.picture()), 1,
                              None, cs, None, None, 2, None)
    assert rc == -22


UNIT_SHAPES = [(2, 2), (2, 4), (4, 2), (4, 4), (4, 8), (8, 4), (4, 16), (16, 4), (8, 8), (8, 16), (16, 8),
               (8, 32), (32, 8), (16, 16), (16, 32), (32, 16), (16, 64), (64, 16), (32, 32), (32, 64),
               (64, 32), (64, 64), (64, 128), (128, 64), (128, 128)]


@pytest.mark.parametrize("shape", UNIT_SHAPES)
def test_mc_unit_shapes(gpu, shape):
    """Every unit geometry (incl. the 4-tap w/h <= 4 filters and 128-wide tiling) on luma."""
    uw, uh = shape
    w, h, bpc = 256, 256, 10
    rng = np.random.default_rng(uw * 131 + uh)
    refs = make_refs(w, h, bpc, 0, 2, rng)
    units, cs = make_mc_grid_units(w, h, uw, uh, 0, rng)
    run_case(gpu, w, h, bpc, 0, units, cs, np.zeros(1, np.uint8), refs, rng)


@pytest.mark.parametrize("layout", [1, 2])
def test_mc_chroma_small_shapes(gpu, layout):
    """Chroma-sized units (2xN / Nx2 under 4:2:0 / 4:2:2) mixed in one frame's chroma group."""
    w, h, bpc = 128, 128, 8
    rng = np.random.default_rng(11 + layout)
    refs = make_refs(w, h, bpc, layout, 2, rng)
    cw, ch = w >> 1, h >> (layout == 1)
    parts = [make_mc_grid_units(cw, ch // 4, uw, uh, pl, rng)[0] for pl in (1, 2)
             for (uw, uh) in [(2, 2), (4, 2)]]
    # stack the grids in disjoint row bands of the chroma planes
    from rav1d_amd.synth import mc_sort_units
    allu = []
    for k, u in enumerate(parts):
        u = u.copy()
        u["y"] += (k % 2) * (ch // 4)
        allu.append(u)
    units, cs = mc_sort_units(np.concatenate(allu))
    run_case(gpu, w, h, bpc, layout, units, cs, np.zeros(1, np.uint8), refs, rng)


def test_mc_4k10_matches_oracle(gpu):
    w, h, bpc = 3840, 2160, 10
    rng = np.random.default_rng(0x4C100001)
    refs = make_refs(w, h, bpc, 1, 2, rng)
    units, ps, masks = make_mc_units(w, h, 1, rng)
    run_case(gpu, w, h, bpc, 1, units, ps, masks, refs, rng)


@pytest.mark.parametrize("bpc", [8, 10])
@pytest.mark.parametrize("layout", [1, 2, 3])
@pytest.mark.parametrize("size", [(256, 192), (640, 384)])
def test_mc_frame_sync_matches_oracle(gpu, bpc, layout, size):
    """mi_mc_frame_sync (one grid, in-launch SEG mask hand-off) against the oracle, SEG masks
    included, with half of the blocks compound."""
    w, h = size
    rng = np.random.default_rng(bpc * 13 + layout * 5 + w)
    refs = make_refs(w, h, bpc, layout, 3, rng)
    units, ps, masks = make_mc_units(w, h, layout, rng, nrefs=3, compound_frac=0.5, mv_px=40, min_bs=8)
    assert mc_sync_ok(units)
    run_case(gpu, w, h, bpc, layout, units, ps, masks, refs, rng, sync=True)


def _sync_units(w, h, layout, seed):
    rng = np.random.default_rng(seed)
    refs = make_refs(w, h, 10, layout, 3, rng)
    units, ps, masks = make_mc_units(w, h, layout, rng, nrefs=3, compound_frac=0.5, mv_px=40, min_bs=8)
    waiting = (units["plane"] > 0) & ((units["param"] & 0x40) != 0)
    assert waiting.any(), "the case needs chroma units that wait for a SEG mask"
    return refs, units, ps, masks


def test_mc_frame_sync_timeout_reported(gpu):
    """A chroma unit flagged MI_MC_AFTER_SEG whose SEG unit is not in the call waits until its
    bound and the status calls report -ETIMEDOUT (mi_mc_sync_status and mi_ctx_device_status
    agree), then clear."""
    from rav1d_amd.synth import mc_sort_units
    w, h = 256, 192
    refs, units, _, masks = _sync_units(w, h, 1, 0x7E0)
    keep = ~((units["plane"] == 0) & (units["comp"] == 3))          # drop every luma SEG unit
    units, ps = mc_sort_units(units[keep])
    cur = Frame(w, h, 10, 1)
    meta = McMeta(units, ps, masks)
    for status in ("mi_mc_sync_status", "mi_ctx_device_status"):
        mc_frame_sync(gpu, cur, refs, meta)
        assert getattr(lib(), status)(gpu.h, _stream_ptr(None)) == -110, status    # -ETIMEDOUT
        assert lib().mi_mc_sync_status(gpu.h, _stream_ptr(None)) == 0, "status not cleared"


def test_mc_frame_sync_mask_offset_past_buffer(gpu):
    """mask_bytes smaller than the units' mask offsets: the kernel skips the flag accesses it
    cannot bound and the status reports -EINVAL (no out-of-bounds flag access)."""
    import ctypes
    from rav1d_amd import MiPicture
    w, h = 256, 192
    refs, units, ps, masks = _sync_units(w, h, 1, 0x7E1)
    assert int(units["mask_off"].max()) >= 64
    cur = Frame(w, h, 10, 1)
    meta = McMeta(units, ps, masks)
    pics = (MiPicture * len(refs))(*[r.picture() for r in refs])
    rc = lib().mi_mc_frame_sync(gpu.h, ctypes.byref(cur.picture()), pics, len(refs),
                                ctypes.c_void_p(meta.blocks.data_ptr()), meta.class_start,
                                ctypes.c_void_p(meta.masks.data_ptr()), 16, None, _stream_ptr(None))
    assert rc == 0
    assert lib().mi_mc_sync_status(gpu.h, _stream_ptr(None)) == -22     # -EINVAL
    assert lib().mi_mc_sync_status(gpu.h, _stream_ptr(None)) == 0

