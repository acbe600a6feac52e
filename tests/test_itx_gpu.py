"""GPU parity: the HIP itx path vs the oracle restatement, bit-exact.

Follows the reference's checkasm pattern (tests/checkasm/itx.c:131-302): identical random
but valid inputs through both implementations, compare destination pixels and the zeroed
coefficient buffer.
"""
import numpy as np
import pytest
import torch

from rav1d_amd import ITX_KEEP_COEFS, lib
from rav1d_amd.frame import Frame, itx_frame
from rav1d_amd.synth import TX_DIMS, itx_band_order, itx_dc_runs, make_coefs, make_itx_frame, tx_types
from tests import oracle_lib
from tests.oracle_lib import ptr

pytestmark = pytest.mark.gpu


def run_frame(gpu, fr, flags=0, banded=False, runs=False):
    f = Frame(fr["w"], fr["h"], fr["bpc"], fr["layout"])
    for p, arr in enumerate(fr["planes"]):
        f.set_plane_np(p, arr)
    blk, bands, dc_end = fr["blocks"], None, None
    if banded or runs:
        ah = (fr["h"] + 127) & ~127
        blk, _, bands = itx_band_order(blk, [ah, ah >> 1, ah >> 1])
        if runs:
            dc_end = itx_dc_runs(blk, bands)
    blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
    coef = torch.from_numpy(fr["coef"].copy()).cuda()
    itx_frame(gpu, f, blocks, fr["size_start"], coef, flags, band_start=bands, dc_end=dc_end)
    torch.cuda.synchronize()
    return [f.plane_np(p) for p in range(len(fr["planes"]))], coef.cpu().numpy()


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("seed", [1, 2])
def test_itx_frame_matches_oracle(gpu, bpc, seed):
    fr = make_itx_frame(256, 192, bpc=bpc, seed=seed, with_wht=(seed == 2))
    got, coef_after = run_frame(gpu, fr)
    ref_planes = [p.copy() for p in fr["planes"]]
    ref_coef = fr["coef"].copy()
    ref = oracle_lib.itx_frame(ref_planes, fr["blocks"], ref_coef, bpc)
    for p in range(3):
        assert np.array_equal(got[p], ref[p]), f"plane {p} differs"
    assert not coef_after.any() and not ref_coef.any()


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("path", ["plain", "banded", "runs"])
def test_itx_packed_blocks_match_dense(gpu, bpc, path):
    """MI_TX_PACKED: the front-end's packed corners give the pixels of the dense arena, consume
    exactly the packed entries, and agree with the oracle (which expands them)."""
    kw = dict(bpc=bpc, seed=40 + bpc, with_wht=True)
    dense, packed = make_itx_frame(640, 360, **kw), make_itx_frame(640, 360, packed=True, **kw)
    fl = packed["blocks"]["flags"]
    assert (fl & 0x80).any() and packed["coef"].size < dense["coef"].size
    if bpc > 8:   # int16 corners (MI_TX_I16) in the int32 arena; at 12 bits int32 ones too
        assert (fl & 0x40).any() and (bpc == 10 or ((fl & 0xc0) == 0x80).any())
    opts = dict(banded=path == "banded", runs=path == "runs")
    got_d, _ = run_frame(gpu, dense, **opts)
    got_p, coef_after = run_frame(gpu, packed, **opts)
    ref_coef = packed["coef"].copy()
    ref = oracle_lib.itx_frame([p.copy() for p in packed["planes"]], packed["blocks"], ref_coef, bpc)
    for p in range(3):
        assert np.array_equal(got_p[p], got_d[p]), f"plane {p}: packed != dense"
        assert np.array_equal(got_p[p], ref[p]), f"plane {p}: packed != oracle"
    assert not coef_after.any() and not ref_coef.any()


def test_itx_packed_flags_rejected(gpu):
    """a packed corner larger than the block's stored coefficients, or a reserved flag bit, is
    skipped and reported (the context's device status -EINVAL), as any illegal descriptor"""
    from rav1d_amd.frame import _stream_ptr
    for bad, bpc in ((0x80 | (7 << 3) | 7, 10), (0x40, 10), (0xc0, 8)):
        fr = make_itx_frame(64, 64, bpc=bpc, seed=8)
        blk = fr["blocks"].copy()
        k = int(np.nonzero((blk["tx"] == 0) & (blk["txtp"] != 0))[0][0])   # a 4x4 block: 16 entries only
        blk["flags"][k] = bad
        fr["blocks"] = blk
        before = [p.copy() for p in fr["planes"]]
        got, _ = run_frame(gpu, fr)
        assert lib().mi_ctx_device_status(gpu.h, _stream_ptr(None)) == -22
        x, y, p = int(blk["x"][k]), int(blk["y"][k]), int(blk["plane"][k])
        assert np.array_equal(got[p][y:y + 4, x:x + 4], before[p][y:y + 4, x:x + 4])


def test_itx_keep_coefs_flag(gpu):
    fr = make_itx_frame(128, 128, bpc=10, seed=5)
    _, coef_after = run_frame(gpu, fr, flags=ITX_KEEP_COEFS)
    assert np.array_equal(coef_after, fr["coef"])


@pytest.mark.parametrize("bpc", [8, 10])
@pytest.mark.parametrize("banded", [False, True])
def test_itx_frame_1080p_matches_oracle(gpu, bpc, banded):
    fr = make_itx_frame(1920, 1080, bpc=bpc, seed=0x1D1C0001)
    got, coef_after = run_frame(gpu, fr, banded=banded)
    ref = oracle_lib.itx_frame([p.copy() for p in fr["planes"]], fr["blocks"], fr["coef"].copy(), bpc)
    for p in range(3):
        assert np.array_equal(got[p], ref[p])
    assert not coef_after.any()


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("size", [(64, 64), (256, 192), (640, 360), (1920, 1080)])
def test_itx_runs_match_oracle(gpu, bpc, size):
    """mi_itx_frame_runs: every band's leading DC-only run on the DC path (up to 128 blocks per
    workgroup), the rest on the transform path; pixels and the zeroed arena as the oracle's."""
    w, h = size
    fr = make_itx_frame(w, h, bpc=bpc, seed=w + bpc, with_wht=True, dc_frac=0.6)
    got, coef_after = run_frame(gpu, fr, runs=True)
    ref = oracle_lib.itx_frame([p.copy() for p in fr["planes"]], fr["blocks"], fr["coef"].copy(), bpc)
    for p in range(3):
        assert np.array_equal(got[p], ref[p]), (w, h, p)
    assert not coef_after.any()


def test_itx_runs_keep_coefs_and_all_dc(gpu):
    # every block DC-only (the whole grid on the DC path), arena left untouched
    fr = make_itx_frame(640, 360, bpc=10, seed=77, dc_frac=1.0)
    got, coef_after = run_frame(gpu, fr, flags=ITX_KEEP_COEFS, runs=True)
    ref = oracle_lib.itx_frame([p.copy() for p in fr["planes"]], fr["blocks"], fr["coef"].copy(), 10)
    for p in range(3):
        assert np.array_equal(got[p], ref[p]), p
    assert np.array_equal(coef_after, fr["coef"])


def test_itx_runs_reject_bad_tables_and_report_non_dc_blocks(gpu):
    import ctypes
    from rav1d_amd.frame import _stream_ptr
    fr = make_itx_frame(256, 192, bpc=10, seed=9, dc_frac=0.6)
    ah = 256
    blk, _, bands = itx_band_order(fr["blocks"], [ah, ah >> 1, ah >> 1])
    dc_end = itx_dc_runs(blk, bands)
    f = Frame(256, 192, 10, 1)
    blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
    coef = torch.from_numpy(fr["coef"].copy()).cuda()
    pic = f.picture()
    bs = (ctypes.c_uint32 * 171)(*[int(v) for v in bands.reshape(-1)])

    def call(de):
        arr = (ctypes.c_uint32 * 152)(*[int(v) for v in de.reshape(-1)])
        return lib().mi_itx_frame_runs(gpu.h, ctypes.byref(pic), ctypes.c_void_p(blocks.data_ptr()), bs, arr,
                                       ctypes.c_void_p(coef.data_ptr()), ITX_KEEP_COEFS, _stream_ptr(None))
    t, q = np.argwhere(bands[:, 1:] > bands[:, :-1])[0]
    past = dc_end.copy()
    past[t, q] = bands[t, q + 1] + 1           # a run ending past its band
    assert call(past) == -22
    before = dc_end.copy()
    before[t, q] = bands[t, q] - 1 if bands[t, q] else 0
    if bands[t, q]:
        assert call(before) == -22
    # a run that claims the band's transform blocks too: they are skipped and reported
    t2, q2 = np.argwhere(bands[:, 1:] > dc_end)[0]
    over = dc_end.copy()
    over[t2, q2] = bands[t2, q2 + 1]
    assert call(over) == 0
    assert lib().mi_ctx_device_status(gpu.h, _stream_ptr(None)) == -22
    assert call(dc_end) == 0
    assert lib().mi_ctx_device_status(gpu.h, _stream_ptr(None)) == 0


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_itx_banded_small_frames_match_oracle(gpu, bpc):
    # bands with no blocks of a size, bands holding a single workgroup's blocks, WHT blocks
    for seed, (w, h) in enumerate([(64, 64), (256, 192), (640, 360)]):
        fr = make_itx_frame(w, h, bpc=bpc, seed=seed + 11, with_wht=True)
        got, coef_after = run_frame(gpu, fr, banded=True)
        ref = oracle_lib.itx_frame([p.copy() for p in fr["planes"]], fr["blocks"], fr["coef"].copy(), bpc)
        for p in range(3):
            assert np.array_equal(got[p], ref[p]), (w, h, p)
        assert not coef_after.any()


def test_itx_banded_rejects_malformed_band_table(gpu):
    import ctypes
    from rav1d_amd.frame import _stream_ptr
    fr = make_itx_frame(128, 128, bpc=10, seed=3)
    ah = 128
    blk, _, bands = itx_band_order(fr["blocks"], [ah, ah >> 1, ah >> 1])
    f = Frame(128, 128, 10, 1)
    blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
    coef = torch.from_numpy(fr["coef"].copy()).cuda()
    assert bands[0, 3] > 0
    pic = f.picture()
    dec = bands.copy()
    dec[0, 4] = dec[0, 3] - 1                  # a band range that runs backwards
    gap = bands.copy()
    gap[1:, :] += 1                            # size 1 does not start where size 0 ends
    for bad in (dec, gap):
        arr = (ctypes.c_uint32 * 171)(*[int(v) for v in bad.reshape(-1)])
        rc = lib().mi_itx_frame_banded(gpu.h, ctypes.byref(pic), ctypes.c_void_p(blocks.data_ptr()), arr,
                                       ctypes.c_void_p(coef.data_ptr()), 0, _stream_ptr(None))
        assert rc == -22


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_per_call_table_entries(gpu, bpc):
    """mi_dsp_itxfm_add over every (size, type) with full/partial/DC coefficients, host buffers."""
    L = lib()
    o = oracle_lib.load_oracle()
    rng = np.random.default_rng(100 + bpc)
    cdt = np.int16 if bpc == 8 else np.int32
    dt = np.uint8 if bpc == 8 else np.uint16
    for tx, (w, h) in enumerate(TX_DIMS):
        types = tx_types(tx) + ([16] if tx == 0 else [])
        for txtp in types:
            for regime in (0, 1, 2):
                if regime == 0 and txtp != 0:
                    continue
                c, eob = make_coefs(rng, tx, txtp, regime, bpc)
                if txtp == 16:
                    c = np.clip(c // 64, -(1 << (bpc + 2)), 1 << (bpc + 2))
                c = c.astype(cdt)
                d = rng.integers(0, 1 << bpc, size=(h, w + 16)).astype(dt)
                c_ref, d_ref = c.copy(), d.copy()
                o.oracle_itxfm_add(tx, txtp, ptr(d_ref), d_ref.strides[0], ptr(c_ref), eob, (1 << bpc) - 1)
                rc = L.mi_dsp_itxfm_add(tx, txtp, ptr(d), d.strides[0], ptr(c), eob, (1 << bpc) - 1)
                assert rc == 0
                assert np.array_equal(d, d_ref), (tx, txtp, regime)
                assert not c.any()


def test_per_call_rejects_bad_args(gpu):
    L = lib()
    d = np.zeros((64, 64), np.uint16)
    c = np.zeros(1024, np.int32)
    assert L.mi_dsp_itxfm_add(4, 9, ptr(d), 128, ptr(c), 0, 1023) == -22   # IDTX illegal at 64x64
    assert L.mi_dsp_itxfm_add(0, 0, ptr(d), 128, ptr(c), 0, 1000) == -22   # bad bitdepth_max
