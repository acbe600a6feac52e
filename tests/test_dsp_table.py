"""The slot-exact drop-in surface (include/mi_dsp_table.h): every declared slot function is
exported, and mi_fill_dsp_tables writes them into a Rav1dDSPContext-layout struct
(src/internal.rs:111-121) at the reference's slot positions, NULL where the reference's table
holds None. No GPU needed (the filler only stores pointers); the -m gpu test calls the slots
through the filled table from C (tests/c/dsp_table_check.c) against the oracle."""
import ctypes
import os
import re
import subprocess

import pytest

from rav1d_amd import LIB_PATH, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mi_dsp_table.h")
PTR = ctypes.sizeof(ctypes.c_void_p)


def declared():
    """Function names the header declares, with its X-macro lists expanded by the C preprocessor."""
    out = subprocess.run(["gcc", "-E", "-P", "-I" + os.path.join(ROOT, "include"), HDR], capture_output=True,
                         text=True, check=True).stdout
    return sorted(set(re.findall(r"\b(mi_[a-z0-9_]+)\s*\(", out)) - set(re.findall(r"\(\s*\*\s*(mi_[a-z0-9_]+)", out)))


def test_slot_functions_exported():
    L = lib()
    names = declared()
    assert len(names) > 250
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing[:10]


def _table(bpc):
    L = lib()
    L.mi_dsp_context_size.restype = ctypes.c_size_t
    n = L.mi_dsp_context_size()
    assert n == 422 * PTR        # 421 slots + the bool (padded), as Rav1dDSPContext
    buf = (ctypes.c_uint8 * n)()
    assert L.mi_fill_dsp_tables(buf, bpc) == 0
    slots = [int.from_bytes(bytes(buf[i * PTR:(i + 1) * PTR]), "little") for i in range(421)]
    return slots, buf[421 * PTR]


def _addr(name):
    return ctypes.cast(getattr(lib(), name), ctypes.c_void_p).value


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_fill_dsp_tables_layout(bpc):
    slots, initialized = _table(bpc)
    assert initialized == 1
    suf = "8bpc" if bpc == 8 else "16bpc"
    # fg (filmgrain.rs:194-199): 8 slots
    assert slots[0] == _addr("mi_generate_grain_y")
    assert slots[1:4] == [_addr(f"mi_generate_grain_uv_{s}") for s in (420, 422, 444)]
    assert slots[4] == _addr("mi_fgy_32x32xn")
    assert slots[5:8] == [_addr(f"mi_fguv_32x32xn_{s}") for s in (420, 422, 444)]
    # ipred (ipred.rs:164-169): intra_pred[14], cfl_ac[3], cfl_pred[6], pal_pred
    ip = ["dc", "v", "h", "dc_left", "dc_top", "dc_128", "z1", "z2", "z3", "smooth", "smooth_v", "smooth_h",
          "paeth", "filter"]
    assert slots[8:22] == [_addr(f"mi_ipred_{n}") for n in ip]
    assert slots[22:25] == [_addr(f"mi_ipred_cfl_ac_{s}_{suf}") for s in (420, 422, 444)]
    unimpl = _addr("mi_ipred_cfl_unimplemented")   # the reference's DefaultValue::DEFAULT slots
    assert slots[25:31] == [_addr("mi_ipred_cfl"), unimpl, unimpl, _addr("mi_ipred_cfl_left"),
                            _addr("mi_ipred_cfl_top"), _addr("mi_ipred_cfl_128")]
    assert slots[31] == _addr(f"mi_pal_pred_{suf}")
    # mc (mc.rs:1322-1338): 53 slots from 32
    f2d = ["8tap_regular", "8tap_regular_smooth", "8tap_regular_sharp", "8tap_sharp_regular", "8tap_sharp_smooth",
           "8tap_sharp", "8tap_smooth_regular", "8tap_smooth", "8tap_smooth_sharp", "bilin"]
    assert slots[32:42] == [_addr(f"mi_put_{n}") for n in f2d]
    assert slots[42:52] == [_addr(f"mi_put_{n}_scaled") for n in f2d]
    assert slots[52:62] == [_addr(f"mi_prep_{n}") for n in f2d]
    assert slots[62:72] == [_addr(f"mi_prep_{n}_scaled") for n in f2d]
    rest = ["mi_avg", "mi_w_avg", "mi_mask", "mi_w_mask_444", "mi_w_mask_422", "mi_w_mask_420", f"mi_blend_{suf}",
            f"mi_blend_v_{suf}", f"mi_blend_h_{suf}", "mi_warp_affine_8x8", "mi_warp_affine_8x8t",
            f"mi_emu_edge_{suf}", "mi_resize"]
    assert slots[72:85] == [_addr(n) for n in rest]
    # itx (itx.rs:194-196): [19][17] from 85; 156 filled (itx.rs:1072-1110)
    itx = slots[85:85 + 19 * 17]
    assert sum(1 for v in itx if v) == 156
    assert itx[0 * 17 + 0] == _addr("mi_inv_txfm_add_dct_dct_4x4")
    assert itx[0 * 17 + 16] == _addr("mi_inv_txfm_add_wht_wht_4x4")
    assert itx[2 * 17 + 1] == _addr("mi_inv_txfm_add_dct_adst_16x16")     # ADST_DCT -> dct_adst
    assert itx[2 * 17 + 12] == 0                                           # no V_ADST at 16x16
    assert itx[3 * 17 + 9] == _addr("mi_inv_txfm_add_identity_identity_32x32")
    assert itx[4 * 17 + 9] == 0                                            # 64x64: DCT_DCT only
    # lf, cdef, lr
    assert slots[408:412] == [_addr(n) for n in ("mi_lpf_h_sb_y", "mi_lpf_v_sb_y", "mi_lpf_h_sb_uv", "mi_lpf_v_sb_uv")]
    assert slots[412:416] == [_addr(n) for n in ("mi_cdef_dir", "mi_cdef_filter_8x8", "mi_cdef_filter_4x8",
                                                 "mi_cdef_filter_4x4")]
    assert slots[416:421] == [_addr(n) for n in ("mi_wiener_filter7", "mi_wiener_filter5", "mi_sgr_filter_5x5",
                                                 "mi_sgr_filter_3x3", "mi_sgr_filter_mix")]


def test_fill_dsp_tables_rejects_bad_bpc():
    buf = (ctypes.c_uint8 * (422 * PTR))()
    assert lib().mi_fill_dsp_tables(buf, 9) == -22
    assert lib().mi_fill_dsp_tables(None, 8) == -22


@pytest.mark.gpu
def test_table_slots_through_function_pointers():
    """tests/c/dsp_table_check: a C caller fills the table and calls every itxfm_add slot
    (3 eob regimes, positive and negative strides), loop_filter_sb[2][2] and cdef dir/fb[3]
    through the pointers, for 8/10/12 bpc, against the oracle."""
    exe = os.path.join(ROOT, "tests", "c", "dsp_table_check")
    assert os.path.exists(exe), "built by __graft_entry__.build() (make -C tests/c)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
