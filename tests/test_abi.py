"""The C-ABI library loads here (no GPU needed) and exports every symbol the header declares."""
import ctypes
import os
import re

from rav1d_amd import EXPORTED, LIB_PATH, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _decl(name):
    txt = open(os.path.join(ROOT, "include", name)).read()
    return set(re.findall(r"\b(mi_[a-z0-9_]+)\s*\(", txt))


def header_symbols():
    """librav1d_amd.so: every mi_av1dsp.h entry plus mi_av1dec.h's device executor and
    mi_av1out.h's device-to-host output."""
    dec, out = _decl("mi_av1dec.h"), _decl("mi_av1out.h")
    return sorted(_decl("mi_av1dsp.h") | {s for s in dec if s.startswith(("mi_frame_", "mi_ctx_"))} |
                  {s for s in out if not s.startswith("mi_muxer_")})


def test_front_end_exports_header_symbols():
    """libmi_av1dec.so (host front-end, no GPU code) exports mi_av1dec.h's mi_dec_* entries."""
    from rav1d_amd.av1dec import dec_lib
    L = dec_lib()
    syms = sorted(s for s in _decl("mi_av1dec.h") if s.startswith("mi_dec_"))
    assert len(syms) >= 5
    syms += sorted(s for s in _decl("mi_av1out.h") if s.startswith("mi_muxer_"))
    for s in syms:
        assert hasattr(L, s), f"{s} missing from libmi_av1dec.so"


def test_library_exports_header_symbols():
    L = lib()
    syms = header_symbols()
    assert syms, "no symbols parsed"
    for s in syms:
        assert hasattr(L, s), f"{s} missing from {LIB_PATH}"
    assert sorted(EXPORTED) == sorted(syms)


def test_version_string():
    assert b"gfx950" in lib().mi_version()


def test_per_call_entries_reject_bad_arguments_without_a_device():
    """Argument checks come before any device work, as the reference's table slots assume
    valid input: out-of-range sizes, kinds, layouts and bit depths return -EINVAL (22)."""
    L = lib()
    buf = (ctypes.c_uint8 * 65536)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    EINVAL = -22
    assert L.mi_dsp_lr_wiener(p, 64, p, p, 0, 8, p, 0, 1023) == EINVAL           # w = 0
    assert L.mi_dsp_lr_wiener(p, 64, p, p, 385, 8, p, 0, 1023) == EINVAL         # w > 384
    assert L.mi_dsp_lr_wiener(p, 64, p, p, 64, 65, p, 0, 1023) == EINVAL         # h > 64
    assert L.mi_dsp_lr_sgr(3, p, 64, p, p, 64, 8, p, 0, 1023) == EINVAL          # kind 3
    assert L.mi_dsp_lr_sgr(0, p, 64, p, p, 64, 8, p, 0, 511) == EINVAL           # 9-bit
    assert L.mi_dsp_fg_generate_grain_uv(0, p, p, p, 0, 1023) == EINVAL          # I400 slot
    assert L.mi_dsp_fg_generate_grain_uv(1, p, p, p, 2, 1023) == EINVAL          # uv 2
    assert L.mi_dsp_fgy_32x32xn(p, p, 64, p, 0, p, p, 8, 0, 1023) == EINVAL      # pw 0
    assert L.mi_dsp_fgy_32x32xn(p, p, 64, p, 64, p, p, 33, 0, 1023) == EINVAL    # bh > 32
    assert L.mi_dsp_fguv_32x32xn(1, p, p, 64, p, 32, p, p, 17, 0, p, 64, 0, 0, 1023) == EINVAL  # 4:2:0 bh > 16
    assert L.mi_dsp_fguv_32x32xn(1, p, p, 64, p, 32, p, p, 8, 0, None, 64, 0, 0, 1023) == EINVAL  # no luma
    assert L.mi_dsp_mc_scaled(0, 10, p, 64, p, 64, 8, 8, 0, 0, 1024, 1024, 1023) == EINVAL  # filter 10
