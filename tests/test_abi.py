"""The C-ABI library loads here (no GPU needed) and exports every symbol the header declares."""
import ctypes
import os
import re

from rav1d_amd import EXPORTED, LIB_PATH, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "mi_av1dsp.h")).read()
    return sorted(set(re.findall(r"\b(mi_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    L = lib()
    syms = header_symbols()
    assert syms, "no symbols parsed"
    for s in syms:
        assert hasattr(L, s), f"{s} missing from {LIB_PATH}"
    assert sorted(EXPORTED) == sorted(syms)


def test_version_string():
    assert b"gfx950" in lib().mi_version()
