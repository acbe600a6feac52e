"""The one-grid MC hand-off's ordering, checked on the shipped gfx950 code object (CPU only).

mi_mc_frame_sync's chroma waves read a SEG mask that luma waves of the same launch write,
ordered by a flag poll without an acquire (rav1d_amd/csrc/mc.hip). That argument
holds only while the compiler emits what it assumes: `global_` (never `flat_`) `sc1` accesses,
mask loads after the poll loop, and a `vmcnt(0)` drain between the mask stores and the flag
store. tests/isa_check.py checks the three on the disassembly; the synthetic cases below show
that each check fails when its property is broken."""
import os
import shutil

import pytest

from tests import isa_check as ic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rav1d_amd", "librav1d_amd.so")

needs_tools = pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which(f"{ic.LLVM}/llvm-objdump")),
                                 reason="library or ROCm llvm tools missing")


@pytest.fixture(scope="module")
def mc_kernels():
    out = {}
    for co in ic.code_objects(LIB):
        for name, ins in ic.functions(ic.disassemble(co)).items():
            if "mc_kernel" in name:
                out[name] = ins
    return out


@needs_tools
def test_shipped_mc_kernel_handoff(mc_kernels):
    assert len(mc_kernels) == 2, sorted(mc_kernels)          # u8 and u16 pixels
    for name, ins in mc_kernels.items():
        errs, summary = ic.check_handoff(ins)
        assert not errs, (name, errs[:5])
        assert summary["poll_loads"] >= 1 and summary["mask_loads"] >= 1 and summary["flag_stores"] >= 1, summary


# ---- the checker itself: a minimal kernel in llvm-objdump's shape, then one defect each ----

def _prog(lines):
    """[(addr, text, target)] from (text, target-label) pairs; labels are instruction indices."""
    return [(4 * k, t, None if tgt is None else 4 * tgt) for k, (t, tgt) in enumerate(lines)]


def _good():
    return [
        ("global_store_dword v[0:1], v2, off sc1", None),       # 0 mask word (producer)
        ("s_waitcnt vmcnt(0)", None),                          # 1 drain
        ("s_barrier", None),                                   # 2
        ("global_store_dword v[4:5], v6, off sc1", None),       # 3 flag
        ("s_cbranch_scc1 9", 9),                               # 4 not a consumer: done
        ("global_load_dword v7, v[8:9], off sc1", None),        # 5 poll
        ("s_waitcnt vmcnt(0)", None),                          # 6
        ("s_sleep 1", None),                                   # 7
        ("s_cbranch_vccnz 5", 5),                              # 8 poll again
        ("global_load_dword v10, v[12:13], off sc1", None),     # 9 mask load
        ("s_endpgm", None),                                    # 10
    ]


def test_checker_accepts_the_pattern():
    errs, summary = ic.check_handoff(_prog(_good()))
    assert not errs, errs
    assert summary["poll_loads"] == 1 and summary["mask_loads"] == 1 and summary["flag_stores"] == 1


def test_checker_rejects_missing_drain():
    p = _good()
    p[1] = ("s_waitcnt lgkmcnt(0)", None)
    errs, _ = ic.check_handoff(_prog(p))
    assert any("drain" in e for e in errs), errs


def test_checker_rejects_mask_load_before_poll():
    p = _good()
    p[4] = ("global_load_dword v10, v[12:13], off sc1", None)     # hoisted above the loop
    p[9] = ("s_nop 0", None)
    errs, _ = ic.check_handoff(_prog(p))
    assert any("before a poll loop" in e for e in errs), errs


def test_checker_rejects_flat_access():
    p = _good()
    p[9] = ("flat_load_dword v10, v[12:13] sc1", None)
    errs, _ = ic.check_handoff(_prog(p))
    assert any("flat" in e for e in errs), errs
