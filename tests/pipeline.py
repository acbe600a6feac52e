"""The whole implemented DSP pipeline, once through the oracle (CPU) and once through the
C-ABI on the device: [MC ->] recon(itx) -> deblock -> CDEF -> LR [-> film grain].
Shared by the end-to-end parity test, smoke() and bench.py's cpu_baseline leg."""
import numpy as np

from tests import oracle_lib
from tests.test_oracle_lf import pad_planes


def oracle_pipeline(fr, sb128=1):
    w, h, bpc, layout = fr["w"], fr["h"], fr["bpc"], fr["layout"]
    A = pad_planes(fr["planes"], w, h, bpc, layout)
    if fr.get("mc") is not None:
        refs = [pad_planes(r, w, h, bpc, layout) for r in fr["refs"]]
        units, _, masks = fr["mc"]
        A, _ = oracle_lib.mc_frame(A, refs, bpc, layout, w, h, units, masks)
    A = oracle_lib.itx_frame(A, fr["blocks"], fr["coef"].copy(), bpc)
    A = oracle_lib.deblock_frame(A, bpc, layout, w, h, fr["lf"], sb128=sb128)
    B = oracle_lib.cdef_frame(A, bpc, layout, w, h, fr["lf"]["masks"], fr["cdef"])
    O = oracle_lib.lr_frame(B, A, bpc, layout, w, h, dict(fr["lr"], sb128=sb128))
    G = oracle_lib.film_grain(O, bpc, layout, w, h, fr["fg"]) if fr["fg"] else O
    return dict(recon_deblocked=A, cdef=B, lr=O, out=G)
