"""itx time of the bench frame's blocks minus the 64-point sizes (banded call, coefficients
kept), for A/B of library variants via MI_LIB (diagnostic)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame, itx_band_order, itx_algorithmic_bytes
fr = make_frame(3840, 2160, 10, 1, seed=0x4C100001, with_fg=False, with_mc=True)
b = fr["blocks"]
if os.environ.get("NO64", "1") == "1":
    b = b[~np.isin(b["tx"], [4, 11, 12, 17, 18])]
ctx = F.Context(0)
A = F.Frame(3840, 2160, 10, 1)
for p, a in enumerate(fr["planes"]):
    A.set_plane_np(p, a)
blk, _, bs = itx_band_order(b, [2176, 1088, 1088])
blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
coef = torch.from_numpy(fr["coef"].copy()).cuda()
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gtime import gtime
us = gtime(lambda s: F.itx_frame(ctx, A, blocks, None, coef, 1, band_start=bs, stream=s))
ab = itx_algorithmic_bytes(blk, 10, zero_coefs=False)
print(f"{os.path.basename(os.environ.get('MI_LIB', 'base'))}: {len(blk)} blocks {us:.1f} us {ab/us/1e3:.0f} GB/s")
