"""The bench frame's itx (banded call, coefficients kept) REPS times, for PMC passes (diagnostic)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame, itx_band_order
fr = make_frame(3840, 2160, 10, 1, seed=0x4C100001, with_fg=False, with_mc=True)
ctx = F.Context(0)
A = F.Frame(3840, 2160, 10, 1)
for p, a in enumerate(fr["planes"]):
    A.set_plane_np(p, a)
blk, _, bs = itx_band_order(fr["blocks"], [2176, 1088, 1088])
blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
coef = torch.from_numpy(fr["coef"].copy()).cuda()
for _ in range(int(os.environ.get("REPS", "10"))):
    F.itx_frame(ctx, A, blocks, None, coef, 1, band_start=bs)
torch.cuda.synchronize()
print("done")
