"""Per-size itx time on the bench's 4K10 frame through mi_itx_frame_banded (the bench's call),
coefficients kept (MI_ITX_KEEP_COEFS), with only one size's range non-empty (diagnostic)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame, TX_DIMS, itx_band_order, itx_algorithmic_bytes
fr = make_frame(3840, 2160, 10, 1, seed=0x4C100001, with_fg=False, with_mc=True)
ctx = F.Context(0)
A = F.Frame(3840, 2160, 10, 1)
for p, a in enumerate(fr["planes"]):
    A.set_plane_np(p, a)
ah = 2176
blk, _, bs = itx_band_order(fr["blocks"], [ah, ah >> 1, ah >> 1])
blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
coef = torch.from_numpy(fr["coef"].copy()).cuda()
bs = np.asarray(bs, np.int64).reshape(19, 9)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gtime import gtime
def t(bsx):
    return gtime(lambda s: F.itx_frame(ctx, A, blocks, None, coef, 1, band_start=bsx, stream=s))
tot = t(bs)
ab = itx_algorithmic_bytes(blk, 10, zero_coefs=False)
print(f"all {tot:.1f} us, {len(blk)} blocks, {ab/1e6:.1f} MB, {ab/tot/1e3:.0f} GB/s")
for s in range(19):
    lo, hi = int(bs[s, 0]), int(bs[s, 8])
    if hi == lo:
        continue
    one = bs.copy()
    for k in range(19):
        one[k, :] = lo if k <= s else hi
    one[s] = bs[s]
    sub = blk[lo:hi]
    dc = int(((sub["txtp"] == 0) & (sub["eob"] < 1)).sum())
    us = t(one)
    b = itx_algorithmic_bytes(sub, 10, zero_coefs=False)
    print(f"tx {s:2d} {TX_DIMS[s][0]:2d}x{TX_DIMS[s][1]:<2d} n={hi-lo:6d} dconly={dc:6d} {us:7.1f} us {b/1e6:6.2f} MB {b/us/1e3:6.0f} GB/s")
