"""Per-size itx time on the bench's 4K10 frame: mi_itx_frame with only one size's range
non-empty (diagnostic, not a test)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame, TX_DIMS
fr = make_frame(3840, 2160, 10, 1, seed=0x4C100001, with_fg=False, with_mc=True)
ctx = F.Context(0)
A = F.Frame(3840, 2160, 10, 1)
blocks = torch.from_numpy(fr["blocks"].view(np.uint8).copy()).cuda()
coef = torch.from_numpy(fr["coef"].copy()).cuda()
ss = np.asarray(fr["size_start"], np.int64)
b = fr["blocks"]
def t(ssx, reps=50):
    for _ in range(3):
        F.itx_frame(ctx, A, blocks, ssx, coef, 0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        F.itx_frame(ctx, A, blocks, ssx, coef, 0)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
print("all", round(t(ss), 1), "us", len(b), "blocks")
for s in range(19):
    n = int(ss[s + 1] - ss[s])
    if not n:
        continue
    one = ss.copy()
    one[:s + 1] = ss[s]
    one[s + 1:] = ss[s + 1]
    sub = b[ss[s]:ss[s + 1]]
    dc = int(((sub["txtp"] == 0) & (sub["eob"] < 1)).sum())
    print(f"tx {s:2d} {TX_DIMS[s][0]:2d}x{TX_DIMS[s][1]:<2d} n={n:6d} dconly={dc:6d} {t(one):7.1f} us")
