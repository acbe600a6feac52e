"""itx timing experiments on subsets of a synthetic 4K10 frame (diagnostic, not a test)."""
import sys, os, ctypes
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rav1d_amd import frame as F, ITX_KEEP_COEFS, N_RECT_TX_SIZES
from rav1d_amd.synth import make_frame, itx_algorithmic_bytes

fr = make_frame(3840, 2160, 10)
ctx = F.Context(0)
A = F.Frame(3840, 2160, 10, 1)
for p, a in enumerate(fr["planes"]):
    A.set_plane_np(p, a)
coef = torch.from_numpy(fr["coef"].copy()).cuda()
allb = fr["blocks"]

def run(mask, name, reps=20):
    b = allb[mask]
    ss = np.searchsorted(b["tx"], np.arange(N_RECT_TX_SIZES + 1)).astype(np.uint32)
    bd = torch.from_numpy(b.view(np.uint8).copy()).cuda()
    for _ in range(3):
        F.itx_frame(ctx, A, bd, ss, coef, ITX_KEEP_COEFS)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        F.itx_frame(ctx, A, bd, ss, coef, ITX_KEEP_COEFS)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    ab = itx_algorithmic_bytes(b, 10, zero_coefs=False)
    print(f"{name:28s} n={len(b):7d} {us:8.1f} us  {ab/us/1e3:8.1f} GB/s")

tx, dc = allb["tx"], (allb["txtp"] == 0) & (allb["eob"] < 1)
small = np.isin(tx, [0, 1, 2, 5, 6, 7, 8, 13, 14])
run(np.ones(len(allb), bool), "all")
run(np.isin(tx, [4, 11, 12, 17, 18]), "64-class sizes")
run(np.isin(tx, [3, 9, 10, 15, 16]), "32-class sizes")
if len(sys.argv) > 1:
    sys.exit(0)
run(small, "small sizes")
run(~small, "large sizes")
run((tx == 0) & dc, "4x4 dc-only")
run((tx == 0) & ~dc, "4x4 full")
run(small & ~(tx == 0), "small non-4x4")
run(dc, "all dc-only")
run(~dc, "all non-dc")

# spatial-order experiments: same blocks, sorted by (tx, dc, plane, y, x) instead of type/coef order
order = np.lexsort((allb["x"], allb["y"], allb["plane"], ~dc, allb["tx"]))
allb_sp = allb[order]
def run_sp(maskfn, name):
    global allb
    save = allb
    allb = allb_sp
    tx2 = allb["tx"]; dc2 = (allb["txtp"] == 0) & (allb["eob"] < 1)
    run(maskfn(tx2, dc2), name)
    allb = save
run_sp(lambda t, d: (t == 0) & d, "4x4 dc-only SPATIAL")
run_sp(lambda t, d: (t == 0) & ~d, "4x4 full SPATIAL (mixed types)")
run_sp(lambda t, d: np.ones(len(t), bool), "all SPATIAL")
