"""Run the bench frame's itx through mi_itx_frame (one-launch kernel when MI_ITX_ALL is set)
REPS times, for PMC passes (diagnostic)."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rav1d_amd import frame as F  # noqa: E402
from rav1d_amd.synth import make_frame, itx_region_sort  # noqa: E402
fr = make_frame(3840, 2160, 10)
ctx = F.Context(0)
A = F.Frame(3840, 2160, 10, 1)
for p, a in enumerate(fr["planes"]):
    A.set_plane_np(p, a)
coef = torch.from_numpy(fr["coef"].copy()).cuda()
b = fr["blocks"]
if os.environ.get("SUBSET") == "4x4dc":
    b = b[(b["tx"] == 0) & (b["txtp"] == 0) & (b["eob"] < 1)]
bd = torch.from_numpy(b.view(np.uint8).copy()).cuda()
ss = np.searchsorted(b["tx"], np.arange(20)).astype(np.uint32)
for _ in range(int(os.environ.get("REPS", "10"))):
    F.itx_frame(ctx, A, bd, ss, coef, 0)
torch.cuda.synchronize()
if os.environ.get("REGIONS"):
    sb, rs = itx_region_sort(b, 3840, 2160, 1)
    bdr = torch.from_numpy(sb.view(np.uint8).copy()).cuda()
    rsd = torch.from_numpy(rs.astype(np.int32)).cuda()
    for _ in range(int(os.environ.get("REPS", "10"))):
        F.itx_frame_regions(ctx, A, bdr, rsd, coef, 0)
    torch.cuda.synchronize()
print("done")
