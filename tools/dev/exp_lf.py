"""Deblock timing on the bench's synthetic 4K10 frame (diagnostic, not a test).
usage: python tools/exp_lf.py [tiles|inplace|both] [noedges]"""
import sys, os
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame, frame_bytes

w, h, bpc = 3840, 2160, 10
fr = make_frame(w, h, bpc, 1, seed=0x4C100001, with_fg=False, with_mc=False)
if "noedges" in sys.argv:
    fr["lf"]["masks"]["filter_y"] = 0
    fr["lf"]["masks"]["filter_uv"] = 0
ctx = F.Context(0)
A, D = F.Frame(w, h, bpc, 1), F.Frame(w, h, bpc, 1)
for p, a in enumerate(fr["planes"]):
    A.set_plane_np(p, a)
meta = F.LoopFilterMeta(fr["lf"])
algo = 2 * frame_bytes(w, h, bpc, 1) + ((w + 3) >> 2) * ((h + 3) >> 2) * 4 + fr["lf"]["masks"].nbytes
mode = sys.argv[1] if len(sys.argv) > 1 else "both"


def run(name, fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{name:10s} {us:8.1f} us  {algo / us / 1e3:7.1f} GB/s (algorithmic)")


if mode in ("tiles", "both"):
    run("tiles", lambda: F.deblock_frame(ctx, A, meta, dst=D))
if mode in ("inplace", "both"):
    run("inplace", lambda: F.deblock_frame(ctx, A, meta))
