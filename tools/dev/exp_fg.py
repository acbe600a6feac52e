"""Film-grain apply timing experiments on a synthetic 4K10 frame (diagnostic, not a test)."""
import sys, os, ctypes, copy
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame

fr = make_frame(3840, 2160, 10, 1, seed=0x4C100001)
ctx = F.Context(0)
O = F.Frame(3840, 2160, 10, 1)
G = F.Frame(3840, 2160, 10, 1)
for p, a in enumerate(fr["planes"]):
    O.set_plane_np(p, a)
lib = F.lib()


def run(fg, name, reps=50):
    d = F.film_grain_data(fg)
    po, pg = O.picture(), G.picture()
    F.check(lib.mi_film_grain_prep(ctx.h, ctypes.byref(po), ctypes.byref(d), None), "prep")
    for _ in range(3):
        F.check(lib.mi_film_grain_apply(ctx.h, ctypes.byref(po), ctypes.byref(pg), ctypes.byref(d), 0, None), "apply")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lib.mi_film_grain_apply(ctx.h, ctypes.byref(po), ctypes.byref(pg), ctypes.byref(d), 0, None)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{name:34s} {us:8.1f} us")


base = fr["fg"]
print("params:", {k: base[k] for k in ("num_y_points", "chroma_scaling_from_luma", "num_uv_points", "overlap_flag")})
run(base, "bench params")
v = copy.deepcopy(base); v["overlap_flag"] = 0; run(v, "no overlap")
v = copy.deepcopy(base); v["overlap_flag"] = 1; run(v, "overlap")
v = copy.deepcopy(base); v["num_y_points"] = 0; v["y_points"] = []; v["chroma_scaling_from_luma"] = 0
v["num_uv_points"] = [0, 0]; v["uv_points"] = [[], []]; run(v, "no grain (copy path)")
v = copy.deepcopy(base); v["chroma_scaling_from_luma"] = 0; v["num_uv_points"] = [0, 0]; v["uv_points"] = [[], []]
run(v, "luma grain only")
# HBM reference: torch copy of the same bytes
src = [O.planes[p] for p in range(3)]
dst = [G.planes[p] for p in range(3)]
for _ in range(3):
    for s, t in zip(src, dst): t.copy_(s)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    for s, t in zip(src, dst): t.copy_(s)
e1.record(); torch.cuda.synchronize()
print(f"{'torch copy of the 3 planes':34s} {e0.elapsed_time(e1) / 50 * 1e3:8.1f} us")
