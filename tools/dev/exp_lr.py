"""Loop-restoration timing on a synthetic 4K10 frame by unit-type mix (diagnostic, not a test)."""
import sys, os
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rav1d_amd import frame as F
from rav1d_amd.synth import make_lr_meta, make_texture, frame_bytes

w, h, bpc = 3840, 2160, 10
ctx = F.Context(0)
rng = np.random.default_rng(1)
C, D, O = (F.Frame(w, h, bpc, 1) for _ in range(3))
for fr in (C, D):
    for p in range(3):
        pw, ph = fr.dims(p)
        fr.set_plane_np(p, make_texture(rng, pw, ph, bpc))
algo = 2 * frame_bytes(w, h, bpc, 1) + frame_bytes(w, h, bpc, 1) * 4 // 64


def run(name, p_none, p_wiener, reps=20):
    meta = F.LrMeta(make_lr_meta(w, h, 1, np.random.default_rng(7), p_none=p_none, p_wiener=p_wiener,
                                 unit_log2=(7, 6)))
    for _ in range(3):
        F.lr_frame(ctx, C, D, O, meta)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        F.lr_frame(ctx, C, D, O, meta)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{name:10s} {us:8.1f} us  {algo / us / 1e3:7.1f} GB/s", flush=True)


CASES = {"mix": (0.2, 0.4), "none": (1.0, 0.0), "wiener": (0.0, 1.0), "sgr": (0.0, 0.0)}
for name in (sys.argv[1:] or CASES):
    run(name, *CASES[name])
