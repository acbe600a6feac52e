"""MC timing on subsets of a synthetic 4K10 inter frame (diagnostic, not a test)."""
import sys, os, ctypes
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rav1d_amd import frame as F
from rav1d_amd.synth import make_mc_units, make_texture, mc_sort_units, mc_class_of, mc_algorithmic_bytes

w, h, bpc = 3840, 2160, 10
rng = np.random.default_rng(0x4C100001)
ctx = F.Context(0)
refs = []
for _ in range(2):
    r = F.Frame(w, h, bpc, 1)
    for p in range(3):
        pw, ph = r.dims(p)
        r.set_plane_np(p, make_texture(rng, pw, ph, bpc))
    refs.append(r)
units, cs, masks = make_mc_units(w, h, 1, rng)
cur = F.Frame(w, h, bpc, 1)


def run(mask, name, reps=20):
    u, c = mc_sort_units(units[mask])
    meta = F.McMeta(u, c, masks)
    for _ in range(3):
        F.mc_frame(ctx, cur, refs, meta)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        F.mc_frame(ctx, cur, refs, meta)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    px = int((u["w"].astype(np.int64) * u["h"]).sum())
    print(f"{name:30s} n={len(u):6d} px={px/1e6:6.2f}M {us:8.1f} us  {mc_algorithmic_bytes(u, bpc)/us/1e3:7.1f} GB/s")


luma = units["plane"] == 0
comp = units["ref"][:, 1] >= 0
cls = mc_class_of(units)
if len(sys.argv) > 1:       # one class only (for counter runs): e.g. 8x8
    cw, ch = [int(v) for v in sys.argv[1].split("x")]
    run(cls == (int(np.log2(cw)) * 8 + int(np.log2(ch))), f"class {sys.argv[1]}")
    sys.exit(0)
run(np.ones(len(units), bool), "all")
run(luma, "luma")
run(~luma, "chroma")
run(~comp, "single")
run(comp, "compound")
for c in np.unique(cls):
    m = cls == c
    run(m, f"class {1 << (c >> 3)}x{1 << (c & 7)}")
