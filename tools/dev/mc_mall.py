"""MC on the bench's 4K10 inter frame with the reference pictures resident in the Infinity
Cache (launches back to back) and evicted from it (a 1 GiB write between launches), uniform and
coherent motion. Dev experiment: python tools/dev/mc_mall.py [reps]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd import frame as F  # noqa: E402
from rav1d_amd.synth import make_frame, mc_algorithmic_bytes  # noqa: E402

W, H, BPC = 3840, 2160, 10
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = F.Context(0)
lib = F.lib()
flush = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
for mv in ("uniform", "coherent"):
    fr = make_frame(W, H, BPC, 1, seed=0x4C100001, with_fg=False, with_mc=True, mv_mode=mv)
    cur = F.Frame(W, H, BPC, 1)
    refs = []
    for planes in fr["refs"]:
        r = F.Frame(W, H, BPC, 1)
        for p, a in enumerate(planes):
            r.set_plane_np(p, a)
        refs.append(r)
    meta = F.McMeta(*fr["mc"])
    pics = (F.MiPicture * len(refs))(*[r.picture() for r in refs])
    pc = cur.picture()
    algo = mc_algorithmic_bytes(fr["mc"][0], BPC) + fr["mc"][2].nbytes

    def mc():
        F.check(lib.mi_mc_frame(ctx.h, ctypes.byref(pc), pics, len(refs), ctypes.c_void_p(meta.blocks.data_ptr()),
                                meta.class_start, ctypes.c_void_p(meta.masks.data_ptr()), None, None), "mc")
    for _ in range(3):
        mc()
    torch.cuda.synchronize()
    for state in ("warm", "cold"):
        tot = 0.0
        for _ in range(reps):
            if state == "cold":
                flush.fill_(1)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            mc()
            b.record()
            torch.cuda.synchronize()
            tot += a.elapsed_time(b)
        ms = tot / reps
        print(f"{mv:9s} {state}: {ms * 1e3:7.1f} us  {algo / (ms / 1e3) / 1e9:7.1f} GB/s algorithmic", flush=True)
