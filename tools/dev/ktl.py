"""Kernel timelines of one bench step (diagnostic; needs MI_LIB=librav1d_amd_ktl.so, built with
MI_BUILD_VARIANT=ktl MI_EXTRA_FLAGS=-DMI_KTL): per workgroup s_memrealtime stamps (100 MHz) at
phase boundaries. Prints per kernel the span, the workgroup lifetimes and phase durations, and
how the starts spread over the span (generations). Saves the raw stamps to gpurun_out/ktl_*.npy."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from rav1d_amd import frame as F  # noqa: E402
from rav1d_amd.synth import make_frame  # noqa: E402

UNITS = os.environ.get("KTL_UNITS", "itx,lf,cdef,lr,mc").split(",")
L = F.lib()
bufs = {}
for u in UNITS:
    b = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")   # 131072 workgroups x 8 slots
    bufs[u] = b
fr = make_frame(3840, 2160, 10, 1, seed=0x4C100001, with_fg=False, with_mc=True, packed=True)
ctx = F.Context(0)
pipe = bench.Pipeline(ctx, fr, ring=2)
s = torch.cuda.current_stream()
for _ in range(3):
    pipe.step(s)
torch.cuda.synchronize()
for u in UNITS:
    fn = getattr(L, f"mi_ktl_set_{u}")
    fn.argtypes = [ctypes.c_void_p]
    assert fn(ctypes.c_void_p(bufs[u].data_ptr())) == 0
torch.cuda.synchronize()
pipe.step(s)
torch.cuda.synchronize()
for u in UNITS:
    getattr(L, f"mi_ktl_set_{u}")(ctypes.c_void_p(0))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for u in UNITS:
    a = bufs[u].view(-1, 8).cpu().numpy()
    n = int((a[:, 0] != 0).sum())
    a = a[:n] if n and (a[:n, 0] != 0).all() else a[a[:, 0] != 0]
    np.save(os.path.join(ROOT, "gpurun_out", f"ktl_{u}.npy"), a)
    if not len(a):
        print(u, "no stamps")
        continue
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) / 100.0                   # us
    slots = [k for k in range(1, 7) if (a[:, k] != 0).all() and (a[:, k] >= a[:, 0]).all() and k != 6 or k == 5]
    end = a[:, 5] if (a[:, 5] != 0).all() else a[:, 1:6].max(1)
    en = (end - t0) / 100.0
    life = en - st
    print(f"== {u}: {len(a)} workgroups, span {en.max():.1f} us, lifetime mean {life.mean():.1f} "
          f"p10 {np.percentile(life, 10):.1f} p50 {np.percentile(life, 50):.1f} p90 {np.percentile(life, 90):.1f} max {life.max():.1f}")
    q = np.percentile(st, [10, 25, 50, 75, 90, 100])
    print("   start percentiles (us) 10/25/50/75/90/100:", " ".join(f"{v:.1f}" for v in q))
    prev = a[:, 0]
    for k in range(1, 6):
        c = a[:, k]
        ok = (c != 0) & (c >= prev)
        if ok.mean() > 0.5:
            d = (c[ok] - prev[ok]) / 100.0
            print(f"   phase {k - 1}->{k}: mean {d.mean():.2f} p50 {np.median(d):.2f} p90 {np.percentile(d, 90):.2f} us")
            prev = np.where(ok, c, prev)
    # concurrency over time: active workgroups at 20 sample points
    ts = np.linspace(0, en.max(), 21)[:-1]
    act = [int(((st <= t) & (en > t)).sum()) for t in ts]
    print("   active workgroups over the span:", act)
    if u == "itx":
        cls = a[:, 6]
        for c in np.unique(cls):
            m = cls == c
            print(f"   size {int(c):2d}: {m.sum():5d} wg, life mean {life[m].mean():6.1f} max {life[m].max():6.1f}, start {st[m].min():5.1f}-{st[m].max():5.1f}")
    if u == "lr":
        cls = a[:, 6]
        for c in np.unique(cls):
            m = cls == c
            line = f"   type {int(c)}: {m.sum():5d} wg, life mean {life[m].mean():5.1f}"
            prev = a[m, 0]
            for k in range(1, 6):
                col = a[m, k]
                ok = (col != 0) & (col >= prev)
                if ok.mean() > 0.5:
                    line += f" | {k - 1}->{k} {((col[ok] - prev[ok]) / 100.0).mean():.2f}"
                    prev = np.where(ok, col, prev)
            print(line)
