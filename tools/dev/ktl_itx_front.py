"""The front of an itx workgroup from a timeline build's stamps (gpurun_out/ktl_itx.npy, written
by tools/dev/ktl.py): slot 0 start, 4 size known, 3 block range known, 1 first descriptor in."""
import numpy as np

a = np.load("gpurun_out/ktl_itx.npy")
ok = (a[:, 4] != 0) & (a[:, 4] >= a[:, 0]) & (a[:, 3] >= a[:, 4]) & (a[:, 1] >= a[:, 3])
print("valid", round(float(ok.mean()), 3))
for name, x, y in (("start -> size known", 0, 4), ("size known -> block range known (into the size path)", 4, 3),
                   ("block range -> first descriptor", 3, 1)):
    d = (a[ok, y] - a[ok, x]) / 100.0
    print(f"{name}: mean {d.mean():.2f} p50 {np.median(d):.2f} p90 {np.percentile(d, 90):.2f} us")
