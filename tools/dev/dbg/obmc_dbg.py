import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from rav1d_amd import frame as F
from rav1d_amd.frame import McMeta, mc_frame
from tests.test_mc_ext_gpu import textured, randomised, planes, obmc_units
from tests import oracle_lib
bpc, layout, bs = 8, 1, 16
w, h = 192, 128
rng = np.random.default_rng(bpc * 5 + layout + bs)
ctx = F.Context(0)
refs = [textured(w, h, bpc, layout, rng) for _ in range(2)]
cur = randomised(w, h, bpc, layout, rng)
init = planes(cur)
(ua, ca), (ul, cl) = obmc_units(w, h, layout, rng, 2, bs)
z = np.zeros(1, np.uint8)
rp = [planes(r) for r in refs]
for name, units, cs in (("above", ua, ca), ("left", ul, cl)):
    c2 = randomised(w, h, bpc, layout, np.random.default_rng(1))
    i2 = planes(c2)
    mc_frame(ctx, c2, refs, McMeta(units, cs, z))
    torch.cuda.synchronize()
    exp, _ = oracle_lib.mc_frame(i2, rp, bpc, layout, w, h, units, z)
    for p in range(3):
        g = c2.buffer_np(p)
        bad = np.argwhere(g != exp[p])
        print(name, "plane", p, "bad", len(bad))
        if len(bad):
            ys, xs = bad[:, 0], bad[:, 1]
            print("  rows%16:", np.bincount(ys % 16, minlength=16), " cols%16:", np.bincount(xs % 16, minlength=16))
            print("  first", bad[:5].tolist(), "got", g[tuple(bad[0])], "exp", exp[p][tuple(bad[0])], "init", i2[p][tuple(bad[0])])
            # which unit covers the first bad pixel
            y0, x0 = bad[0]
            for u in units:
                if u["plane"] == p and u["x"] <= x0 < u["x"] + u["w"] and u["y"] <= y0 < u["y"] + u["h"]:
                    print("  unit", u)
