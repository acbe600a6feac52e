"""itx of the 4K10 bench frame split by block class (diagnostic): the whole list, the non-DC
blocks alone and the DC-only blocks alone, each graph-timed with a fresh coefficient arena per
call (a 20-arena ring, as bench.py's step). Outputs are not checked (the split lists leave
pixels of the other class untouched)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench  # noqa: E402
from gtime import gtime  # noqa: E402
from rav1d_amd import frame as F  # noqa: E402
from rav1d_amd.synth import itx_band_order, itx_dc_runs, make_frame  # noqa: E402

fr = make_frame(3840, 2160, 10, 1, seed=0x4C100001, with_fg=False, with_mc=True)
ctx = F.Context(0)
pipe = bench.Pipeline(ctx, fr, ring=2)
L = F.lib()
pa = pipe.A.picture()
ah = (2160 + 127) & ~127
blocks = fr["blocks"]
dc = (blocks["txtp"] == 0) & (blocks["eob"] < 1)
ring = [pipe.coef0.clone() for _ in range(20)]


def prep(sel, runs=False):
    blk, _, bs = itx_band_order(blocks[sel], [ah, ah >> 1, ah >> 1])
    de = itx_dc_runs(blk, bs) if runs else None
    return (torch.from_numpy(blk.view(np.uint8).copy()).cuda(), (ctypes.c_uint32 * bs.size)(*[int(v) for v in bs.reshape(-1)]),
            None if de is None else (ctypes.c_uint32 * de.size)(*[int(v) for v in de.reshape(-1)]))


everything = np.ones(len(blocks), bool)
cases = {"all": prep(everything), "runs": prep(everything, True), "nondc": prep(~dc), "dc": prep(dc),
         "dc_runs": prep(dc, True)}
for rep in range(2):
    for name, (bt, bands, de) in cases.items():
        k = [0]

        def one(stream, bt=bt, bands=bands, de=de):
            c = ring[k[0] % len(ring)]
            k[0] += 1
            if de is None:
                F.check(L.mi_itx_frame_banded(ctx.h, ctypes.byref(pa), ctypes.c_void_p(bt.data_ptr()), bands,
                                              ctypes.c_void_p(c.data_ptr()), bench.ITX_KEEP_COEFS, F._stream_ptr(stream)), "itx")
            else:
                F.check(L.mi_itx_frame_runs(ctx.h, ctypes.byref(pa), ctypes.c_void_p(bt.data_ptr()), bands, de,
                                            ctypes.c_void_p(c.data_ptr()), bench.ITX_KEEP_COEFS, F._stream_ptr(stream)), "itx")
        print(f"itx {name} {gtime(one):.2f} us", flush=True)
