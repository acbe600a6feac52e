"""Dependency structure of the intra reconstruction per frame (front-end on the CPU, no GPU):
units, levels, and along the critical path how many hand-offs are between consecutive units
of one plane (a worker running such runs back to back would keep those edges local).
Dev experiment: python tools/dev/ir_chain.py <vector name> [max_frames]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests.stream_lib import decode_stream  # noqa: E402

g = os.path.join(ROOT, "tests/golden/streams")
vecs = {v["name"]: v for v in json.load(open(g + "/vectors.json"))}
name = sys.argv[1]
maxf = int(sys.argv[2]) if len(sys.argv) > 2 else 2


IB = np.dtype([("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"), ("plane", "u1"), ("mode", "u1"),
               ("angle", "i1"), ("flags", "u1"), ("filt", "u1"), ("alpha", "i1"), ("tw", "<u2"), ("th", "<u2"),
               ("mw", "<u2"), ("mh", "<u2"), ("aux", "<u4"), ("pal", "<u4"), ("res", "<u4")])
assert IB.itemsize == 32


def stats(fr, refs):
    n = fr.n_intra
    if n == 0:
        return [np.zeros((1, 1), np.uint8)] * (3 if fr.layout else 1)
    def arr(ptr, cnt, dt):
        return np.frombuffer((ctypes.c_char * (cnt * np.dtype(dt).itemsize)).from_address(ptr), dt).copy()
    ds = arr(fr.dep_start, n + 1, np.int32)
    deps = arr(fr.deps, max(1, int(ds[-1])), np.int32)
    ib = arr(fr.intra, n, IB)
    plane = ib["plane"].astype(int)
    area = ib["w"].astype(int) * ib["h"]
    level = np.zeros(n, np.int64)
    pred = np.full(n, -1)
    for i in range(n):
        d = deps[ds[i]:ds[i + 1]]
        if len(d):
            j = d[np.argmax(level[d])]
            level[i] = level[j] + 1
            pred[i] = j
    # critical path
    i = int(np.argmax(level))
    path = []
    while i >= 0:
        path.append(i)
        i = pred[i]
    path = path[::-1]
    seq = sum(1 for a, b in zip(path, path[1:]) if b == a + 1 and plane[a] == plane[b])
    # levels if runs of consecutive same-plane units with a dep on the predecessor were one
    # worker's job (edges inside a run: no hand-off, cost 0.3 of one)
    w = np.zeros(n)
    for i in range(n):
        best = 0.0
        for j in deps[ds[i]:ds[i + 1]]:
            c = w[j] + (0.3 if (j == i - 1 and plane[j] == plane[i]) else 1.0)
            best = max(best, c)
        w[i] = best
    print(f"frame {fr.w}x{fr.h} units {n} levels {level.max() + 1} path: {len(path)} units, "
          f"{seq} consecutive-unit edges, areas {np.bincount(np.log2(area[path]).astype(int), minlength=13)[4:13]}"
          f" | run-merged weighted depth {w.max():.0f}", flush=True)
    return [np.zeros((1, 1), np.uint8)] * (3 if fr.layout else 1)


v = vecs[name]
data = open(os.path.join(g, v["file"]), "rb").read()
decode_stream(data, recon=stats, max_frames=maxf, hash_output=False)
