"""Front-end wall time per stream (stream_events, every event consumed): min / median of
interleaved repetitions at 1 and 8 threads. python tools/dev/fe_time.py NAME[,NAME..] [REPS]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.getcwd())
from rav1d_amd.av1dec import stream_events  # noqa: E402

G = "tests/golden/streams"
V = {v["name"]: v for v in json.load(open(G + "/vectors.json"))}
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
for name in sys.argv[1].split(","):
    data = open(os.path.join(G, V[name]["file"]), "rb").read()
    ts = {1: [], 8: []}
    for r in range(reps):
        for th in ts:
            t = time.perf_counter()
            sum(1 for e in stream_events(data, th))
            ts[th].append((time.perf_counter() - t) * 1e3)
    print(name, " ".join(f"t{th}: min {min(v):.1f} med {statistics.median(v):.1f}" for th, v in ts.items()), flush=True)
