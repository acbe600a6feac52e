"""A/B of two front-end libraries (MI_DEC_LIB) on stream decode time, interleaved runs in fresh
processes: python tools/dev/fe_ab.py LIB_A LIB_B NAME[,NAME..] [REPS] [THREADS]
(LOOKAHEAD=0 in the environment: one temporal unit at a time, as bench.py's unpipelined pass)"""
import json
import os
import statistics
import subprocess
import sys

liba, libb, names = sys.argv[1], sys.argv[2], sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
th = int(sys.argv[5]) if len(sys.argv) > 5 else 8
code = r'''
import sys, os, json, time
sys.path.insert(0, os.getcwd())
from rav1d_amd.av1dec import stream_events
G = "tests/golden/streams"; V = {v["name"]: v for v in json.load(open(G + "/vectors.json"))}
out = {}
for name in sys.argv[1].split(","):
    data = open(os.path.join(G, V[name]["file"]), "rb").read()
    la = int(os.environ["LOOKAHEAD"]) if os.environ.get("LOOKAHEAD") else None
    sum(1 for e in stream_events(data, int(sys.argv[2]), lookahead=la))
    t = time.perf_counter()
    sum(1 for e in stream_events(data, int(sys.argv[2]), lookahead=la))
    out[name] = (time.perf_counter() - t) * 1e3
print(json.dumps(out))
'''
res = {"A": [], "B": []}
for r in range(reps):
    for tag, lib in (("A", liba), ("B", libb)):
        p = subprocess.run([sys.executable, "-c", code, names, str(th)], env=dict(os.environ, MI_DEC_LIB=lib),
                           capture_output=True, text=True, check=True)
        res[tag].append(json.loads(p.stdout))
for name in names.split(","):
    a = [x[name] for x in res["A"]]
    b = [x[name] for x in res["B"]]
    print(f"{name}: A min {min(a):.1f} med {statistics.median(a):.1f} | B min {min(b):.1f} med {statistics.median(b):.1f}")
