"""The front-end's MI_DEC_TRACE lines for one stream decoded one temporal unit at a time
(lookahead 0, as bench.py's unpipelined pass): python tools/dev/fe_trace_la0.py NAME [THREADS]"""
import json, os, subprocess, sys

name = sys.argv[1]
th = int(sys.argv[2]) if len(sys.argv) > 2 else 8
code = f"""
import sys, os, json, time; sys.path.insert(0, os.getcwd())
from rav1d_amd.av1dec import stream_events
G = "tests/golden/streams"; V = {{v["name"]: v for v in json.load(open(G + "/vectors.json"))}}
data = open(os.path.join(G, V["{name}"]["file"]), "rb").read()
sum(1 for e in stream_events(data, {th}, lookahead=0))
t = time.perf_counter(); sum(1 for e in stream_events(data, {th}, lookahead=0))
print("wall_ms", (time.perf_counter() - t) * 1e3, file=sys.stderr)
"""
err = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, MI_DEC_TRACE="1"), capture_output=True,
                     text=True).stderr
lines = err.splitlines()
# the second pass only
k = max(i for i, l in enumerate(lines) if l.startswith("frame 0:"))
print("\n".join(lines[k:]))
