"""Sum the front-end's MI_DEC_TRACE phases over a stream: python tools/dev/fe_trace_sum.py NAME THREADS"""
import json, os, re, subprocess, sys

name, th = sys.argv[1], int(sys.argv[2])
code = f"""
import sys, os; sys.path.insert(0, os.getcwd())
import json
from rav1d_amd.av1dec import stream_events
G = "tests/golden/streams"; V = {{v["name"]: v for v in json.load(open(G + "/vectors.json"))}}
data = open(os.path.join(G, V["{name}"]["file"]), "rb").read()
n = sum(1 for e in stream_events(data, {th}))
"""
err = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, MI_DEC_TRACE="1"), capture_output=True,
                     text=True).stderr
acc = dict(init=0.0, tiles_wall=0.0, tile_max=0.0, tile_sum=0.0, merge=0.0, result=0.0, job_decode=0.0, plan=0.0,
           frames=0, serial_frame=0.0)
for line in err.splitlines():
    if m := re.match(r"\s+init ([\d.]+) ms", line):
        acc["init"] += float(m[1])
    elif m := re.match(r"\s+tiles ([\d.]+) ms, each ms \(started at\):(.*)", line):
        acc["tiles_wall"] += float(m[1])
        ts = [float(x) for x in re.findall(r"([\d.]+)\(", m[2])]
        acc["tile_max"] += max(ts)
        acc["tile_sum"] += sum(ts)
    elif m := re.match(r"\s+merge ([\d.]+) ms", line):
        acc["merge"] += float(m[1])
    elif m := re.match(r"\s+job \d+: refs [\d.]+ decode ([\d.]+) plan ([\d.]+)", line):
        acc["job_decode"] += float(m[1])
        acc["plan"] += float(m[2])
    elif m := re.match(r"\s+frame ([\d.]+) ms", line):
        acc["serial_frame"] += float(m[1])
    elif line.startswith("frame "):
        acc["frames"] += 1
print(name, th, {k: round(v, 2) for k, v in acc.items()})
