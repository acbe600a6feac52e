"""One real stream through the executor, unpipelined, with the per-stage host/device split
(diagnostic): python tools/dev/run_rs.py NAME [reps]."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd.frame import Context
from rav1d_amd.output import Muxer
from rav1d_amd.stream import decode_to_muxer
G = os.path.join(ROOT, "tests", "golden", "streams")
V = {v["name"]: v for v in json.load(open(os.path.join(G, "vectors.json")))}
name = sys.argv[1] if len(sys.argv) > 1 else "itut_t35_10bit"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
data = open(os.path.join(G, V[name]["file"]), "rb").read()
ctx = Context(0)
m = Muxer("md5")
decode_to_muxer(ctx, data, m, apply_grain=bool(V[name].get("filmgrain")))
print(name, "md5 ok" if m.verify(V[name]["md5"]) == 0 else "MD5 MISMATCH", flush=True)
m.close()
for _ in range(reps):
    st = {}
    mm = Muxer("null")
    decode_to_muxer(ctx, data, mm, apply_grain=bool(V[name].get("filmgrain")), pipelined=False, stats=st)
    mm.close()
    print({k: round(st[k], 3) for k in ("front_end_ms", "run_host_ms", "run_levels_ms", "run_stage_ms", "intra_ms", "inter_ms", "filter_ms")}, flush=True)
