"""Real streams through decode_to_muxer at 1, 2, 4 and 8 frames in flight (diagnostic):
python tools/dev/inflight.py [NAME,..]"""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
from rav1d_amd import frame as F  # noqa: E402
from rav1d_amd.output import Muxer  # noqa: E402
from rav1d_amd.stream import decode_to_muxer  # noqa: E402

G = "tests/golden/streams"
V = {v["name"]: v for v in json.load(open(G + "/vectors.json"))}
ctx = F.Context(0)
names = (sys.argv[1] if len(sys.argv) > 1 else "av1-1-b8-02-allintra,issue_318,issue_295,itut_t35,00001141").split(",")
for name in names:
    data = open(os.path.join(G, V[name]["file"]), "rb").read()
    m = Muxer("md5")
    decode_to_muxer(ctx, data, m, in_flight=4)
    ok = m.verify(V[name]["md5"]) == 0
    m.close()
    res = {}
    for k in (1, 2, 4, 8):
        best = 1e9
        for _ in range(3):
            mm = Muxer("null")
            t = time.perf_counter()
            decode_to_muxer(ctx, data, mm, in_flight=k)
            best = min(best, time.perf_counter() - t)
            mm.close()
        res[k] = round(best * 1e3, 2)
    print(name, "md5", ok, res, flush=True)
