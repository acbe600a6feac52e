"""decode_to_muxer wall time with 1 and 2 device lanes (null muxer), best of N. Dev experiment."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd.frame import Context  # noqa: E402
from rav1d_amd.output import Muxer  # noqa: E402
from rav1d_amd.stream import decode_to_muxer  # noqa: E402

g = os.path.join(ROOT, "tests/golden/streams")
vecs = {v["name"]: v for v in json.load(open(g + "/vectors.json"))}
ctx = Context(0)
for name in sys.argv[1:] or ["av1-1-b8-02-allintra", "ccvb_film_grain-fg", "00000623"]:
    data = open(os.path.join(g, vecs[name]["file"]), "rb").read()
    for fl in (1, 2, 1, 2):
        best = 1e9
        for _ in range(3):
            m = Muxer("null")
            t = time.perf_counter()
            n = decode_to_muxer(ctx, data, m, in_flight=fl, apply_grain=False)
            best = min(best, time.perf_counter() - t)
            m.close()
        m = Muxer("md5")
        decode_to_muxer(ctx, data, m, in_flight=fl, apply_grain=bool(vecs[name].get("filmgrain")))
        ok = m.digest() == vecs[name]["md5"]
        m.close()
        print(name, "in_flight", fl, "frames", n, "ms", round(best * 1e3, 2), "md5_ok", ok, flush=True)
