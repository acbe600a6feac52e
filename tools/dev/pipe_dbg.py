import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd import frame as F
from rav1d_amd.output import Muxer
from rav1d_amd.stream import decode_to_muxer
g = os.path.join(ROOT, "tests/golden/streams")
for name in ("av1-1-b8-02-allintra", "itut_t35_10bit"):
    v = [x for x in json.load(open(g + "/vectors.json")) if x["name"] == name][0]
    data = open(os.path.join(g, v["file"]), "rb").read()
    for th, fl in [(8, 1)] * 6 + [(1, 1)] * 2:
        ctx = F.Context(0)
        m = Muxer("md5")
        t = time.perf_counter()
        n = decode_to_muxer(ctx, data, m, threads=th, in_flight=fl)
        dt = time.perf_counter() - t
        print(name, th, fl, n, m.digest() == v["md5"], round(dt * 1e3, 1), "ms", flush=True)
        m.close()
