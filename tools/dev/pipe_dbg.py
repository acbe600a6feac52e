import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd import frame as F
from rav1d_amd.output import Muxer
from rav1d_amd.stream import decode_to_muxer
g = os.path.join(ROOT, "tests/golden/streams")
v = [x for x in json.load(open(g + "/vectors.json")) if x["name"] == "av1-1-b8-02-allintra"][0]
data = open(os.path.join(g, v["file"]), "rb").read()
for th, fl in [(8, 2)] * 4 + [(1, 2)] * 4 + [(8, 1)] * 4:
    ctx = F.Context(0)
    m = Muxer("md5")
    n = decode_to_muxer(ctx, data, m, threads=th, in_flight=fl)
    print(th, fl, n, m.digest() == v["md5"], flush=True)
    m.close()
