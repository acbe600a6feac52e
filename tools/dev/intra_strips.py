"""Device intra time of the reference's intra-heavy streams through mi_frame_run (frames split in
XCD strips unless MI_IR_STRIPS=1), MD5-checked. Dev experiment: python tools/dev/intra_strips.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd.frame import Context  # noqa: E402
from rav1d_amd.output import Muxer  # noqa: E402
from rav1d_amd.stream import decode_to_muxer  # noqa: E402

g = os.path.join(ROOT, "tests/golden/streams")
vecs = {v["name"]: v for v in json.load(open(g + "/vectors.json"))}
ctx = Context(0)
tag = os.environ.get("MI_IR_STRIPS", "8")
for name in sys.argv[1:] or ["itut_t35", "itut_t35_10bit", "00001141", "av1-1-b8-02-allintra", "issue_318"]:
    v = vecs[name]
    data = open(os.path.join(g, v["file"]), "rb").read()
    best, ok = None, True
    for _ in range(3):
        m = Muxer("md5")
        st = {}
        decode_to_muxer(ctx, data, m, apply_grain=bool(v.get("filmgrain")), pipelined=False, stats=st)
        ok = ok and m.digest() == v["md5"]
        m.close()
        best = st["intra_ms"] if best is None else min(best, st["intra_ms"])
    print(f"strips={tag} {name:24s} intra_ms {best:8.3f} md5_ok {ok}", flush=True)
