"""Per-stage breakdown (decode_to_muxer stats) of a few reference streams. Dev experiment."""
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
for name in sys.argv[1:] or ["itut_t35_10bit", "00001141", "issue_318"]:
    data = open(os.path.join(g, vecs[name]["file"]), "rb").read()
    for _ in range(2):
        st = {}
        m = Muxer("null")
        decode_to_muxer(ctx, data, m, apply_grain=False, pipelined=False, stats=st)
        m.close()
    print(name, {k: round(v, 2) if isinstance(v, float) else v for k, v in st.items()}, flush=True)
