import json, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from rav1d_amd.frame import Context
from rav1d_amd.output import Muxer
from rav1d_amd.stream import decode_to_muxer
d = os.environ.get("MI_VDIR", "sweep_vectors")
table = json.load(open(os.path.join(d, "vectors.json")))
names = sys.argv[1].split(",")
ctx = Context(0)
for v in table:
    if v["name"] not in names: continue
    m = Muxer("md5")
    n = decode_to_muxer(ctx, open(os.path.join(d, v["file"]), "rb").read(), m, apply_grain=bool(v["filmgrain"]))
    got = m.digest(); m.close()
    print(os.environ.get("MI_LIB", "base").split("/")[-1], v["name"], n, "ok" if got == v["md5"] else "MISMATCH", flush=True)
