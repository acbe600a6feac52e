"""Single-frame intra reconstruction with and without XCD spreading (MI_IR_SPREAD): bench's
1080p8 intra measurement and the real streams end to end (diagnostic, not a test)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
from rav1d_amd import frame as F
ctx = F.Context(0)
r = bench.intra_1080p8(ctx)
print(os.environ.get("MI_IR_SPREAD", "0"), "intra", json.dumps({k: v for k, v in r.items() if "single" in k or "batch" in k or "ms" in k})[:400])
rs = bench.real_streams(ctx, reps=3)
for k, v in rs.items():
    print(os.environ.get("MI_IR_SPREAD", "0"), k, v["md5_verified"], v["gpu_end_to_end_ms"], v["front_end_ms"])
