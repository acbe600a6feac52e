"""Debug: fused intra recon on a small frame, short spin limit, host-mapped progress words."""
import sys, os, time, ctypes
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rav1d_amd.frame import Frame, Context
from rav1d_amd.ipred_synth import make_intra_frame
from rav1d_amd.intra import IntraFrame, make_intra_residuals, intra_recon
from rav1d_amd import frame as F
w, h, bpc, layout = int(sys.argv[1]), int(sys.argv[2]), 8, 0
rng = np.random.default_rng(5)
fr = make_intra_residuals(make_intra_frame(w, h, bpc, layout, rng), bpc, rng)
n = len(fr["blocks"])
print("blocks", n, "levels", len(fr["level_start"]) - 1, flush=True)
ctx = Context(0)
cur = Frame(w, h, bpc, layout)
it = IntraFrame(ctx, fr)
print("dep_start", it.dep_start.cpu().numpy()[:10], "deps", it.deps.cpu().numpy()[:10], flush=True)
ev = torch.cuda.Event()
intra_recon(ctx, [(it, cur.picture())])
ev.record()
libc = ctypes.CDLL(None); libc.getenv.restype = ctypes.c_char_p
p = int(libc.getenv(b"MI_IR_DBG_PTR"))
dbg = (ctypes.c_int * 65536).from_address(p)
for t in range(6):
    time.sleep(0.25)
    done = ev.query()
    print(f"t={t} done={done} per-xcc WGs {list(dbg[16:24])} per-b%8 {list(dbg[32:40])} stages {list(dbg[64:64 + min(n, 32)])} info {[hex(v & 0xffffffff) for v in dbg[64 + 1024:64 + 1024 + min(n, 8)]]}", flush=True)
    if done:
        break
if not ev.query():
    print("HUNG", flush=True)
    os._exit(3)
print("status", F.lib().mi_ctx_device_status(ctx.h, F._stream_ptr(None)), flush=True)
