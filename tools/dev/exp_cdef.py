"""CDEF timing on the bench's synthetic 4K10 frame for each library in argv (diagnostic, not a test).
usage: python tools/dev/exp_cdef.py lib1.so [lib2.so ...]  (each run in a child process)"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if len(sys.argv) > 1 and sys.argv[1] != "--child":
    for lib in sys.argv[1:]:
        r = subprocess.run([sys.executable, __file__, "--child"], env=dict(os.environ, MI_LIB=lib),
                           capture_output=True, text=True, timeout=300)
        print(os.path.basename(lib), r.stdout.strip(), r.stderr.strip()[-300:] if r.returncode else "")
    sys.exit(0)

sys.path.insert(0, ROOT)
import torch
from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame, frame_bytes

w, h, bpc = 3840, 2160, 10
fr = make_frame(w, h, bpc, 1, seed=0x4C100001, with_fg=False, with_mc=False)
ctx = F.Context(0)
A, C = F.Frame(w, h, bpc, 1), F.Frame(w, h, bpc, 1)
for p, a in enumerate(fr["planes"]):
    A.set_plane_np(p, a)
meta = F.CdefMeta(fr["lf"]["masks"], fr["cdef"])
algo = 2 * frame_bytes(w, h, bpc, 1)
fn = lambda: F.cdef_frame(ctx, A, C, meta)
for _ in range(5):
    fn()
torch.cuda.synchronize()
best = 1e9
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) / 50 * 1e3)
print(f"cdef {best:8.1f} us  {algo / best / 1e3:7.1f} GB/s (algorithmic)")
