"""Host-side cost of mi_frame_run without a GPU (diagnostic): validation and planning per
frame of a stream (mi_frame_validate, mi_frame_plan_ms)."""
import ctypes, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd import lib
from tests.test_frame_validate import frames_with_pictures, validate, GOLDEN, VECTORS
V = {v["name"]: v for v in VECTORS}
L = lib()
for name in sys.argv[1:] or ["itut_t35_10bit"]:
    data = open(os.path.join(GOLDEN, V[name]["file"]), "rb").read()
    for fr, ps, _ in frames_with_pictures(data):
        vb = 1e9
        for _ in range(5):
            t0 = time.perf_counter(); rc, why = validate(fr, ps); vb = min(vb, time.perf_counter() - t0)
        pm = L.mi_frame_plan_ms(ctypes.byref(fr), 5)
        print(f"{name}: n_intra {fr.n_intra} validate {vb * 1e3:.3f} ms (rc {rc}) plan {pm:.3f} ms", flush=True)
