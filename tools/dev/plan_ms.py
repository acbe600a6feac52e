"""Host planning time of mi_frame_run per frame (mi_frame_plan_ms; CPU only, no GPU needed)."""
import ctypes, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd import lib
from rav1d_amd.av1dec import Av1Decoder, stream_units
G = os.path.join(ROOT, "tests", "golden", "streams")
V = {v["name"]: v for v in json.load(open(os.path.join(G, "vectors.json")))}
L = lib()
L.mi_frame_plan_ms.restype = ctypes.c_double
L.mi_frame_plan_ms.argtypes = [ctypes.c_void_p, ctypes.c_int]
for name in sys.argv[1:] or ["itut_t35_10bit", "00001141", "issue_318"]:
    data = open(os.path.join(G, V[name]["file"]), "rb").read()
    dec = Av1Decoder()
    tot, nf, mx = 0.0, 0, 0.0
    for u in stream_units(data):
        dec.send(u)
        for e in dec.events():
            if e.frame:
                ms = L.mi_frame_plan_ms(ctypes.cast(e.frame, ctypes.c_void_p), 3)
                tot += ms; nf += 1; mx = max(mx, ms)
    print(f"{name}: {nf} frames, plan {tot:.2f} ms total, max {mx:.2f} ms/frame")
