"""Phase stamps of the film-grain prep kernel (diagnostic; MI_LIB=librav1d_amd_ktl.so): fill,
AR wavefronts, template export, scaling LUTs, in us (s_memrealtime, 100 MHz)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from rav1d_amd import frame as F
from rav1d_amd.synth import make_fg_params
L = F.lib()
buf = torch.zeros(64, dtype=torch.int64, device="cuda")
ctx = F.Context(0)
src = F.Frame(7680, 4320, 10, 1)
ps = src.picture()
for lag in (int(a) for a in os.environ.get("LAGS", "3,2,1,0").split(",")):
    rng = np.random.default_rng(0xF6000001)
    fg = make_fg_params(rng, 1)
    fg["ar_coeff_lag"] = lag
    d = F.film_grain_data(fg)
    s = torch.cuda.current_stream()
    for it in range(3):
        L.mi_ktl_set_fg(ctypes.c_void_p(buf.data_ptr() if it == 2 else 0))
        F.check(L.mi_film_grain_prep(ctx.h, ctypes.byref(ps), ctypes.byref(d), F._stream_ptr(s)), "prep")
        torch.cuda.synchronize()
    t = buf.cpu().numpy()[:5].astype(np.float64)
    print(f"lag {lag}: fill {(t[1]-t[0])/100:.2f} ar {(t[2]-t[1])/100:.2f} export {(t[3]-t[2])/100:.2f} "
          f"scaling {(t[4]-t[3])/100:.2f} total {(t[4]-t[0])/100:.2f} us", flush=True)
