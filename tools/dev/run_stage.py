"""One bench stage (STAGE=deblock|cdef|lr|itx|mc|mc_onegrid|mc_split|mc_sync) of the 4K10 bench frame, REPS times, for PMC
passes (diagnostic). The pipeline runs once first so every input is the real one."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import ctypes
import torch
import bench
from rav1d_amd import frame as F
from rav1d_amd.synth import make_frame
fr = make_frame(3840, 2160, 10, 1, seed=0x4C100001, with_fg=False, with_mc=True, packed=not os.environ.get("DENSE"))
ctx = F.Context(0)
pipe = bench.Pipeline(ctx, fr, ring=2)
s = torch.cuda.current_stream()
pipe.step(s)
torch.cuda.synchronize()
L = F.lib()
st = os.environ.get("STAGE", "deblock")
lr_grid = F.MiLr.from_buffer_copy(pipe.lr.s)   # the same LR call in grid order
lr_grid.order = None
cdef_grid = F.MiCdef.from_buffer_copy(pipe.cdef.s)
cdef_grid.order = None
sp = F._stream_ptr(s)
pa, pb, po, pd = pipe.A.picture(), pipe.B.picture(), pipe.O.picture(), pipe.D.picture()
def mc(p, flags=0):
    F.check(L.mi_mc_frame_ex(ctx.h, ctypes.byref(pa), pipe.ref_pics, len(pipe.refs), ctypes.c_void_p(pipe.mc.blocks.data_ptr()),
                             pipe.mc.class_start, ctypes.c_void_p(pipe.mc.masks.data_ptr()), None, flags, p), "mc")


def mc_sync(p):
    F.check(L.mi_mc_frame_sync(ctx.h, ctypes.byref(pa), pipe.ref_pics, len(pipe.refs), ctypes.c_void_p(pipe.mc.blocks.data_ptr()),
                               pipe.mc.class_start, ctypes.c_void_p(pipe.mc.masks.data_ptr()), pipe.mc.masks.numel(), None, p),
            "mc sync")


split = None


def mc_split(p):
    """the caller-side split: luma + independent chroma in one grid, the chroma MASK units after"""
    global split
    if split is None:
        split = F.McSplitMeta(fr["mc"][0], fr["mc"][2])
    F.check(L.mi_mc_frame_ex(ctx.h, ctypes.byref(pa), pipe.ref_pics, len(pipe.refs), ctypes.c_void_p(split.a.blocks.data_ptr()),
                             split.a.class_start, ctypes.c_void_p(split.masks.data_ptr()), None, 1, p), "mc a")
    if split.b.n:
        F.check(L.mi_mc_frame(ctx.h, ctypes.byref(pa), pipe.ref_pics, len(pipe.refs), ctypes.c_void_p(split.b.blocks.data_ptr()),
                              split.b.class_start, ctypes.c_void_p(split.masks.data_ptr()), None, p), "mc b")


def itx(p):
    # STAGE=itx_dc: as the bench runs it, the DC-only runs deferred into the DC map
    fl = bench.ITX_KEEP_COEFS | (bench.ITX_DC_DEFER if st == "itx_dc" else 0)
    F.check(L.mi_itx_frame_runs(ctx.h, ctypes.byref(pa), ctypes.c_void_p(pipe.blocks.data_ptr()), pipe.itx_bands,
                                pipe.itx_dc_end, ctypes.c_void_p(pipe.coefs[0].data_ptr()), fl, p), "itx")


for _ in range(int(os.environ.get("REPS", "10"))):
    if st in ("itx", "itx_dc"):
        itx(sp)
    elif st == "mc":
        mc(sp)
    elif st == "mc_onegrid":   # (timing only: chroma units that read a luma SEG mask race with it)
        mc(sp, 1)
    elif st == "mc_split":
        mc_split(sp)
    elif st == "mc_sync":
        mc_sync(sp)
    elif st == "deblock":
        F.check(L.mi_deblock_frame_to(ctx.h, ctypes.byref(pa), ctypes.byref(pd), ctypes.byref(pipe.lf.s), sp), "lf")
    elif st == "cdef":
        F.check(L.mi_cdef_frame(ctx.h, ctypes.byref(pd), ctypes.byref(pb), ctypes.byref(pipe.cdef.s), sp), "cdef")
    elif st == "lr":
        F.check(L.mi_lr_frame(ctx.h, ctypes.byref(pb), ctypes.byref(pd), ctypes.byref(po), ctypes.byref(pipe.lr.s), sp), "lr")
    elif st == "lr_grid":
        F.check(L.mi_lr_frame(ctx.h, ctypes.byref(pb), ctypes.byref(pd), ctypes.byref(po), ctypes.byref(lr_grid), sp), "lr")
    elif st == "cdef_grid":
        F.check(L.mi_cdef_frame(ctx.h, ctypes.byref(pd), ctypes.byref(pb), ctypes.byref(cdef_grid), sp), "cdef")
torch.cuda.synchronize()
print("done")
if os.environ.get("TIME"):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gtime import gtime

    def one(stream):
        p = F._stream_ptr(stream)
        if st in ("itx", "itx_dc"):
            itx(p)
        elif st == "mc":
            mc(p)
        elif st == "mc_onegrid":
            mc(p, 1)
        elif st == "mc_split":
            mc_split(p)
        elif st == "mc_sync":
            mc_sync(p)
        elif st == "deblock":
            F.check(L.mi_deblock_frame_to(ctx.h, ctypes.byref(pa), ctypes.byref(pd), ctypes.byref(pipe.lf.s), p), "lf")
        elif st == "cdef":
            F.check(L.mi_cdef_frame(ctx.h, ctypes.byref(pd), ctypes.byref(pb), ctypes.byref(pipe.cdef.s), p), "cdef")
        elif st == "lr":
            F.check(L.mi_lr_frame(ctx.h, ctypes.byref(pb), ctypes.byref(pd), ctypes.byref(po), ctypes.byref(pipe.lr.s), p), "lr")
        elif st == "lr_grid":
            F.check(L.mi_lr_frame(ctx.h, ctypes.byref(pb), ctypes.byref(pd), ctypes.byref(po), ctypes.byref(lr_grid), p), "lr")
        elif st == "cdef_grid":
            F.check(L.mi_cdef_frame(ctx.h, ctypes.byref(pd), ctypes.byref(pb), ctypes.byref(cdef_grid), p), "cdef")
    print(f"{st} {gtime(one):.2f} us", flush=True)
