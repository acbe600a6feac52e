"""Benchmark: decoded Mpixels/s of the post-entropy AV1 reconstruction DSP path, 4K 10-bit 4:2:0.

One step = one frame through every implemented GPU stage, inputs resident in HBM:
  itx (inverse transform + add into the prediction) -> deblock (all column edges, then all
  row edges) -> CDEF (D -> C) -> loop restoration (C + D -> O) -> film grain (O -> output).
Motion compensation and intra prediction are not implemented yet: the
prediction planes are synthetic and resident. Descriptors follow SURVEY.md §8(d).

`python bench.py` runs 1 GPU. Under torch.distributed.run every rank drives its own GPU on
its own independent stream (replicas; no data-path collective; "scaling": "weak"); the
timed region is bracketed by barrier + synchronize and the max over ranks is reported.
Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from rav1d_amd import ITX_KEEP_COEFS  # noqa: E402
from rav1d_amd import frame as F  # noqa: E402
from rav1d_amd.synth import frame_bytes, itx_algorithmic_bytes, make_frame  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
W, H, BPC, LAYOUT = 3840, 2160, 10, 1


class Pipeline:
    """Device buffers + descriptors for one stream's frames."""

    def __init__(self, ctx, fr):
        self.ctx, self.fr = ctx, fr
        w, h, bpc, lay = fr["w"], fr["h"], fr["bpc"], fr["layout"]
        self.A = F.Frame(w, h, bpc, lay)      # prediction -> recon -> deblocked (in place)
        self.B = F.Frame(w, h, bpc, lay)      # CDEF output
        self.O = F.Frame(w, h, bpc, lay)      # LR output (the reference frame)
        self.G = F.Frame(w, h, bpc, lay)      # displayed picture with film grain
        for p, a in enumerate(fr["planes"]):
            self.A.set_plane_np(p, a)
        self.blocks = torch.from_numpy(fr["blocks"].view(np.uint8).copy()).cuda()
        self.coef = torch.from_numpy(fr["coef"].copy()).cuda()
        self.lf = F.LoopFilterMeta(fr["lf"])
        self.cdef = F.CdefMeta(fr["lf"]["masks"], fr["cdef"], masks_dev=self.lf.masks)
        self.lr = F.LrMeta(fr["lr"])
        self.fgd = F.film_grain_data(fr["fg"])
        self.side = torch.cuda.Stream()
        fb = frame_bytes(w, h, bpc, lay)
        # algorithmic bytes per launch: read inputs once, write outputs once
        lvl_bytes = ((w + 3) >> 2) * ((h + 3) >> 2) * 4
        mask_bytes = fr["lf"]["masks"].nbytes
        self.algo = {
            "itx": itx_algorithmic_bytes(fr["blocks"], bpc, zero_coefs=False),
            "deblock": 2 * fb + lvl_bytes + mask_bytes,
            "cdef": 2 * fb + mask_bytes,
            "lr": 2 * fb + fb * 4 // 64 + fr["lr"]["lr_mask"].nbytes,
            "fg": 2 * fb,
        }
        self.kernels = {"itx": "itx_frame_kernel", "deblock": "lf_cols_kernel+lf_rows_kernel",
                        "cdef": "cdef_kernel", "lr": "lr_kernel", "fg": "fg_apply_kernel"}

    def step(self, stream, ev=None):
        """Enqueue one frame. ev: optional dict stage -> list of (start, end) events."""
        lib = F.lib()
        ctx = self.ctx.h
        sp = F._stream_ptr(stream)
        pa, pb, po, pg = self.A.picture(), self.B.picture(), self.O.picture(), self.G.picture()

        # film-grain prep depends only on the grain parameters: side stream, overlapped
        start = torch.cuda.Event()
        start.record(stream)
        self.side.wait_event(start)
        F.check(lib.mi_film_grain_prep(ctx, ctypes.byref(pa), ctypes.byref(self.fgd),
                                       F._stream_ptr(self.side)), "fg prep")
        prep_done = torch.cuda.Event()
        prep_done.record(self.side)

        def timed(name, fn):
            if ev is not None:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                fn()
                b.record(stream)
                ev.setdefault(name, []).append((a, b))
            else:
                fn()

        ss = (ctypes.c_uint32 * 20)(*[int(v) for v in self.fr["size_start"]])
        timed("itx", lambda: F.check(lib.mi_itx_frame(ctx, ctypes.byref(pa), ctypes.c_void_p(self.blocks.data_ptr()),
                                                      ss, ctypes.c_void_p(self.coef.data_ptr()), ITX_KEEP_COEFS, sp), "itx"))
        timed("deblock", lambda: F.check(lib.mi_deblock_frame(ctx, ctypes.byref(pa), ctypes.byref(self.lf.s), sp), "lf"))
        timed("cdef", lambda: F.check(lib.mi_cdef_frame(ctx, ctypes.byref(pa), ctypes.byref(pb),
                                                        ctypes.byref(self.cdef.s), sp), "cdef"))
        timed("lr", lambda: F.check(lib.mi_lr_frame(ctx, ctypes.byref(pb), ctypes.byref(pa), ctypes.byref(po),
                                                    ctypes.byref(self.lr.s), sp), "lr"))
        stream.wait_event(prep_done)
        timed("fg", lambda: F.check(lib.mi_film_grain_apply(ctx, ctypes.byref(po), ctypes.byref(pg),
                                                            ctypes.byref(self.fgd), 0, sp), "fg"))


def cpu_baseline(fr, budget_s=20.0):
    """The oracle (single-threaded C restatement, oracle/) on a bounded sample of the same
    workload: whole 4K10 frames through all stages until ~budget_s. Luma Mpixels/s."""
    from tests.pipeline import oracle_pipeline
    n, t0 = 0, time.perf_counter()
    while True:
        oracle_pipeline(fr)
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 20:
            break
    return dict(value=round(n * fr["w"] * fr["h"] / el / 1e6, 3), unit="Mpixels/s", cores=1, kind="port",
                sample=f"{n} frame(s) of the same synthetic 4K10 descriptors through oracle/ "
                       f"(itx+deblock+cdef+lr+film grain), 1 thread, {el:.1f}s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    stream = torch.cuda.current_stream()

    fr = make_frame(W, H, BPC, LAYOUT, seed=0x4C100001 + rank)
    ctx = F.Context(local)
    pipe = Pipeline(ctx, fr)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        pipe.step(stream)
    torch.cuda.synchronize()

    # per-kernel timing pass (HIP events on the launch stream), then the clean timed pass
    ev = {}
    for _ in range(max(5, args.steps // 5)):
        pipe.step(stream, ev)
    torch.cuda.synchronize()
    stage_ms = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in ev.items()}

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.step(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    dom = max(stage_ms, key=stage_ms.get)
    achieved = pipe.algo[dom] / (stage_ms[dom] / 1e3) / 1e9
    frames = args.steps * world
    value = frames * W * H / elapsed / 1e6
    if rank == 0:
        out = {
            "metric": "decoded Mpixels/s (4K 10-bit 4:2:0, post-entropy reconstruction DSP)",
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "fps": round(frames / elapsed, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (seeded frame descriptors per SURVEY.md §8d; no CPU front-end yet)",
            "config": {"workload": f"4K10 4:2:0 {W}x{H} frame: itx+deblock+cdef+lr+film_grain "
                                   f"(mc/ipred not yet implemented; prediction planes resident)",
                       "parallelism": f"replicas{world} (one independent stream per GPU)"},
            "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
            "stage_gbs": {k: round(pipe.algo[k] / (stage_ms[k] / 1e3) / 1e9, 1) for k in stage_ms if k in pipe.algo},
            "roofline": {"kernel": pipe.kernels[dom], "stage": dom, "bound": "hbm",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "algo_bytes_per_launch": pipe.algo[dom]},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(fr)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
