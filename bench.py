"""Benchmark: decoded Mpixels/s of the post-entropy reconstruction DSP path on 4K 10-bit 4:2:0.

One step = one frame through every implemented GPU stage (inputs already resident in HBM):
see STAGES below and DESIGN.md §Measurement. Launch: `python bench.py` (1 GPU) or under
torch.distributed.run with one rank per GPU (independent streams, no data-path collective,
"scaling": "weak"). Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from rav1d_amd.frame import Context, Frame, itx_frame  # noqa: E402
from rav1d_amd.synth import itx_algorithmic_bytes, make_itx_frame  # noqa: E402
from rav1d_amd import ITX_KEEP_COEFS  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
W, H, BPC = 3840, 2160, 10


class ItxStage:
    name = "itx"
    kernel = "itx_frame_kernel"

    def __init__(self, ctx, frame, seed):
        fr = make_itx_frame(W, H, bpc=BPC, seed=seed)
        self.fr = fr
        self.ctx, self.frame = ctx, frame
        for p, arr in enumerate(fr["planes"]):
            frame.set_plane_np(p, arr)
        self.blocks = torch.from_numpy(fr["blocks"].view(np.uint8).copy()).cuda()
        self.coef = torch.from_numpy(fr["coef"].copy()).cuda()
        self.size_start = fr["size_start"]
        # The device arena is re-uploaded per frame by the front-end, so the batched path
        # leaves it untouched (MI_ITX_KEEP_COEFS); see DESIGN.md.
        self.algo_bytes = itx_algorithmic_bytes(fr["blocks"], BPC, zero_coefs=False)
        self.n_blocks = len(fr["blocks"])

    def run(self, stream):
        itx_frame(self.ctx, self.frame, self.blocks, self.size_start, self.coef,
                  ITX_KEEP_COEFS, stream)

    def cpu_sample(self, oracle_lib):
        planes = [p.copy() for p in self.fr["planes"]]
        oracle_lib.itx_frame(planes, self.fr["blocks"], self.fr["coef"].copy(), BPC)


def build_stages(ctx, frame, seed):
    return [ItxStage(ctx, frame, seed)]


def cpu_baseline(stages, budget_s=12.0):
    """Oracle (single-threaded C restatement) on a bounded sample: whole frames of the same
    workload, repeated until ~budget_s. Reported as Mpx/s of luma."""
    from tests import oracle_lib
    oracle_lib.load_oracle()
    n, t0 = 0, time.perf_counter()
    while True:
        for st in stages:
            st.cpu_sample(oracle_lib)
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 50:
            break
    return dict(value=round(n * W * H / el / 1e6, 3), unit="Mpixels/s", cores=1, kind="port",
                sample=f"{n} frame(s) of the same 4K10 synthetic workload through oracle/ "
                       f"(stages: {','.join(s.name for s in stages)}), 1 thread, {el:.1f}s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    stream = torch.cuda.current_stream()

    ctx = Context(local)
    frame = Frame(W, H, BPC, 1)
    stages = build_stages(ctx, frame, seed=0x4C100001 + rank)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        for st in stages:
            st.run(stream)
    torch.cuda.synchronize()

    ev = {st.name: [] for st in stages}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for st in stages:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record(stream)
            st.run(stream)
            b.record(stream)
            ev[st.name].append((a, b))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    per_stage_ms = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in ev.items()}
    dom = max(stages, key=lambda s: per_stage_ms[s.name])
    dom_s = per_stage_ms[dom.name] / 1e3
    achieved = dom.algo_bytes / dom_s / 1e9

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
            "data": "synthetic (seeded frame descriptors, SURVEY.md §8d; no front-end yet)",
            "config": {"workload": f"4K10 4:2:0 {W}x{H} frame: " + "+".join(s.name for s in stages),
                       "parallelism": f"replicas{world} (independent streams, one per GPU)"},
            "stage_ms": {k: round(v, 4) for k, v in per_stage_ms.items()},
            "roofline": {"kernel": dom.kernel, "bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None, "algo_bytes_per_launch": dom.algo_bytes},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(stages)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
