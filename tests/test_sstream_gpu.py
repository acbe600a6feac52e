"""Single-stream frame pipelining on the device: two ranks (processes) on cuda:0 exchange
reference pictures (host-staged gloo here; RCCL send/recv under nccl on a multi-GPU node) and
reconstruct their frames with the batched kernels; every frame equals the oracle's sequential
decode of the same stream, and frame k ran on rank k % 2."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from rav1d_amd.sstream import make_stream_specs, picture_digest
from tests.test_sstream_dist import _free_port, sequential_digests, W, H, BPC, LAYOUT, N, SEED

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, q, bands=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rav1d_amd.frame import Context
    from rav1d_amd.sstream import DeviceExecutor, PipelinedStream
    ctx = Context(0)
    specs = make_stream_specs(W, H, BPC, LAYOUT, N, SEED)
    ex = DeviceExecutor(ctx, bands=bands)
    for s in specs:
        if s.idx % world == rank:
            ex.prepare(s)
    mine = PipelinedStream(ex, ex.alloc, rank, world, "cuda", bands=bands).run(specs)
    torch.cuda.synchronize()
    local = {i: picture_digest([f.plane_np(p) for p in range(len(f.planes))]) for i, f in mine.items()}
    out = [None] * world
    dist.all_gather_object(out, local)
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("bands", [1, 3])
def test_device_pipelined_stream_equals_oracle_sequential(bands):
    """bands 3: row-level progress (references in bands, MC launched per band group)."""
    specs = make_stream_specs(W, H, BPC, LAYOUT, N, SEED)
    want = sequential_digests(specs)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, bands)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    got = {}
    for _, gathered in res:
        for r, d in enumerate(gathered):
            assert all(i % world == r for i in d)
            got.update(d)
    assert got == want


def test_device_single_rank_stream_equals_oracle_sequential(gpu):
    """world 1 (no process group): the same scheduler runs every frame locally."""
    import torch
    from rav1d_amd.sstream import DeviceExecutor, PipelinedStream
    specs = make_stream_specs(W, H, BPC, LAYOUT, N, SEED)
    ex = DeviceExecutor(gpu)
    mine = PipelinedStream(ex, ex.alloc, 0, 1, "cuda").run(specs)
    torch.cuda.synchronize()
    got = {i: picture_digest([f.plane_np(p) for p in range(len(f.planes))]) for i, f in mine.items()}
    assert got == sequential_digests(specs)
