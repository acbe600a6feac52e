"""The multi-GPU bench harness on CPU: world_size-2 gloo, each rank a replica with its own
step cost; the timed region reports the MAX over ranks (bench.timed_region), as the driver's
N-GPU runs do over RCCL."""
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    delay = 0.01 * (rank + 1)           # rank 1 is the slow replica
    calls = []
    el = bench.timed_region(lambda: (calls.append(1), time.sleep(delay)), 5, lambda: None, world, "cpu")
    q.put((rank, el, len(calls)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_timed_region_max_over_ranks(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    els = [e for _, e, _ in res]
    assert all(n == 5 for _, _, n in res)          # exactly `steps` steps per rank
    assert max(els) - min(els) < 1e-9              # every rank reports the same (reduced) time
    assert els[0] >= 5 * 0.02                      # ... and it is the slow rank's
