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


def _digest_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from rav1d_amd.synth import make_frame
    cfg = bench.broadcast_config({"w": 256, "h": 128, "seeds": [1000 + 7 * r for r in range(world)]}
                                 if rank == 0 else None, world)
    fr = make_frame(cfg["w"], cfg["h"], 10, 1, seed=cfg["seeds"][rank], with_fg=False, with_mc=True)
    d = bench.oracle_digest(fr)
    res = bench.gather_results({"rank": rank, "frames": 1, "ns": 1, "sha256": d, "verified": True}, world)
    q.put((rank, cfg, res))
    dist.destroy_process_group()


def test_config_broadcast_and_per_rank_digests():
    """SURVEY.md 8(e) collectives on gloo: rank 0's config reaches every rank, and every rank
    sees all ranks' output digests; each digest is that rank's own pipeline output (seed + rank),
    recomputed here through the oracle."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_digest_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    res = sorted((q.get() for _ in range(world)), key=lambda x: x[0])
    import bench
    from rav1d_amd.synth import make_frame
    cfg = res[0][1]
    assert res[1][1] == cfg
    for rank, _, gathered in res:
        assert [g["rank"] for g in gathered] == list(range(world))
        for g in gathered:
            fr = make_frame(cfg["w"], cfg["h"], 10, 1, seed=cfg["seeds"][g["rank"]], with_fg=False, with_mc=True)
            assert g["sha256"] == bench.oracle_digest(fr)
    assert res[0][2][0]["sha256"] != res[0][2][1]["sha256"]   # different streams per rank
