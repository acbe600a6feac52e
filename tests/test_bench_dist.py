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


class _Ev:
    """A host-clock stand-in for a pair of HIP events (elapsed_time in ms)."""

    def __init__(self):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class _OraclePipeline:
    """CPU stand-in for bench.Pipeline with its step / refill / restore / output_digest
    interface: one step runs the frame through the oracle (tests only: it exercises bench.py's
    replica harness over gloo, not the device path)."""

    def __init__(self, fr):
        import bench
        self.fr, self.digest = fr, None
        fb = 2 * fr["w"] * fr["h"] * 3 // 2
        self.algo = {k: 2 * fb for k in ("mc", "itx", "deblock", "cdef", "lr")}
        self.launches = {k: 1 for k in self.algo}
        self.kernels = {k: k for k in self.algo}
        self._bench = bench

    def step(self, stream, ev=None, mark=None):
        a = _Ev()
        self.digest = self._bench.oracle_digest(self.fr)
        if ev is not None:
            ev.setdefault("lr", []).append((a, _Ev()))

    def refill(self):
        pass

    def restore(self):
        self.digest = None

    def output_digest(self):
        return self.digest


class _CpuHw:
    device, backend = "cpu", "gloo"

    def setup(self, local):
        pass

    def pg_kwargs(self, local):
        return {}

    def context(self, local):
        return None

    def pipeline(self, ctx, fr, ring):
        return _OraclePipeline(fr)

    def sync(self):
        pass

    def stream(self, new=False):
        return None

    def oracle_digest(self, fr):
        import bench
        return bench.oracle_digest(fr)


def _main_worker(rank, world, port, q):
    import contextlib
    import io
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import bench
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.main(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--frame", "128x64"], hw=_CpuHw())
    q.put((rank, rc, buf.getvalue()))


def test_main_replica_path_world2():
    """bench.main()'s replica path end to end over gloo at world 2 (tiny frame, oracle
    stand-in for the device): one JSON line from rank 0 with n_gpus 2, both ranks in per_rank,
    and each rank's digest equal to the oracle's for its own stream (seed + rank)."""
    import json
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_main_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    res = sorted((q.get() for _ in range(world)), key=lambda x: x[0])
    assert [rc for _, rc, _ in res] == [0, 0]
    lines = [ln for ln in res[0][2].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and not res[1][2].strip()       # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and out["verified"] is True
    assert [r["rank"] for r in out["per_rank"]] == [0, 1]
    import bench
    from rav1d_amd.synth import make_frame
    for r in out["per_rank"]:
        fr = make_frame(128, 64, 10, 1, seed=0x4C100001 + r["rank"], with_fg=False, with_mc=True)
        assert r["sha256"] == bench.oracle_digest(fr)
    assert out["per_rank"][0]["sha256"] != out["per_rank"][1]["sha256"]
    assert out["value"] > 0 and out["frame"] == "128x64"


def test_world_size_must_match_gpus(monkeypatch):
    """Under a launcher, --gpus must equal WORLD_SIZE (a mismatch would report the wrong n_gpus)."""
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.main(["--gpus", "4"], hw=_CpuHw()) == 2


def test_gpus_n_without_launcher_spawns_ranks(monkeypatch):
    """--gpus N with no WORLD_SIZE starts N rank processes (no GPU call in the parent) and
    returns the first failing rank's exit code. Without a GPU each child fails at its first
    device call (torch.cuda.set_device), so the parent must report a failure."""
    import torch

    import bench
    if torch.cuda.is_available():
        pytest.skip("needs a host without a GPU")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    rc = bench.main(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert rc not in (0, None)
