"""Single-stream frame pipelining across ranks (rav1d_amd.sstream), world_size 2 on gloo/CPU:
the scheduler and its reference exchange, with the oracle reconstructing each frame, must give
exactly the pictures of a sequential decode of the same stream (and the GPU test runs the
device executor through the same scheduler)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rav1d_amd.sstream import gop_specs, make_stream_specs, picture_digest, transfer_plan

W, H, BPC, LAYOUT, N, SEED = 128, 64, 8, 1, 11, 0x55000001


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OraclePicture:
    def __init__(self, planes_np):
        self.np = [np.ascontiguousarray(a) for a in planes_np]
        self.planes = [torch.from_numpy(a.view(np.uint8)) for a in self.np]


def oracle_executor(spec, refs):
    """Test executor: the CPU restatement of the same stages (tests/pipeline.py)."""
    from tests.pipeline import oracle_pipeline
    fr = dict(spec.desc)
    fr["refs"] = [r.np for r in refs] if refs else None
    if not refs:
        fr["mc"] = None
    out = oracle_pipeline(fr)["lr"]
    ss_h, ss_v = int(LAYOUT in (1, 2)), int(LAYOUT == 1)
    dims = [(H, W)] + [((H + ss_v) >> ss_v, (W + ss_h) >> ss_h)] * 2
    return OraclePicture([out[p][:dims[p][0], :dims[p][1]] for p in range(len(out))])


def oracle_alloc(spec):
    ss_h, ss_v = int(LAYOUT in (1, 2)), int(LAYOUT == 1)
    dt = np.uint8 if BPC == 8 else np.uint16
    dims = [(H, W)] + [((H + ss_v) >> ss_v, (W + ss_h) >> ss_h)] * 2
    # receive buffers start as a sentinel: a row still holding it was not received
    return OraclePicture([np.full(d, SENTINEL, dt) for d in dims])


SENTINEL = 0xA5
BANDS = 3


def band_oracle_executor(spec, refs, ready):
    """Row-level progress check: for every band group g, after ready(g) every reference row
    the group's MC units read (bands 0..g of every plane) must have arrived; then the frame
    is reconstructed from the complete references as before."""
    from rav1d_amd.sstream import band_height, band_rows, mc_band_groups
    if ready is not None and spec.desc.get("mc") is not None:
        units = spec.desc["mc"][0]
        grp = mc_band_groups(units, H, LAYOUT, BANDS)
        bh, ss_v = band_height(H, BANDS), int(LAYOUT == 1)
        for g in range(BANDS):
            ready(g)
            if not (grp == g).any():
                continue
            for r in refs:
                for p, a in enumerate(r.np):
                    hi = band_rows(g, bh, H, ss_v if p else 0)[1]
                    assert not (a[:hi] == SENTINEL).all(axis=1).any(), (spec.idx, g, p)
    return oracle_executor(spec, refs)


def sequential_digests(specs):
    pics = {}
    for s in specs:
        pics[s.idx] = oracle_executor(s, [pics[r] for r in s.refs])
    return {i: picture_digest(p.np) for i, p in pics.items()}


def _worker(rank, world, port, q, bands=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rav1d_amd.sstream import PipelinedStream
    specs = make_stream_specs(W, H, BPC, LAYOUT, N, SEED)
    ex = band_oracle_executor if bands > 1 else oracle_executor
    mine = PipelinedStream(ex, oracle_alloc, rank, world, "cpu", bands=bands).run(specs)
    local = {i: picture_digest([p.view(np.uint8 if BPC == 8 else np.uint16) for p in [t.numpy() for t in pic.planes]])
             for i, pic in mine.items()}
    out = [None] * world
    dist.all_gather_object(out, local)
    q.put((rank, out))
    dist.destroy_process_group()


def test_gop_structure():
    g = gop_specs(9, 8)
    assert [d for d, _ in g] == [0, 8, 4, 2, 1, 3, 6, 5, 7]
    dec = {d: i for i, (d, _) in enumerate(g)}
    for d, refs in g:
        assert all(r < dec[d] for r in refs)            # references precede in decode order
    assert gop_specs(1, 8) == [(0, [])]


def test_transfer_plan_only_cross_rank():
    specs = make_stream_specs(64, 32, 8, 1, 9, 1)
    plan = transfer_plan(specs, 2)
    for r, dsts in plan.items():
        assert r % 2 not in dsts
        assert all(any(s.idx % 2 == q and r in s.refs for s in specs) for q in dsts)


def test_mc_band_groups_cover_reads():
    """Every unit's group covers the reference rows its 8-tap window reads, and a chroma MASK
    unit never runs before the luma unit whose mask it reads."""
    from rav1d_amd.sstream import band_height, mc_band_groups
    from rav1d_amd.synth import make_mc_units
    w, h, bands = 256, 192, 5
    rng = np.random.default_rng(7)
    units, _, _ = make_mc_units(w, h, 1, rng, nrefs=2, compound_frac=0.6, mv_px=48)
    g = mc_band_groups(units, h, 1, bands)
    bh = band_height(h, bands)
    for u, gi in zip(units, g):
        sv = 1 if u["plane"] else 0
        for k in range(2):
            if u["ref"][k] < 0:
                continue
            last = ((int(u["y"]) + int(u["h"]) + (int(u["mvy"][k]) >> (3 + sv)) + 4) << sv) + sv
            assert last >= h - 1 and gi == bands - 1 or last < (gi + 1) * bh, (u, gi)
    lg = {(int(u["x"]), int(u["y"])): gi for u, gi in zip(units, g) if u["plane"] == 0}
    for u, gi in zip(units, g):
        if u["plane"] > 0 and u["ref"][1] >= 0 and u["comp"] == 2:
            assert gi >= lg[(int(u["x"]) * 2, int(u["y"]) * 2)]
    assert len(set(g.tolist())) > 1


@pytest.mark.parametrize("world,bands", [(2, 1), (2, BANDS)])
def test_pipelined_stream_equals_sequential(world, bands):
    """bands > 1: references travel in bands and MC waits per band (row-level progress)."""
    specs = make_stream_specs(W, H, BPC, LAYOUT, N, SEED)
    want = sequential_digests(specs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, bands)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    got = {}
    for rank, gathered in res:
        for r, d in enumerate(gathered):
            assert all(i % world == r for i in d)        # frame k ran on rank k % N
            got.update(d)
    assert got == want
