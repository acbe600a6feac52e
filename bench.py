"""Benchmark: decoded Mpixels/s of the post-entropy AV1 reconstruction DSP path,
4K 10-bit 4:2:0 inter frames (BASELINE.json configs[2]: mc + loopfilter + cdef + looprestoration).

One step = one frame through every GPU stage, inputs resident in HBM:
  MC (inter prediction of every block from 2 resident reference pictures) -> itx (residual
  add) -> deblock (A -> D, 64x64 tiles: column edges then row edges) -> CDEF (D -> C) -> loop restoration
  (C + D -> O, the reference picture). Descriptors follow SURVEY.md §8(d) config 3.
Film grain (output-only, configs[3] = 8K10) is timed separately on an 8K10 frame and
reported under "film_grain_8k10"; the intra path (configs[1], 1080p8: intra prediction +
itx residual per block in one persistent launch) under "intra_1080p8". Neither is part of
the headline step.

`python bench.py` runs 1 GPU. Under torch.distributed.run every rank drives its own GPU on
its own independent stream (replicas; no data-path collective; "scaling": "weak"); the
timed region is bracketed by barrier + synchronize and the max over ranks is reported.
Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from rav1d_amd import ITX_DC_DEFER, ITX_KEEP_COEFS  # noqa: E402
from rav1d_amd import frame as F  # noqa: E402
from rav1d_amd.synth import dc_map_bytes, frame_bytes, itx_algorithmic_bytes, itx_band_order, itx_dc_runs, make_frame, mc_algorithmic_bytes, mc_sync_ok  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
W, H, BPC, LAYOUT = 3840, 2160, 10, 1


class Pipeline:
    """Device buffers + descriptors for one stream's frames. `ring` pre-filled copies of the
    coefficient arena: every step reads the next arena, as a decoder uploads a new one per
    frame (the device arena is a staged copy that itx reads once and leaves as it is, so the
    ring is not there for zeroing but so that no step finds its coefficients in a cache)."""

    def __init__(self, ctx, fr, ring=1):
        self.ctx, self.fr = ctx, fr
        w, h, bpc, lay = fr["w"], fr["h"], fr["bpc"], fr["layout"]
        self.A = F.Frame(w, h, bpc, lay)      # prediction -> reconstruction
        self.D = F.Frame(w, h, bpc, lay)      # deblocked (out of place: one fused tile launch)
        self.B = F.Frame(w, h, bpc, lay)      # CDEF output
        self.O = F.Frame(w, h, bpc, lay)      # LR output (the reference frame)
        self.G = F.Frame(w, h, bpc, lay) if fr["fg"] else None   # displayed picture with film grain
        for p, a in enumerate(fr["planes"]):
            self.A.set_plane_np(p, a)
        self.refs, self.mc = [], None
        if fr.get("mc") is not None:
            for planes in fr["refs"]:
                r = F.Frame(w, h, bpc, lay)
                for p, a in enumerate(planes):
                    r.set_plane_np(p, a)
                self.refs.append(r)
            self.mc = F.McMeta(*fr["mc"])
            self.ref_pics = (F.MiPicture * len(self.refs))(*[r.picture() for r in self.refs])
            # one grid, the chroma units of SEG blocks waiting in-launch for their luma mask
            # (mi_mc_frame_sync, as the frame executor runs it when the offsets allow)
            self.mc_sync = mc_sync_ok(fr["mc"][0])
        self.blocks = torch.from_numpy(fr["blocks"].view(np.uint8).copy()).cuda()
        # itx over picture bands, one XCD per band, each band's DC-only blocks first on the DC
        # path (mi_itx_frame_runs, as the frame executor runs it)
        ah = (h + 127) & ~127
        ssv = 1 if lay == 1 else 0
        blk, _, bs = itx_band_order(fr["blocks"], [ah, ah >> ssv, ah >> ssv])
        de = itx_dc_runs(blk, bs)
        self.blocks = torch.from_numpy(blk.view(np.uint8).copy()).cuda()
        self.itx_bands = (ctypes.c_uint32 * bs.size)(*[int(v) for v in bs.reshape(-1)])
        self.itx_dc_end = (ctypes.c_uint32 * de.size)(*[int(v) for v in de.reshape(-1)])
        self.coef = torch.from_numpy(fr["coef"].copy()).cuda()
        self.coef0 = self.coef.clone()               # itx zeroes the arena it consumes
        self.coefs = [self.coef] + [self.coef0.clone() for _ in range(max(1, ring) - 1)]
        self.k = 0
        self.A0 = [t.clone() for t in self.A.planes]
        self.lf = F.LoopFilterMeta(fr["lf"])
        self.cdef = F.CdefMeta(fr["lf"]["masks"], fr["cdef"], masks_dev=self.lf.masks, geometry=(w, h, lay))
        self.lr = F.LrMeta(fr["lr"], geometry=(w, h, lay))
        self.fgd = F.film_grain_data(fr["fg"]) if fr["fg"] else None
        self.side = torch.cuda.Stream()
        fb = frame_bytes(w, h, bpc, lay)
        # algorithmic bytes per launch: read inputs once, write outputs once
        lvl_bytes = ((w + 3) >> 2) * ((h + 3) >> 2) * 4
        mask_bytes = fr["lf"]["masks"].nbytes
        self.algo = {
            # coefficients counted once: the device arena is the frame's staged
            # copy, read once and not zeroed (MI_ITX_KEEP_COEFS, as the frame executor runs it)
            # the DC-only blocks' constant goes through the DC map (MI_ITX_DC_DEFER): itx writes
            # the map, deblock reads it while staging (as the frame executor runs inter frames
            # without intra blocks)
            "itx": itx_algorithmic_bytes(fr["blocks"], bpc, zero_coefs=False, dc_defer=True),
            "deblock": 2 * fb + lvl_bytes + mask_bytes + dc_map_bytes(w, h, lay),
            "cdef": 2 * fb + mask_bytes,
            "lr": 2 * fb + fb * 4 // 64 + fr["lr"]["lr_mask"].nbytes,
            "fg": 2 * fb,
        }
        if self.mc is not None:
            self.algo["mc"] = mc_algorithmic_bytes(fr["mc"][0], bpc) + fr["mc"][2].nbytes
        # kernel launches per stage per frame: mc = one grid (mi_mc_frame_sync), or luma + chroma group
        self.launches = {"mc": 1 if self.mc is not None and self.mc_sync else 2, "itx": 1, "deblock": 1, "cdef": 1,
                         "lr": 1, "fg": 1}
        self.kernels = {"mc": "mc_kernel", "itx": "itx_frame_kernel", "deblock": "lf_tile_kernel",
                        "cdef": "cdef_kernel", "lr": "lr_kernel", "fg": "fg_apply_kernel"}

    def step(self, stream, ev=None, mark=None):
        """Enqueue one frame. ev: optional dict stage -> list of (start, end) events; mark:
        optional event recorded on `stream` once the frame's motion compensation is done."""
        lib = F.lib()
        ctx = self.ctx.h
        sp = F._stream_ptr(stream)
        pa, pb, po, pd = self.A.picture(), self.B.picture(), self.O.picture(), self.D.picture()

        prep_done = None
        if self.fgd is not None:
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

        if self.mc is not None and self.mc_sync:
            timed("mc", lambda: F.check(lib.mi_mc_frame_sync(ctx, ctypes.byref(pa), self.ref_pics, len(self.refs),
                                                             ctypes.c_void_p(self.mc.blocks.data_ptr()), self.mc.class_start,
                                                             ctypes.c_void_p(self.mc.masks.data_ptr()), self.mc.masks.numel(),
                                                             None, sp), "mc"))
        elif self.mc is not None:
            timed("mc", lambda: F.check(lib.mi_mc_frame(ctx, ctypes.byref(pa), self.ref_pics, len(self.refs),
                                                        ctypes.c_void_p(self.mc.blocks.data_ptr()), self.mc.class_start,
                                                        ctypes.c_void_p(self.mc.masks.data_ptr()), None, sp), "mc"))
        if mark is not None:
            mark.record(stream)
        coef = self.coefs[self.k % len(self.coefs)]
        self.k += 1
        timed("itx", lambda: F.check(lib.mi_itx_frame_runs(ctx, ctypes.byref(pa), ctypes.c_void_p(self.blocks.data_ptr()),
                                                           self.itx_bands, self.itx_dc_end, ctypes.c_void_p(coef.data_ptr()),
                                                           ITX_KEEP_COEFS | ITX_DC_DEFER, sp), "itx"))
        timed("deblock", lambda: F.check(lib.mi_deblock_frame_dc(ctx, ctypes.byref(pa), ctypes.byref(pd),
                                                                 ctypes.byref(self.lf.s), sp), "lf"))
        timed("cdef", lambda: F.check(lib.mi_cdef_frame(ctx, ctypes.byref(pd), ctypes.byref(pb),
                                                        ctypes.byref(self.cdef.s), sp), "cdef"))
        timed("lr", lambda: F.check(lib.mi_lr_frame(ctx, ctypes.byref(pb), ctypes.byref(pd), ctypes.byref(po),
                                                    ctypes.byref(self.lr.s), sp), "lr"))
        if self.fgd is not None:
            pg = self.G.picture()
            stream.wait_event(prep_done)
            timed("fg", lambda: F.check(lib.mi_film_grain_apply(ctx, ctypes.byref(po), ctypes.byref(pg),
                                                                ctypes.byref(self.fgd), 0, sp), "fg"))


    def refill(self):
        """Every arena of the ring back to the frame's coefficients (outside timed regions)."""
        for c in self.coefs:
            c.copy_(self.coef0)
        self.k = 0

    def restore(self):
        """Pass-2 inputs back to their initial state (coefficient arenas, prediction picture),
        so that one more step reproduces the oracle's single-pass output."""
        self.refill()
        for t, t0 in zip(self.A.planes, self.A0):
            t.copy_(t0)

    def uploads(self):
        """(device tensor, pinned host copy) of every input a frame's step reads that a decoder
        produces per frame on the host: coefficient arena, transform / MC descriptors, wedge
        masks, deblock levels + masks (CDEF reads the same Av1Filter array), LR units."""
        devs = [self.coefs[0], self.blocks, self.lf.level, self.lf.masks, self.lr.mask]
        if self.mc is not None:
            devs += [self.mc.blocks, self.mc.masks]
        return [(d, self.coef0.cpu().pin_memory() if d is self.coefs[0] else d.cpu().pin_memory()) for d in devs]

    def output_digest(self):
        """sha256 over the visible pixels of the reference picture O (every plane)."""
        import hashlib
        h = hashlib.sha256()
        for p in range(len(self.O.planes)):
            h.update(np.ascontiguousarray(self.O.plane_np(p)).tobytes())
        return h.hexdigest()


def oracle_digest(fr):
    """The same digest over the oracle's output for the same descriptors (CPU restatement)."""
    import hashlib
    from tests.pipeline import oracle_pipeline
    out = oracle_pipeline(fr)["lr"]
    ss_hor, ss_ver = int(fr["layout"] in (1, 2)), int(fr["layout"] == 1)
    h = hashlib.sha256()
    for p, a in enumerate(out):
        w = fr["w"] if p == 0 else (fr["w"] + ss_hor) >> ss_hor
        hh = fr["h"] if p == 0 else (fr["h"] + ss_ver) >> ss_ver
        h.update(np.ascontiguousarray(a[:hh, :w]).tobytes())
    return h.hexdigest()


def broadcast_config(cfg, world):
    """rank 0's run configuration / seed table, broadcast to every rank."""
    if world == 1:
        return cfg
    box = [cfg]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def gather_results(local, world):
    """every rank's {rank, frames, ns, sha256, verified} gathered to all ranks."""
    if world == 1:
        return [local]
    out = [None] * world
    dist.all_gather_object(out, local)
    return out


def film_grain_8k(ctx, stream, reps=20):
    """configs[3]: film grain on an 8K10 frame (prep + apply), HBM-bound stress. Returns
    (Mpixels/s of apply, apply ms, prep ms, apply GB/s algorithmic)."""
    from rav1d_amd.synth import make_fg_params, make_texture
    w, h, bpc = 7680, 4320, 10
    rng = np.random.default_rng(0xF6000001)
    src, dst = F.Frame(w, h, bpc, 1), F.Frame(w, h, bpc, 1)
    for p in range(3):
        pw, ph = src.dims(p)
        src.set_plane_np(p, make_texture(rng, pw, ph, bpc))
    fg = make_fg_params(rng, 1)
    fg["overlap_flag"] = 1
    d = F.film_grain_data(fg)
    lib = F.lib()
    ps, pd = src.picture(), dst.picture()
    sp = F._stream_ptr(stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(3):
        F.check(lib.mi_film_grain_frame(ctx.h, ctypes.byref(ps), ctypes.byref(pd), ctypes.byref(d), 0, sp), "fg")
    torch.cuda.synchronize()
    prep_t, apply_t = 0.0, 0.0
    for _ in range(reps):
        # a short spin kernel first keeps the stream busy while the host enqueues, so the event
        # pairs time the kernels and not the host's launch latency
        with torch.cuda.stream(stream):
            torch.cuda._sleep(200000)
        ev[0].record(stream)
        F.check(lib.mi_film_grain_prep(ctx.h, ctypes.byref(ps), ctypes.byref(d), sp), "fg prep")
        ev[1].record(stream)
        F.check(lib.mi_film_grain_apply(ctx.h, ctypes.byref(ps), ctypes.byref(pd), ctypes.byref(d), 0, sp), "fg apply")
        ev[2].record(stream)
        torch.cuda.synchronize()
        prep_t += ev[0].elapsed_time(ev[1])
        apply_t += ev[1].elapsed_time(ev[2])
    apply_ms, prep_ms = apply_t / reps, prep_t / reps
    fb = frame_bytes(w, h, bpc, 1)
    return dict(mpx_per_s=round(w * h / (apply_ms / 1e3) / 1e6, 1), apply_ms=round(apply_ms, 4),
                prep_ms=round(prep_ms, 4), apply_gbs=round(2 * fb / (apply_ms / 1e3) / 1e9, 1))


def mc_coherent(ctx, stream, reps=20):
    """MC alone on a 4K10 inter frame whose motion is spatially coherent (one motion per 64x64
    superblock and reference + noise of +-2 px per block: rav1d_amd.synth mv_mode "coherent"),
    beside the headline's uniformly random MVs (the worst case for
    reference-window reuse). Same block shapes, filters and compound mix."""
    fr = make_frame(W, H, BPC, LAYOUT, seed=0x4C100001, with_fg=False, with_mc=True, mv_mode="coherent")
    cur = F.Frame(W, H, BPC, LAYOUT)
    refs = []
    for planes in fr["refs"]:
        r = F.Frame(W, H, BPC, LAYOUT)
        for p, a in enumerate(planes):
            r.set_plane_np(p, a)
        refs.append(r)
    meta = F.McMeta(*fr["mc"])
    lib, pc = F.lib(), cur.picture()
    pics = (F.MiPicture * len(refs))(*[r.picture() for r in refs])
    blocks, masks, sp = ctypes.c_void_p(meta.blocks.data_ptr()), ctypes.c_void_p(meta.masks.data_ptr()), F._stream_ptr(stream)
    fn = lambda: F.check(lib.mi_mc_frame(ctx.h, ctypes.byref(pc), pics, len(refs), blocks, meta.class_start,
                                         masks, None, sp), "mc")
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    algo = mc_algorithmic_bytes(fr["mc"][0], BPC) + fr["mc"][2].nbytes
    gbs = algo / (ms / 1e3) / 1e9
    return dict(ms=round(ms, 4), algo_bytes=int(algo), gbs=round(gbs, 1), frac=round(gbs / HBM_PEAK_GBS, 4),
                traffic_per_step=pmc_traffic("mc", "r03_traffic_coherent.json"),
                mv_field="coherent: per-64x64 motion per reference uniform in +-64 px, +-2 px noise per block")


def output_4k10(ctx, stream, reps=10):
    """The output side at 4K10 (include/mi_av1out.h): the displayed picture written into pinned
    host memory by mi_output_picture, as a DMA copy of the visible area and with film grain
    stored by the grain kernel straight into host memory (one pass). PCIe-bound: this is the
    host-buffer rate DESIGN.md §5 quotes, never the headline value."""
    from rav1d_amd.output import HostPicture, output_picture
    from rav1d_amd.synth import make_fg_params, make_texture
    rng = np.random.default_rng(0x0F7E0001)
    src = F.Frame(W, H, BPC, LAYOUT)
    for p in range(3):
        pw, ph = src.dims(p)
        src.set_plane_np(p, make_texture(rng, pw, ph, BPC))
    host = HostPicture(W, H, BPC, LAYOUT)
    fg = F.film_grain_data(make_fg_params(rng, LAYOUT))
    fb = frame_bytes(W, H, BPC, LAYOUT)
    res = {}
    for name, g in (("copy", None), ("grain_fused", fg)):
        fn = lambda: output_picture(ctx, src, host, g, 0, stream)
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        res[name] = dict(ms=round(ms, 3), fps=round(1e3 / ms, 1), host_gbs=round(fb / (ms / 1e3) / 1e9, 1))
    host.free()
    return res


def end_to_end_4k10(fr, want=None, steps=20):
    """SURVEY.md 8(d)'s end-to-end figure for the headline frame, "from first upload to last
    output-ready event": per frame, the inputs a decoder produces on the host (coefficient arena
    and descriptors, in pinned memory) uploaded, the five device stages, and the displayed
    picture copied into pinned host memory (mi_output_picture). One lane (one stream), and two
    lanes (two frames in flight on two streams / contexts: one frame's copies overlap the other's
    kernels; the DMA engines and PCIe are full duplex). PCIe-inclusive: never the headline.
    want: the oracle's digest of the frame; the last frame's host picture is checked against it."""
    import hashlib

    from rav1d_amd.output import HostPicture, output_picture
    lanes = []
    for _ in range(2):
        c = F.Context(torch.cuda.current_device())
        pk = Pipeline(c, fr)
        lanes.append((c, pk, torch.cuda.Stream(), pk.uploads(), [HostPicture(W, H, BPC, LAYOUT) for _ in range(2)]))
    up_bytes = sum(d.numel() * d.element_size() for d, _ in lanes[0][3])
    out_bytes = frame_bytes(W, H, BPC, LAYOUT)

    def frame(lane, i, ev=None):
        c, pk, st, ups, hosts = lane
        with torch.cuda.stream(st):
            if ev:
                ev[0].record(st)
            for d, h in ups:
                d.copy_(h, non_blocking=True)
            if ev:
                ev[1].record(st)
            pk.step(st)
            if ev:
                ev[2].record(st)
            output_picture(c, pk.O, hosts[i % 2], None, 0, st)
            if ev:
                ev[3].record(st)

    for i in range(4):
        frame(lanes[i % 2], i)
    torch.cuda.synchronize()
    # stage breakdown (HIP events on the lane's stream)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(5)]
    for i, e in enumerate(evs):
        frame(lanes[0], i, e)
    torch.cuda.synchronize()
    parts = [float(np.mean([e[k].elapsed_time(e[k + 1]) for e in evs])) for k in range(3)]
    res = {}
    for name, nl in (("one_lane", 1), ("two_lanes", 2)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            frame(lanes[i % nl], i // nl)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        res[name] = dict(ms_per_frame=round(dt * 1e3, 4), fps=round(1 / dt, 1), mpx_per_s=round(W * H / dt / 1e6, 1))
    # the last one-lane frame's displayed picture (host memory) against the oracle
    verified = None
    if want is not None:
        for lane in lanes:
            lane[1].refill()
        torch.cuda.synchronize()             # refill copies on the current stream, the frame on the lane's
        frame(lanes[0], 0)
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for p in range(3):
            h.update(np.ascontiguousarray(lanes[0][4][0].plane_np(p)).tobytes())
        verified = h.hexdigest() == want
    for lane in lanes:
        for hp in lane[4]:
            hp.free()
    return dict(res, upload_ms=round(parts[0], 4), device_ms=round(parts[1], 4), d2h_ms=round(parts[2], 4),
                upload_bytes=int(up_bytes), d2h_bytes=int(out_bytes),
                upload_gbs=round(up_bytes / (parts[0] / 1e3) / 1e9, 1), d2h_gbs=round(out_bytes / (parts[2] / 1e3) / 1e9, 1),
                verified=verified, steps=steps,
                what="per frame: H2D of coefficient arena + descriptors from pinned host memory, mc + itx + deblock "
                     "+ cdef + lr, D2H of the displayed picture into pinned host memory (mi_output_picture)")


# SURVEY.md 8(d) / BASELINE configs on the reference's own streams (tests/golden/streams; MD5s
# from its meson files): intra 1080p8 / 352x288 / 4K10, and its largest inter vectors
REAL_STREAMS = ["itut_t35", "av1-1-b8-02-allintra", "itut_t35_10bit", "issue_318", "00001141", "issue_295"]


def real_streams(ctx, reps=3, oracle_reps=5, oracle_budget_s=25.0):
    """The reference's streams end to end: host front-end (libmi_av1dec.so) -> device
    reconstruction + in-loop filters (mi_frame_run) -> mi_output_picture into pinned host memory
    -> muxer. As the reference's own benchmark runs (tools/dav1d.rs with --muxer null), the timed
    passes use the null muxer; the MD5 is verified in a separate pass through the product md5
    muxer. Per stream:
      gpu_ms             pipelined decode (front-end threads ahead, muxer one picture behind), best of `reps`
      gpu_unpipelined_ms one frame at a time, mi_frame_end after each
      stages_ms          one unpipelined pass broken down: front-end (host, waiting for events; each
                         frame's tiles on 8 threads, no temporal unit ahead),
                         mi_frame_run host time, upload / inter / intra / filter device time
                         (mi_ctx_timing), output copy (events), muxer (host)
      stages_pipelined_ms the same for one pipelined pass (front-end frame threads running ahead)
      front_end_only_ms  the front-end alone (single thread); front_end_8_threads_ms: 8 threads
      cpu_oracle_ms      front-end + the CPU restatement (oracle/, single thread, no hashing), best
                         of up to `oracle_reps` within `oracle_budget_s` (kind "port": rav1d's own
                         CLI cannot be built here)"""
    from rav1d_amd.av1dec import Av1Decoder, stream_events, stream_units
    from rav1d_amd.output import Muxer
    from rav1d_amd.stream import decode_to_muxer
    from tests.stream_lib import decode_stream
    gold = os.path.join(ROOT, "tests", "golden", "streams")
    vecs = {v["name"]: v for v in json.load(open(os.path.join(gold, "vectors.json")))}
    out = {}
    for name in REAL_STREAMS:
        v = vecs[name]
        data = open(os.path.join(gold, v["file"]), "rb").read()
        grain = bool(v.get("filmgrain"))
        m = Muxer("md5")
        n = decode_to_muxer(ctx, data, m, apply_grain=grain)
        ok = m.verify(v["md5"]) == 0
        m.close()

        def best_of(k, **kw):
            b = 1e9
            for _ in range(k):
                mm = Muxer("null")
                t0 = time.perf_counter()
                decode_to_muxer(ctx, data, mm, apply_grain=grain, **kw)
                b = min(b, time.perf_counter() - t0)
                mm.close()
            return b
        best = best_of(reps)
        best_seq = best_of(reps, pipelined=False)
        st = {}
        mm = Muxer("null")
        decode_to_muxer(ctx, data, mm, apply_grain=grain, pipelined=False, stats=st)
        mm.close()
        # the same breakdown of one pipelined pass: the front-end's frame and tile threads run
        # ahead of the device (frame k+1's entropy decoding while frame k is reconstructed), so
        # front_end_ms is what the host still waits for events
        stp = {}
        mm = Muxer("null")
        decode_to_muxer(ctx, data, mm, apply_grain=grain, stats=stp)
        mm.close()
        # the front-end alone (one thread, and 8 threads: frame jobs + tile decoders, temporal
        # units ahead as the pipelined decode runs it); shown-picture pixels for the Mpixels/s figures
        fe_mt = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            for _ev in stream_events(data, 8):
                pass
            fe_mt = min(fe_mt, time.perf_counter() - t0)
        fe, px, bits, size = 1e9, 0, 8, None
        for _ in range(reps):
            t0 = time.perf_counter()
            dec = Av1Decoder()
            dims, px = {}, 0
            for tu in stream_units(data):
                dec.send(tu)
                for ev in dec.events():
                    if ev.frame:
                        f = ev.frame.contents
                        dims[ev.pic_id] = (f.up_w, f.h)
                        bits, size = f.bpc, (f.up_w, f.h)
                    if ev.show_pic >= 0:
                        px += dims[ev.show_pic][0] * dims[ev.show_pic][1]
            fe = min(fe, time.perf_counter() - t0)
        cpu, creps, spent = 1e9, 0, 0.0
        while creps < oracle_reps and (creps == 0 or spent + cpu <= oracle_budget_s):
            t0 = time.perf_counter()
            decode_stream(data, hash_output=False)
            dt = time.perf_counter() - t0
            cpu, spent, creps = min(cpu, dt), spent + dt, creps + 1
        out[name] = dict(
            frames=n, size=f"{size[0]}x{size[1]} {bits}-bit", md5_verified=ok, muxer="null (md5 verified in a separate pass)",
            gpu_ms=round(best * 1e3, 3), gpu_fps=round(n / best, 1), gpu_mpx_per_s=round(px / best / 1e6, 2),
            gpu_unpipelined_ms=round(best_seq * 1e3, 3),
            stages_ms={k: round(st[k], 3) for k in ("front_end_ms", "run_host_ms", "run_levels_ms", "run_stage_ms",
                                                     "upload_ms", "inter_ms", "intra_ms", "filter_ms", "d2h_ms",
                                                     "mux_ms")},
            stages_pipelined_ms={k: round(stp[k], 3) for k in ("front_end_ms", "run_host_ms", "upload_ms", "inter_ms",
                                                                "intra_ms", "filter_ms", "d2h_ms", "mux_ms")},
            upload_mb=round(st["upload_bytes"] / 1e6, 2),
            front_end_only_ms=round(fe * 1e3, 3), front_end_8_threads_ms=round(fe_mt * 1e3, 3),
            cpu_oracle_ms=round(cpu * 1e3, 1), cpu_oracle_reps=creps, cpu_oracle_mpx_per_s=round(px / cpu / 1e6, 2))
    return out


def per_launch(v, launches):
    return None if v is None else int(v // launches)


def pmc_traffic(stage, name=None):
    """HBM bytes per step of `stage` from the committed PMC run (profiles/r06_traffic.json,
    written by tools/traffic_json.py from tools/gpu_pmc.sh's FETCH_SIZE / WRITE_SIZE passes of
    this same bench command, calibrated per access width by tools/pmc_calib; the round-1 file
    when this round's is absent). None if absent."""
    path = None
    for n in ([name] if name else ["r06_traffic.json", "r05_traffic.json", "r04_traffic.json", "r03_traffic.json", "r02_traffic.json",
                                   "r01_traffic.json"]):
        if os.path.exists(os.path.join(ROOT, "profiles", n)):
            path = os.path.join(ROOT, "profiles", n)
            break
    if path is None:
        return None
    ent = json.load(open(path)).get("stages", {}).get(stage)
    return None if ent is None else ent.get("hbm_bytes_per_step")


def intra_1080p8(ctx, reps=5, nframes=24, ndesc=4):
    """configs[1]: 1080p 8-bit 4:2:0 intra frames, intra prediction (device edge gathering) +
    itx residual per transform block, reconstructed by the persistent fused kernel
    (mi_intra_recon: one launch, per-block dependency waits, frame f on XCD f % 8). Reports the
    single-frame latency, the throughput of `nframes` independent frames per launch (an
    all-intra stream's frames do not depend on each other; ndesc distinct synthetic descriptor
    sets, cycled, each frame its own picture) and, for comparison, the per-level launch path
    (two launches per dependency level, graph-replayed)."""
    from rav1d_amd.intra import IntraFrame, device_status, intra_recon, make_intra_residuals
    from rav1d_amd.ipred_synth import make_intra_frame
    w, h, bpc = 1920, 1080, 8
    frs = []
    for k in range(ndesc):
        rng = np.random.default_rng(0x1A7A0001 + k)
        frs.append(make_intra_residuals(make_intra_frame(w, h, bpc, 1, rng), bpc, rng))
    # one descriptor set (and coefficient arena: itxfm_add zeroes what it consumes) per frame
    descs = [IntraFrame(ctx, frs[f % ndesc]) for f in range(nframes)]
    curs = [F.Frame(w, h, bpc, 1) for _ in range(nframes)]
    batch = [(descs[f], curs[f].picture()) for f in range(nframes)]
    s = torch.cuda.Stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(fn):
        fn()
        s.synchronize()
        ev[0].record(s)
        for _ in range(reps):
            fn()
        ev[1].record(s)
        s.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps

    with torch.cuda.stream(s):
        # edge granules (MI_IR_EDGE_GRANULES: the frames are intra-only) and done flags
        one_ms = timed(lambda: intra_recon(ctx, batch[:1], s, keep_coefs=False, granules=True))
        batch_ms = timed(lambda: intra_recon(ctx, batch, s, keep_coefs=False, granules=True))
        one_flags_ms = timed(lambda: intra_recon(ctx, batch[:1], s, keep_coefs=False))
        batch_flags_ms = timed(lambda: intra_recon(ctx, batch, s, keep_coefs=False))
        device_status(ctx, s)
        intra, pic = descs[0], batch[0][1]
        g = torch.cuda.CUDAGraph()
        intra.step(pic, s, keep_coefs=False)
        with torch.cuda.graph(g, stream=s):
            intra.step(pic, s, keep_coefs=False)
        level_ms = timed(g.replay)
    fr = descs[0].fr
    return dict(mpx_per_s=round(nframes * w * h / (batch_ms / 1e3) / 1e6, 1),
                fps=round(nframes / (batch_ms / 1e3), 1), ms_per_frame=round(one_ms, 3),
                frames_per_launch=nframes, batch_ms=round(batch_ms, 3),
                single_frame_mpx_per_s=round(w * h / (one_ms / 1e3) / 1e6, 1),
                ms_per_frame_flags=round(one_flags_ms, 3), batch_ms_flags=round(batch_flags_ms, 3),
                level_launch_ms=round(level_ms, 3), levels=len(intra.levels), tx_blocks=int(len(fr["blocks"])),
                kernel="intra_recon_kernel (persistent, one-wave workers, 3 frames per XCD, edge granules)")


def host_cpu():
    """lscpu model / sockets / cores of the host the baseline runs on."""
    info = {}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "CPU(s)", "Thread(s) per core"):
                info[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def cpu_share():
    """The job's CPU share: cgroup cpu.max (v2) or cfs quota / period (v1) as a CPU count, the
    affinity mask's size, and OMP_NUM_THREADS as the box exports it."""
    info = {"affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_max"] = f"{q} {per}"
        info["cgroup_cpus"] = None if q in ("max", "-1") else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            info["cgroup_cpu_max"] = f"{q} {per}"
            info["cgroup_cpus"] = None if q < 0 else round(q / per, 2)
        except (OSError, ValueError):
            info["cgroup_cpu_max"] = None
    return info


def cpu_baseline(fr, reps=5):
    """The oracle (the C restatement in oracle/, driven from C by oracle/cpu_bench.c: no Python
    in the timed loop) on a bounded sample of the same workload: whole 4K10 inter frames through
    MC + itx + deblock + CDEF + LR. Single thread, and N threads each decoding its own frame
    (independent streams, as the GPU replicas); best of `reps`. Luma Mpixels/s."""
    from tests.pipeline import oracle_bench
    # the box exports OMP_NUM_THREADS as this job's CPU share; nproc counts the whole machine
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    res, t_total = {}, 0.0
    for th in sorted({1, n}):
        best = None
        for _ in range(reps):
            t = oracle_bench(fr, th, 1)
            t_total += t
            best = t if best is None else min(best, t)
        res[th] = th * fr["w"] * fr["h"] / best / 1e6
    return dict(value=round(res[n], 3), unit="Mpixels/s", cores=n, kind="port",
                threads={str(k): round(v, 3) for k, v in res.items()}, host=host_cpu(), cpu_share=cpu_share(),
                sample=f"1 whole synthetic 4K10 inter frame per thread (the bench's own descriptors) through "
                       f"oracle/ (mc+itx+deblock+cdef+lr) from C, best of {reps}, at 1 and {n} threads "
                       f"(independent frames per thread); {t_total:.1f}s of CPU-timed work")


def timed_region(step, steps, sync, world, device):
    """The timed region of the bench contract: barrier + sync, exactly `steps` steps, sync +
    barrier, then the MAX of the per-rank wall times over all ranks (world > 1: an initialised
    process group; `device` holds the reduction tensor: "cuda" under RCCL, "cpu" under gloo)."""
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def single_stream(args, world, rank, local):
    """One stream, frame-pipelined over the ranks: every rank builds the same
    synthetic GOP (descriptor sets shared by reference count), prepares its own frames, and the
    timed region decodes the whole stream `steps` times; value = frames decoded / wall time."""
    from rav1d_amd.sstream import DeviceExecutor, PipelinedStream, make_stream_specs
    specs = make_stream_specs(W, H, BPC, LAYOUT, args.single_stream, 0x55400001, reuse=True)
    ctx = F.Context(local)
    ex = DeviceExecutor(ctx, bands=args.bands)
    for s in specs:
        if s.idx % world == rank:
            ex.prepare(s)
    ps = PipelinedStream(ex, ex.alloc, rank, world, "cuda", bands=args.bands)
    for _ in range(max(1, args.warmup)):
        ps.run(specs)
    torch.cuda.synchronize()
    elapsed = timed_region(lambda: ps.run(specs), args.steps, torch.cuda.synchronize, world, "cuda")
    frames = args.steps * len(specs)
    if rank == 0:
        print(json.dumps({
            "metric": "decoded Mpixels/s (one 4K 10-bit 4:2:0 stream, frames pipelined over the GPUs)",
            "value": round(frames * W * H / elapsed / 1e6, 2), "unit": "Mpixels/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "fps": round(frames / elapsed, 2), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u16", "data": "synthetic hierarchical GOP (rav1d_amd.sstream)",
            "config": {"workload": f"one 4K10 stream of {len(specs)} frames per step, frame k on rank k % N, "
                                   f"references sent point to point"
                                   + (f" in {args.bands} bands, MC per band (row-level progress)" if args.bands > 1 else ""),
                       "parallelism": f"frame-pipelined x{world}"}}))
    if world > 1:
        dist.destroy_process_group()


class CudaHw:
    """The device side of the replica path: one HIP device per rank, RCCL ("nccl") for the
    control collectives. tests/test_bench_dist.py swaps in a CPU stand-in with the same
    methods to run main()'s replica path end to end over gloo."""
    device, backend = "cuda", "nccl"

    def setup(self, local):
        torch.cuda.set_device(local)

    def pg_kwargs(self, local):
        return {"device_id": torch.device("cuda", local)}

    def context(self, local):
        return F.Context(local)

    def pipeline(self, ctx, fr, ring):
        return Pipeline(ctx, fr, ring=ring)

    def sync(self):
        torch.cuda.synchronize()

    def stream(self, new=False):
        return torch.cuda.Stream() if new else torch.cuda.current_stream()

    def oracle_digest(self, fr):
        return oracle_digest(fr)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`--gpus N` (N > 1) without a launcher: start N ranks as fresh child processes, one per
    GPU, with the environment torch.distributed.run would give them (rendezvous on 127.0.0.1).
    This process never touches the GPU (only children initialise HIP), and it exits with the
    first non-zero exit code of its ranks. Rank 0 prints the JSON line."""
    import signal
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    codes = [None] * n
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        if any(c not in (None, 0) for c in codes):
            # one rank failed: the others would wait for it in a collective
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.send_signal(signal.SIGTERM)
            for i, p in enumerate(procs):
                if codes[i] is None:
                    try:
                        codes[i] = p.wait(30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [c for c in codes if c]
    return bad[0] if bad else 0


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks) of this node. Under torch.distributed.run it must equal WORLD_SIZE; "
                         "without a launcher, N > 1 starts N rank processes itself")
    ap.add_argument("--frame", default=f"{W}x{H}", help=argparse.SUPPRESS)   # tests: a small frame
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fg", action="store_true", help="skip the separate 8K10 film-grain measurement")
    ap.add_argument("--no-intra", action="store_true", help="skip the separate 1080p8 intra measurement")
    ap.add_argument("--no-verify", action="store_true", help="skip the per-rank oracle check of the output")
    ap.add_argument("--no-extra", action="store_true", help="skip the coherent-motion MC and output-side measurements")
    ap.add_argument("--bands", type=int, default=1,
                    help="--single-stream: references sent in this many row bands, MC launched per band")
    ap.add_argument("--single-stream", type=int, default=0, metavar="FRAMES",
                    help="instead of replicas: one 4K10 stream of FRAMES frames (hierarchical GOP of 8), frame k "
                         "reconstructed on rank k %% N, references exchanged point to point (rav1d_amd.sstream)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="frames reconstructed concurrently per GPU, each on its own HIP stream and context "
                         "(rav1d's frame threads, n_fc): a step is then that many frames")
    ap.add_argument("--graph", type=int, default=0, help="1: replay the step as one captured HIP graph")
    ap.add_argument("--two-in-flight", action=argparse.BooleanOptionalAction, default=True,
                    help="also time two independent frames per step on two streams (two_frames_in_flight; "
                         "reported beside the headline, never as `value`)")
    ap.add_argument("--stagger", type=int, default=0, help="with --inflight > 1: frame k's MC waits for frame k-1's")
    ap.add_argument("--dense-coefs", action="store_true",
                    help="the coefficient arena dense (min(w,32) x min(h,32) per non-DC block) instead of "
                         "the front-end's packed corners (MI_TX_PACKED)")
    ap.add_argument("--mv", choices=["uniform", "coherent"], default="uniform",
                    help="motion field of the timed frame (uniform: SURVEY.md 8(d) config 3)")
    return ap.parse_args(argv)


def main(argv=None, hw=None):
    """Returns the process exit code. hw: the device side (CudaHw unless a test injects one)."""
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus, argv)
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    hw = hw or CudaHw()
    hw.setup(local)
    if world > 1:
        dist.init_process_group(hw.backend, **hw.pg_kwargs(local))

    if args.single_stream:
        single_stream(args, world, rank, local)
        return 0
    replicas(args, world, rank, local, hw)
    if world > 1:
        dist.destroy_process_group()
    return 0


def replicas(args, world, rank, local, hw):
    """The headline: every rank decodes its own independent stream (seed + rank) on its own
    GPU; no data-path collective."""
    fw, fh = (int(v) for v in args.frame.split("x"))
    stream = hw.stream()
    cfg = broadcast_config({"w": fw, "h": fh, "bpc": BPC, "layout": LAYOUT,
                            "seeds": [0x4C100001 + r for r in range(world)]}, world)
    fr = make_frame(cfg["w"], cfg["h"], cfg["bpc"], cfg["layout"], seed=cfg["seeds"][rank], with_fg=False,
                    with_mc=True, mv_mode=args.mv, packed=not args.dense_coefs)
    ctx = hw.context(local)
    # one pre-filled coefficient arena per timed step (each step reads a fresh one)
    ring = min(max(args.steps, 1), 512)
    pipe = hw.pipeline(ctx, fr, ring)
    hw.sync()

    for _ in range(args.warmup):
        pipe.step(stream)
    hw.sync()
    pipe.refill()

    # per-kernel timing pass (HIP events on the launch stream), then the clean timed pass
    ev = {}
    for _ in range(max(5, args.steps // 5)):
        pipe.step(stream, ev)
    hw.sync()
    pipe.refill()
    hw.sync()
    stage_ms = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in ev.items()}

    # frames in flight: independent frames on their own streams (and contexts: a context's
    # scratch belongs to one stream), the first on the default stream. The headline runs
    # --inflight frames per step (default 1: every launch has the GPU to itself, so the event
    # durations above are the kernels' own); with --two-in-flight, two frames in flight (rav1d's
    # frame threads) are measured beside it (not in the default run: its concurrent launches
    # would mix into a profiler's per-kernel averages of this command).
    n_pipes = max(args.inflight, 2 if args.two_in_flight else 1)
    pipes = [(pipe, stream)]
    for _ in range(n_pipes - 1):
        pk = hw.pipeline(hw.context(local), fr, ring)
        pipes.append((pk, hw.stream(new=True)))
    for pk, sk in pipes[1:]:
        for _ in range(args.warmup):
            pk.step(sk)
        hw.sync()
        pk.refill()
    hw.sync()
    marks = [torch.cuda.Event() for _ in pipes] if args.stagger else [None] * len(pipes)

    def step_k(k):
        def run():
            # staggered: frame i starts its motion compensation once frame i-1's is done
            for i, (pk, sk) in enumerate(pipes[:k]):
                if args.stagger and i:
                    sk.wait_event(marks[i - 1])
                pk.step(sk, mark=marks[i] if args.stagger else None)
        return run
    step_fn = step_k(args.inflight)
    if args.graph:
        # the step's launches captured into HIP graphs (the C-ABI calls only enqueue kernels on
        # the stream they are given), one graph per arena of the coefficient ring, replayed in
        # ring order: every step still reads a fresh arena
        cap = torch.cuda.Stream()
        cap.wait_stream(stream)
        graphs = []
        for _ in range(len(pipe.coefs)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                for pk, _ in pipes[:args.inflight]:
                    pk.step(cap)
            graphs.append(g)
        hw.sync()
        gi = [0]

        def step_fn():
            graphs[gi[0] % len(graphs)].replay()
            gi[0] += 1
        for _ in range(args.warmup):
            step_fn()
        hw.sync()
    elapsed = timed_region(step_fn, args.steps, hw.sync, world, hw.device)
    # the picture the last timed step left (every timed step consumed a fresh arena, so it is
    # the frame the oracle computes); checked below with the rank's oracle digest
    timed_digest = pipe.output_digest()
    want = hw.oracle_digest(fr) if not args.no_verify else None
    elapsed2, concurrent_ok = None, None
    if args.inflight == 1 and n_pipes >= 2:
        for pk, _ in pipes[:2]:
            pk.refill()
        hw.sync()
        elapsed2 = timed_region(step_k(2), args.steps, hw.sync, world, hw.device)
        conc = [pk.output_digest() for pk, _ in pipes[:2]]
        concurrent_ok = conc[0] == conc[1] == (want or timed_digest)

    # per-rank correctness: the last timed frame, and one more step from the initial inputs,
    # against the oracle on this rank's host cores (outside the timed region)
    pipe.restore()
    hw.sync()
    pipe.step(stream)
    hw.sync()
    digest = pipe.output_digest()
    verified = (digest == want and (args.graph or timed_digest == want)) if want is not None else None
    # the other in-flight frames (own buffers, streams and contexts) produce the same picture
    for pk, sk in pipes[1:]:
        # restore's copies run on the current stream, the step on the frame's own: order them
        pk.restore()
        hw.sync()
        pk.step(sk)
        hw.sync()
        if verified is not None:
            verified = verified and pk.output_digest() == digest
    ranks = gather_results({"rank": rank, "frames": args.steps * args.inflight, "ns": int(elapsed * 1e9),
                            "sha256": digest, "verified": verified}, world)

    dom = max(stage_ms, key=stage_ms.get)
    achieved = pipe.algo[dom] / (stage_ms[dom] / 1e3) / 1e9
    frames = args.steps * world * args.inflight
    value = frames * fw * fh / elapsed / 1e6
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
            "frames_in_flight": args.inflight,
            "two_frames_in_flight": None if elapsed2 is None else {
                "value": round(2 * args.steps * world * fw * fh / elapsed2 / 1e6, 2),
                "ms_per_step": round(elapsed2 / args.steps * 1e3, 4),
                "outputs_match_sequential": concurrent_ok,
                "note": "two independent frames per step on two HIP streams / contexts (frame threading); "
                        "the pictures of the concurrent steps compared with a step run alone"},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (seeded inter-frame descriptors per SURVEY.md §8d config 3: uniformly random MVs, the "
                    "worst case for reference reuse); the reference's real 4K / 1080p inter and intra streams are "
                    "under real_streams",
            "frame": f"{fw}x{fh}",
            "headline": "kernel-only: every input resident in HBM, one fresh coefficient arena per step; the "
                        "PCIe-inclusive figure (upload + kernels + output copy) is end_to_end_4k10",
            "arena_ring": ring,
            "config": {"workload": f"4K10 4:2:0 {fw}x{fh} inter frame: mc (2 refs, 30% compound) + itx residual "
                                   f"+ deblock + cdef + lr",
                       "parallelism": f"replicas{world} (one independent stream per GPU)"},
            "verified": all(r["verified"] for r in ranks) if not args.no_verify else None,
            "per_rank": ranks,
            "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
            "stage_gbs": {k: round(pipe.algo[k] / (stage_ms[k] / 1e3) / 1e9, 1) for k in stage_ms if k in pipe.algo},
            # per launch: algorithmic bytes / mean launch duration (the stage's events span its
            # launches_per_step launches); traffic = PMC HBM bytes per launch (r01_traffic.json)
            "roofline": {"kernel": pipe.kernels[dom], "stage": dom, "bound": "hbm",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": per_launch(pmc_traffic(dom), pipe.launches[dom]),
                         "algo_bytes_per_launch": pipe.algo[dom] // pipe.launches[dom],
                         "launch_us": round(stage_ms[dom] * 1e3 / pipe.launches[dom], 2),
                         "launches_per_step": pipe.launches[dom]},
            # the same figures for every stage's kernel (north_star sets >= 0.5 on itx and deblock)
            "stage_roofline": {k: {"kernel": pipe.kernels[k], "achieved": round(pipe.algo[k] / (stage_ms[k] / 1e3) / 1e9, 1),
                                   "frac": round(pipe.algo[k] / (stage_ms[k] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "traffic": per_launch(pmc_traffic(k), pipe.launches[k]),
                                   "algo_bytes_per_launch": pipe.algo[k] // pipe.launches[k],
                                   "launch_us": round(stage_ms[k] * 1e3 / pipe.launches[k], 2)}
                               for k in stage_ms if k in pipe.algo},
            "mv_field": args.mv,
        }
        if world == 1 and not args.no_fg:
            out["film_grain_8k10"] = film_grain_8k(ctx, stream)
        if world == 1 and not args.no_intra:
            out["intra_1080p8"] = intra_1080p8(ctx)
        if world == 1 and not args.no_extra:
            out["end_to_end_4k10"] = end_to_end_4k10(fr, want)
            out["mc_coherent_4k10"] = mc_coherent(ctx, stream)
            out["output_4k10"] = output_4k10(ctx, stream)
            out["real_streams"] = real_streams(ctx)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(fr)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    sys.exit(main())
