"""Single-stream multi-GPU decode: frame pipelining with reference exchange.

rav1d decodes one stream with frame threads (src/thread_task.rs:301-575): frame k's
reconstruction waits until the reference frames it reads have progressed far enough, and
frames whose references are ready run concurrently. Here every GPU is one frame context: frame
k (decode order) runs on rank k % N, and a reference picture produced on another rank arrives
by a point-to-point transfer — RCCL send/recv over xGMI under the "nccl" backend (device
tensors, no host staging), host-staged under "gloo". Dependencies are whole frames (a frame
starts once its references are complete), which is rav1d's frame-threading model without
row-level progress.

Row-level progress (bands > 1), after rav1d's per-sbrow reference waits
(src/thread_task.rs:450-575, recon.rs's `wait_for_ref` before each superblock row's MC): a
reference picture travels in `bands` horizontal bands, top first, and a consumer runs its MC
in the same bands: the units of band group g (mc_band_groups: every reference row a unit's
8-tap window reads lies in bands 0..g) are launched once bands 0..g of every remote reference
have arrived, so the transfer of the lower bands overlaps the MC of the upper ones. The
residual and the loop filters follow the last band, as in rav1d, where the filters of a row
need the rows below it.

Transfer protocol, deadlock-free by construction:
  * the producer of frame r posts a non-blocking send of r's output picture to every rank that
    owns a later frame referencing r, as soon as r is reconstructed (sends never block the
    producer);
  * a consumer receives the pictures coming from one peer strictly in increasing r (the order
    the peer sends them), buffering any it does not need yet, so the per-pair message order
    always matches;
  * the two directions of a pair travel on two communicators (one process group carries every
    lower -> higher rank message, another every higher -> lower one). RCCL / NCCL put a
    pair's unbatched sends and receives of one communicator on one stream, where A's send to
    B queued before A's receive from B, and B's send to A before B's receive from A, would
    wait on each other for large pictures; with one communicator per direction a send never
    sits in front of the receive its peer's send needs.
The "nccl" (RCCL over xGMI) path is experimental: the tests exercise this scheduler over gloo
(tests/test_sstream_dist.py) and on one GPU; the round-end driver owns the 8-GPU node.
The per-frame work is an `executor(spec, ref_pictures) -> picture` callable: the device
executor below runs the batched C-ABI kernels (mi_mc_frame -> mi_itx_frame ->
mi_deblock_frame_to -> mi_cdef_frame -> mi_lr_frame); tests drive the same scheduler with
other executors.
"""
import hashlib
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class FrameSpec:
    """One frame of the stream in decode order: indices of the (earlier) frames it references,
    whether it is shown, and the descriptors its executor needs."""
    idx: int
    refs: list
    shown: bool = True
    desc: dict = field(default=None, repr=False)


def owner(idx, world):
    return idx % world


def transfer_plan(specs, world):
    """r -> sorted ranks (other than r's owner) that own a frame referencing r."""
    plan = {}
    for s in specs:
        for r in s.refs:
            q = owner(s.idx, world)
            if q != owner(r, world):
                plan.setdefault(r, set()).add(q)
    return {r: sorted(v) for r, v in plan.items()}


def last_use(specs):
    """r -> decode index of the last frame referencing r (pictures are freed after it)."""
    lu = {}
    for s in specs:
        for r in s.refs:
            lu[r] = max(lu.get(r, -1), s.idx)
    return lu


def gop_specs(n, gop=8):
    """Decode order and references of a hierarchical (random-access) GOP structure, the
    shape libaom / rav1e use: per group of `gop`, the key/anchor first, then the pyramid
    middle-out; every frame references the nearest decoded frames before and after it in
    display order. Returns [(display_index, [ref decode indices])] in decode order."""
    order, refs_disp = [0], {0: []}
    start = 0
    while start + 1 < n:
        end = min(start + gop, n - 1)
        order.append(end)
        refs_disp[end] = [start]

        def split(lo, hi):
            if hi - lo < 2:
                return
            mid = (lo + hi) // 2
            order.append(mid)
            refs_disp[mid] = [lo, hi]
            split(lo, mid)
            split(mid, hi)
        split(start, end)
        start = end
    dec_of = {d: i for i, d in enumerate(order)}
    return [(d, [dec_of[r] for r in refs_disp[d]]) for d in order]


def band_height(h, bands):
    """Luma rows per band: h split into `bands` bands of a multiple of 8 rows (the last may be
    shorter)."""
    return max(8, ((h + bands - 1) // bands + 7) // 8 * 8)


def band_rows(b, bh, h, ss_v):
    """Rows [lo, hi) of band b in a plane subsampled by ss_v (luma band height bh)."""
    lo, hi = (b * bh) >> ss_v, (min(h, (b + 1) * bh) + ss_v) >> ss_v
    return lo, hi


def mc_band_groups(units, h, layout, bands):
    """Band group of every MC unit (MiMcBlock records): the smallest g such that every
    reference row the unit's 8-tap window can read (rows up to y + h + mv_y / 8 + 4, in the
    unit's plane, per reference) lies in luma bands 0..g. A unit reading beyond the frame's
    last row (the border replicate of emu_edge) needs the last band. A chroma MASK unit reads
    the mask the luma unit of its block writes (a SEG block's chroma), so it joins the luma
    unit's group when that is later."""
    bh = band_height(h, bands)
    ss_h, ss_v = int(layout in (1, 2)), int(layout == 1)
    sv = np.where(units["plane"] > 0, ss_v, 0).astype(np.int64)
    end = np.zeros(len(units), np.int64)
    for k in range(2):
        used = (units["ref"][:, k] >= 0)
        dy = units["mvy"][:, k].astype(np.int64) >> (3 + sv)
        e = ((units["y"].astype(np.int64) + units["h"] + dy + 5) << sv) + sv   # luma row bound
        end = np.where(used, np.maximum(end, e), end)
    g = np.clip((np.minimum(end, h) + bh - 1) // bh - 1, 0, bands - 1)
    g = np.where(end >= h, bands - 1, g)
    later = (units["plane"] > 0) & (units["ref"][:, 1] >= 0) & (units["comp"] == 2)
    if later.any():
        luma = {(int(u["x"]), int(u["y"])): int(gi) for u, gi in zip(units[units["plane"] == 0], g[units["plane"] == 0])}
        for i in np.nonzero(later)[0]:
            key = (int(units["x"][i]) << ss_h, int(units["y"][i]) << ss_v)
            g[i] = max(int(g[i]), luma.get(key, bands - 1))
    return g


class PipelinedStream:
    """Frame-pipelined decode of one stream over the ranks of the default process group."""

    def __init__(self, executor, alloc, rank, world, device, bands=1):
        """executor(spec, [ref pictures]) -> picture (an object with .planes: uint8 tensors), or
        with bands > 1 executor(spec, [ref pictures], ready), where ready(g) returns once bands
        0..g of every reference have arrived (None when every reference is local);
        alloc(spec) -> an empty picture of the frame's geometry (receive buffer)."""
        self.executor, self.alloc = executor, alloc
        self.rank, self.world, self.device = rank, world, device
        self.bands = max(1, int(bands))
        self.gloo = dist.is_initialized() and dist.get_backend() == "gloo"
        # one communicator per direction (every rank creates both, in the same order)
        self.up = self.down = None
        if dist.is_initialized() and world > 1:
            self.up, self.down = dist.new_group(), dist.new_group()

    def _group(self, peer, sending):
        """lower -> higher rank messages on `up`, higher -> lower on `down`"""
        return self.up if (peer > self.rank) == sending else self.down

    def _geom(self, spec):
        fr = spec.desc
        return fr["h"], int(fr["layout"] == 1)

    def _send(self, spec, pic, dst, pending):
        """Every band of `pic`, top first, each band as one message per plane."""
        g = self._group(dst, True)
        h, ss_v = self._geom(spec) if self.bands > 1 else (0, 0)
        bh = band_height(h, self.bands) if self.bands > 1 else 0
        for b in range(self.bands):
            for p, t in enumerate(pic.planes):
                if self.bands > 1:
                    lo, hi = band_rows(b, bh, h, ss_v if p else 0)
                    t = t[lo:hi]
                src = t.cpu() if self.gloo and t.is_cuda else t.contiguous()
                pending.append((dist.isend(src, dst, group=g), src))

    def _recv_band(self, spec, pic, b, src):
        g = self._group(src, False)
        h, ss_v = self._geom(spec) if self.bands > 1 else (0, 0)
        bh = band_height(h, self.bands) if self.bands > 1 else 0
        for p, t in enumerate(pic.planes):
            if self.bands > 1:
                lo, hi = band_rows(b, bh, h, ss_v if p else 0)
                t = t[lo:hi]
            if self.gloo and t.is_cuda:
                hbuf = torch.empty_like(t, device="cpu")
                dist.recv(hbuf, src, group=g)
                t.copy_(hbuf)
            else:
                dist.recv(t, src, group=g)

    def run(self, specs):
        """Decode my frames; returns {decode index: output picture} for the frames this rank
        reconstructed (the caller hashes / outputs them)."""
        plan, lu = transfer_plan(specs, self.world), last_use(specs)
        spec_of = {s.idx: s for s in specs}
        B = self.bands
        # per peer: the (frame, band) messages it will send me, in its send order (increasing
        # r, bands top first)
        incoming = {}
        for r, dsts in sorted(plan.items()):
            if self.rank in dsts:
                incoming.setdefault(owner(r, self.world), []).extend((r, b) for b in range(B))
        got = {}          # r -> picture (mine or received), freed after last use
        have = {}         # r -> bands of r received so far (B: complete)
        mine = {}
        pending = []      # (work, tensor) of non-blocking sends

        def pull(r, band):
            """Receive, in the peer's order, until bands 0..band of r are here."""
            src = owner(r, self.world)
            q = incoming[src]
            while have.get(r, 0) <= band:
                n, b = q.pop(0)
                if n not in got:
                    got[n] = self.alloc(spec_of[n])
                self._recv_band(spec_of[n], got[n], b, src)
                have[n] = b + 1

        for s in specs:
            if owner(s.idx, self.world) != self.rank:
                continue
            remote = [r for r in s.refs if owner(r, self.world) != self.rank and have.get(r, 0) < B]
            if B > 1 and remote:
                for r in remote:               # allocate (first band may come later)
                    pull(r, 0)

                def ready(g, remote=remote):
                    for r in remote:
                        pull(r, min(g, B - 1))
                out = self.executor(s, [got[r] for r in s.refs], ready)
                for r in remote:
                    pull(r, B - 1)
            else:
                for r in s.refs:
                    if owner(r, self.world) != self.rank:
                        pull(r, B - 1)
                out = self.executor(s, [got[r] for r in s.refs], None) if B > 1 else \
                    self.executor(s, [got[r] for r in s.refs])
            got[s.idx] = out
            have[s.idx] = B
            mine[s.idx] = out
            for d in plan.get(s.idx, []):
                self._send(s, out, d, pending)
            for r in list(got):
                if lu.get(r, -1) <= s.idx and r not in mine:
                    del got[r]
        for w, _ in pending:
            w.wait()
        return mine


def picture_digest(planes_np):
    h = hashlib.sha256()
    for a in planes_np:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


class DeviceExecutor:
    """Reconstruct one synthetic frame on the device with the batched C-ABI: [MC from the
    reference pictures ->] itx residual -> deblock -> CDEF -> LR, all enqueued on one stream.
    prepare() uploads the frame's descriptors and allocates its pictures once, outside the
    decode loop, so a frame costs five C calls at decode time."""

    def __init__(self, ctx, stream=None, bands=1):
        self.ctx, self.stream, self.bands = ctx, stream, bands
        self.prepared = {}

    def prepare(self, spec):
        import ctypes
        from . import frame as F
        fr = spec.desc
        d = dict(blocks=torch.from_numpy(fr["blocks"].view(np.uint8).copy()).cuda(),
                 coef0=torch.from_numpy(fr["coef"].copy()).cuda(),
                 lf=F.LoopFilterMeta(fr["lf"]), lr=F.LrMeta(fr["lr"]),
                 mc=F.McMeta(*fr["mc"]) if fr.get("mc") is not None else None)
        d["coef"] = d["coef0"].clone()
        d["cdef"] = F.CdefMeta(fr["lf"]["masks"], fr["cdef"], masks_dev=d["lf"].masks)
        if d["mc"] is not None and self.bands > 1:
            # row-level progress: the units split by band group, one mi_mc_frame per group
            # (one shared mask buffer)
            from .synth import mc_sort_units
            units = fr["mc"][0]
            grp = mc_band_groups(units, fr["h"], fr["layout"], self.bands)
            d["mc_bands"] = []
            for g in range(self.bands):
                ug = units[grp == g]
                if len(ug) == 0:
                    d["mc_bands"].append(None)
                    continue
                ug, cs = mc_sort_units(ug)
                m = F.McMeta(ug, cs, np.zeros(1, np.uint8))
                m.masks = d["mc"].masks
                d["mc_bands"].append(m)
        d["frames"] = [self.alloc(spec) for _ in range(4)]            # A, D, B, O
        d["pics"] = [f.picture() for f in d["frames"]]
        d["ss"] = (ctypes.c_uint32 * 20)(*[int(v) for v in fr["size_start"]])
        if d["mc"] is None:
            A = d["frames"][0]
            d["A0"] = [torch.empty_like(t) for t in A.planes]
            for p, a in enumerate(fr["planes"]):
                A.set_plane_np(p, a)
            for t0, t in zip(d["A0"], A.planes):
                t0.copy_(t)
        self.prepared[spec.idx] = d

    def alloc(self, spec):
        from . import frame as F
        fr = spec.desc
        return F.Frame(fr["w"], fr["h"], fr["bpc"], fr["layout"])

    def __call__(self, spec, refs, ready=None):
        """ready (row-level progress, bands > 1): ready(g) returns once bands 0..g of every
        reference have arrived; the MC of band group g is enqueued after it."""
        import ctypes
        from . import frame as F
        if spec.idx not in self.prepared:
            self.prepare(spec)
        d = self.prepared[spec.idx]
        L, h, sp = F.lib(), self.ctx.h, F._stream_ptr(self.stream)
        pa, pd, pb, po = d["pics"]
        d["coef"].copy_(d["coef0"])                 # itxfm_add zeroes the arena it consumes
        if d["mc"] is not None:
            rp = (F.MiPicture * len(refs))(*[r.picture() for r in refs])
            if ready is not None and d.get("mc_bands"):
                for g, m in enumerate(d["mc_bands"]):
                    ready(g)
                    if m is not None:
                        F.check(L.mi_mc_frame(h, ctypes.byref(pa), rp, len(refs), ctypes.c_void_p(m.blocks.data_ptr()),
                                              m.class_start, ctypes.c_void_p(m.masks.data_ptr()), None, sp), "mc")
            else:
                F.check(L.mi_mc_frame(h, ctypes.byref(pa), rp, len(refs), ctypes.c_void_p(d["mc"].blocks.data_ptr()),
                                      d["mc"].class_start, ctypes.c_void_p(d["mc"].masks.data_ptr()), None, sp), "mc")
        else:
            for t, t0 in zip(d["frames"][0].planes, d["A0"]):
                t.copy_(t0)
        F.check(L.mi_itx_frame(h, ctypes.byref(pa), ctypes.c_void_p(d["blocks"].data_ptr()), d["ss"],
                               ctypes.c_void_p(d["coef"].data_ptr()), 0, sp), "itx")
        F.check(L.mi_deblock_frame_to(h, ctypes.byref(pa), ctypes.byref(pd), ctypes.byref(d["lf"].s), sp), "lf")
        F.check(L.mi_cdef_frame(h, ctypes.byref(pd), ctypes.byref(pb), ctypes.byref(d["cdef"].s), sp), "cdef")
        F.check(L.mi_lr_frame(h, ctypes.byref(pb), ctypes.byref(pd), ctypes.byref(po), ctypes.byref(d["lr"].s), sp), "lr")
        return d["frames"][3]


def make_stream_specs(w, h, bpc, layout, n, seed, gop=8, reuse=False):
    """A synthetic stream of n frames in a hierarchical GOP: frame 0 intra (its prediction
    planes given), every other frame predicted by MC from its references' reconstructed
    pictures; descriptors from rav1d_amd.synth.make_frame (seed + display index). reuse: one
    descriptor set per reference count (0, 1, 2) shared by the frames (large frames: the
    generator is slow; the references still differ per frame)."""
    from .synth import make_frame
    specs, cache = [], {}
    for i, (disp, refs) in enumerate(gop_specs(n, gop)):
        key = len(refs) if reuse else i
        if key not in cache:
            fr = make_frame(w, h, bpc, layout, seed=seed + (len(refs) if reuse else disp), with_fg=False,
                            with_mc=bool(refs), nrefs=max(1, len(refs)))
            fr["refs"] = None        # the references are the decoded pictures of `refs`
            cache[key] = fr
        specs.append(FrameSpec(i, refs, True, cache[key]))
    return specs
