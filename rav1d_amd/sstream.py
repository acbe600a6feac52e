"""Single-stream multi-GPU decode: frame pipelining with reference exchange.

rav1d decodes one stream with frame threads (src/thread_task.rs:301-575): frame k's
reconstruction waits until the reference frames it reads have progressed far enough, and
frames whose references are ready run concurrently. Here every GPU is one frame context: frame
k (decode order) runs on rank k % N, and a reference picture produced on another rank arrives
by a point-to-point transfer — RCCL send/recv over xGMI under the "nccl" backend (device
tensors, no host staging), host-staged under "gloo". Dependencies are whole frames (a frame
starts once its references are complete), which is rav1d's frame-threading model without
row-level progress.

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


class PipelinedStream:
    """Frame-pipelined decode of one stream over the ranks of the default process group."""

    def __init__(self, executor, alloc, rank, world, device):
        """executor(spec, [ref pictures]) -> picture (an object with .planes: uint8 tensors);
        alloc(spec) -> an empty picture of the frame's geometry (receive buffer)."""
        self.executor, self.alloc = executor, alloc
        self.rank, self.world, self.device = rank, world, device
        self.gloo = dist.is_initialized() and dist.get_backend() == "gloo"
        # one communicator per direction (every rank creates both, in the same order)
        self.up = self.down = None
        if dist.is_initialized() and world > 1:
            self.up, self.down = dist.new_group(), dist.new_group()

    def _group(self, peer, sending):
        """lower -> higher rank messages on `up`, higher -> lower on `down`"""
        return self.up if (peer > self.rank) == sending else self.down

    def _send(self, pic, dst, pending):
        g = self._group(dst, True)
        for t in pic.planes:
            src = t.cpu() if self.gloo and t.is_cuda else t
            pending.append((dist.isend(src, dst, group=g), src))

    def _recv(self, spec_of, r, src):
        pic = self.alloc(spec_of[r])
        g = self._group(src, False)
        for t in pic.planes:
            if self.gloo and t.is_cuda:
                h = torch.empty_like(t, device="cpu")
                dist.recv(h, src, group=g)
                t.copy_(h)
            else:
                dist.recv(t, src, group=g)
        return pic

    def run(self, specs):
        """Decode my frames; returns {decode index: output picture} for the frames this rank
        reconstructed (the caller hashes / outputs them)."""
        plan, lu = transfer_plan(specs, self.world), last_use(specs)
        spec_of = {s.idx: s for s in specs}
        # per peer: the frames it will send me, in its send order (increasing r)
        incoming = {}
        for r, dsts in sorted(plan.items()):
            if self.rank in dsts:
                incoming.setdefault(owner(r, self.world), []).append(r)
        got = {}          # r -> picture (mine or received), freed after last use
        mine = {}
        pending = []      # (work, tensor) of non-blocking sends
        for s in specs:
            if owner(s.idx, self.world) != self.rank:
                continue
            for r in s.refs:
                if r in got:
                    continue
                src = owner(r, self.world)
                q = incoming[src]
                while True:                    # in the peer's order, up to r
                    n = q.pop(0)
                    got[n] = self._recv(spec_of, n, src)
                    if n == r:
                        break
            out = self.executor(s, [got[r] for r in s.refs])
            got[s.idx] = out
            mine[s.idx] = out
            for d in plan.get(s.idx, []):
                self._send(out, d, pending)
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

    def __init__(self, ctx, stream=None):
        self.ctx, self.stream = ctx, stream
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

    def __call__(self, spec, refs):
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
