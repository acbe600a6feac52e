"""Two device lanes (decode_to_muxer in_flight=2): per-frame comparison against one lane, with
variants that isolate the cause. GPU box only (dev experiment).

    python tools/dev/lane_race.py [vector] [reps]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from rav1d_amd import frame as F  # noqa: E402
from rav1d_amd.av1dec import stream_events  # noqa: E402
from rav1d_amd.output import HostPicture, output_picture  # noqa: E402
from rav1d_amd.stream import _refs, frame_end, run_frame  # noqa: E402


class Collect:
    """A muxer that keeps a copy of every picture it is given."""

    def __init__(self):
        self.frames = []

    def write(self, pic):
        from rav1d_amd.output import HostPicture
        h = HostPicture.__new__(HostPicture)
        h.pic = pic
        self.frames.append([h.plane_np(p) for p in range(3 if pic.layout else 1)])


def d2m(ctx, data, in_flight, threads=8):
    from rav1d_amd.stream import decode_to_muxer
    m = Collect()
    decode_to_muxer(ctx, data, m, in_flight=in_flight, threads=threads)
    return m.frames


def decode(ctxs, data, streams, keep_alive=False, serialize=False, threads=8, sync_frame=False, lazy=False):
    """decode_to_muxer's loop, frames alternating over (ctx, stream) lanes; returns per-shown-frame
    plane copies. serialize: each frame's stream waits for the previous frame's event."""
    pics, done_ev, out = {}, {}, []
    kept = []
    k, last = 0, None
    nl = len(ctxs)
    for st in streams[1:]:
        st.wait_stream(streams[0])
    for ev in stream_events(data, threads):
        if ev.frame:
            li = k % nl
            k += 1
            for r in ev.ref_pic:
                if r >= 0 and r in done_ev:
                    streams[li].wait_event(done_ev[r])
            if serialize and last is not None:
                streams[li].wait_event(last)
            with torch.cuda.stream(streams[li]):
                ps = run_frame(ctxs[li], ev.frame.contents, streams[li], _refs(pics, ev, key=lambda p: p[0]))
            pics[ev.pic_id] = (ps, li)
            e = torch.cuda.Event()
            e.record(streams[li])
            done_ev[ev.pic_id] = e
            last = e
            if sync_frame:
                torch.cuda.synchronize()
        if ev.show_pic >= 0:
            ps, li = pics[ev.show_pic]
            o = ps.output()
            h = HostPicture(o.w, o.h, o.bpc, o.layout)
            output_picture(ctxs[li], o, h, None, 0, streams[li])
            d = torch.cuda.Event()
            d.record(streams[li])
            if lazy:
                out.append((h, d, o.layout))
            else:
                d.synchronize()
                out.append([h.plane_np(p) for p in range(3 if o.layout else 1)])
                h.free()
        for i in range(ev.n_release):
            x = pics.pop(ev.release[i], None)
            done_ev.pop(ev.release[i], None)
            if keep_alive and x is not None:
                kept.append(x)
    torch.cuda.synchronize()
    for c, s in zip(ctxs, streams):
        frame_end(c, s)
    if lazy:
        res = []
        for h, d, lay in out:
            d.synchronize()
            res.append([h.plane_np(p) for p in range(3 if lay else 1)])
            h.free()
        out = res
    return out


def compare(ref, got):
    bad = []
    for f, (a, b) in enumerate(zip(ref, got)):
        for p, (x, y) in enumerate(zip(a, b)):
            if not np.array_equal(x, y):
                d = np.argwhere(x != y)
                (y0, x0), (y1, x1) = d.min(0), d.max(0)
                bad.append(dict(frame=f, plane=p, n=int(len(d)), bbox=[int(x0), int(y0), int(x1), int(y1)]))
    return bad


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "av1-1-b8-02-allintra"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    g = os.path.join(ROOT, "tests/golden/streams")
    v = [x for x in json.load(open(g + "/vectors.json")) if x["name"] == name][0]
    data = open(os.path.join(g, v["file"]), "rb").read()
    c0 = F.Context(0)
    s0 = torch.cuda.current_stream()
    ref = decode([c0], data, [s0], threads=1)
    print(name, "frames", len(ref), flush=True)
    c1, s1 = F.Context(0), torch.cuda.Stream()
    s0b = torch.cuda.Stream()
    for r in range(reps):
        bad = compare(ref, d2m(c0, data, 1))
        print("d2m_1lane", r, "frames_bad", len({b["frame"] for b in bad}), bad[:6], flush=True)
    for r in range(reps):
        bad = compare(ref, d2m(c0, data, 2))
        print("d2m_2lanes", r, "frames_bad", len({b["frame"] for b in bad}), bad[:6], flush=True)
    variants = [
        ("2lanes_lazy", dict(ctxs=[c0, c1], streams=[s0, s1], lazy=True)),
        ("2lanes_lazy_keepalive", dict(ctxs=[c0, c1], streams=[s0, s1], lazy=True, keep_alive=True)),
        ("2lanes", dict(ctxs=[c0, c1], streams=[s0, s1])),
        ("2lanes_lazy_serialized", dict(ctxs=[c0, c1], streams=[s0, s1], lazy=True, serialize=True)),
        ("2ctx_1stream_lazy", dict(ctxs=[c0, c1], streams=[s0, s0], lazy=True)),
    ]
    for vn, kw in variants:
        for r in range(reps):
            got = decode(data=data, **kw)
            bad = compare(ref, got)
            print(vn, r, "frames_bad", len({b["frame"] for b in bad}), bad[:6], flush=True)


if __name__ == "__main__":
    main()
