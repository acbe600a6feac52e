"""Diagnostic: one reference vector through the device path and the oracle, frame by frame, at
each inloop_filters setting (0 = reconstruction only, 1 deblock, 2 CDEF, 4 LR, 14 all; the
reference's --inloopfilters mask): prints the first differing shown frame, plane, pixel count
and bounding box. usage: python tools/dev/vec_diff.py NAME [DIR]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rav1d_amd import stream as S  # noqa: E402
from rav1d_amd.av1dec import stream_events  # noqa: E402
from rav1d_amd.frame import Context  # noqa: E402
from tests.stream_lib import oracle_frame  # noqa: E402


class Collect:
    def __init__(self):
        self.frames = []

    def write(self, pic):
        from rav1d_amd.output import HostPicture
        h = HostPicture.__new__(HostPicture)
        h.pic = pic
        self.frames.append([h.plane_np(p).copy() for p in range(3 if pic.layout else 1)])


def oracle_frames(data, lf):
    pics, out, info = {}, [], []
    for ev in stream_events(data, inloop_filters=lf):
        if ev.frame:
            fr = ev.frame.contents
            refs = [None if r < 0 else pics[r][:3] for r in ev.ref_pic]
            pics[ev.pic_id] = (oracle_frame(fr, refs), fr.up_w, fr.h, fr.layout)
        if ev.show_pic >= 0:
            planes, w, h, lay = pics[ev.show_pic]
            ss_hor, ss_ver = int(lay in (1, 2)), int(lay == 1)
            dims = [(w, h)] + [((w + ss_hor) >> ss_hor, (h + ss_ver) >> ss_ver)] * 2
            out.append([planes[p][:dims[p][1], :dims[p][0]] for p in range(len(planes))])
            info.append((w, h, lay))
        for i in range(ev.n_release):
            pics.pop(ev.release[i], None)
    return out, info


def main():
    name = sys.argv[1]
    d = sys.argv[2] if len(sys.argv) > 2 else "sweep_vectors"
    v = next(x for x in json.load(open(os.path.join(d, "vectors.json"))) if x["name"] == name)
    data = open(os.path.join(d, v["file"]), "rb").read()
    ctx = Context(0)
    for lf in (0, 1, 3, 7, 14):
        want, info = oracle_frames(data, lf)
        m = Collect()
        S.decode_to_muxer(ctx, data, m, apply_grain=False, in_flight=1, inloop_filters=lf)
        first = None
        for k, (got, exp) in enumerate(zip(m.frames, want)):
            for p in range(len(exp)):
                if not np.array_equal(got[p], exp[p]):
                    ys, xs = np.nonzero(got[p] != exp[p])
                    first = (k, p, len(ys), (int(ys.min()), int(ys.max()), int(xs.min()), int(xs.max())), info[k])
                    break
            if first:
                break
        print("inloop_filters", lf, "frames", len(m.frames), len(want), "first diff", first, flush=True)


if __name__ == "__main__":
    main()
