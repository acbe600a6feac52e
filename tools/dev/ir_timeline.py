"""Where the persistent intra reconstruction's time goes, from an MI_IR_TIMELINE dump
(s_memrealtime stamps per unit: 0 dequeued, 1 row pass done, 2 flag wait done, 3 prediction done,
4 column pass done / granules stored, 5 tile stored, 6 flag stored). Walks the critical path
back from the last unit: per hop the producer's stamp 4 -> the consumer's stamp 3 (hand-off +
edges + prediction) and the consumer's 3 -> 4 (column pass).
Dev experiment: MI_IR_TIMELINE=f python tools/dev/intra_strips.py X; python tools/dev/ir_timeline.py f"""
import sys

import numpy as np

IB = np.dtype([("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"), ("plane", "u1"), ("mode", "u1"),
               ("angle", "i1"), ("flags", "u1"), ("filt", "u1"), ("alpha", "i1"), ("tw", "<u2"), ("th", "<u2"),
               ("mw", "<u2"), ("mh", "<u2"), ("aux", "<u4"), ("pal", "<u4"), ("res", "<u4")])
buf = open(sys.argv[1], "rb").read()
off = 0
rec = 0
while off < len(buf):
    n, nd, ns, gran = np.frombuffer(buf, np.int32, 4, off)
    off += 16
    t8 = np.frombuffer(buf, np.uint64, n * 16, off).reshape(n, 16).astype(np.int64)
    t = t8[:, :7]
    off += n * 128
    b = np.frombuffer(buf, IB, n, off)
    off += n * IB.itemsize
    ds = np.frombuffer(buf, np.int32, n + 1, off)
    off += (n + 1) * 4
    deps = np.frombuffer(buf, np.int32, nd, off)
    off += nd * 4
    off += ns * 4
    rec += 1
    if rec > 1 and len(sys.argv) < 3:
        continue
    us = (t - t[:, 0].min()) / 100.0
    span = us[:, 6].max()
    ph = np.diff(us, axis=1)
    g7 = (t8[:, 7] - t[:, 0].min()) / 100.0
    print(f"units {n} granules {gran} span {span:.1f} us; mean stage us: "
          + " ".join(f"{k}->{k + 1} {ph[:, k].mean():.2f}" for k in range(6)))
    if gran:
        ep = us[:, 3] - g7
        m = b["mode"].astype(int)
        sz = b["w"].astype(int) * b["h"]
        print("  edges->pred us by mode (4x4 units): " + ", ".join(
            f"{k}:{ep[(m == k) & (sz == 16)].mean():.2f}/{((m == k) & (sz == 16)).sum()}" for k in np.unique(m)
            if ((m == k) & (sz == 16)).any()))
        print("  by size (all modes): " + ", ".join(f"{k}:{ep[sz == k].mean():.2f}/{(sz == k).sum()}"
                                                    for k in np.unique(sz)))
        t0 = t[:, 0].min()
        st = [(t8[:, k] - t0) / 100.0 for k in (7, 8, 9, 10)]
        m0 = (m == 0) & (sz == 16)
        print(f"  4x4 DC: fetch->8 {(st[1] - st[0])[m0].mean():.2f} 8->9 (edge LDS + syncs) {(st[2] - st[1])[m0].mean():.2f} "
              f"9->10 (predict) {(st[3] - st[2])[m0].mean():.2f} 10->3 {(us[:, 3] - st[3])[m0].mean():.2f}")
        d = [(t8[:, k] - t0) / 100.0 for k in (11, 12, 13)]
        print(f"  4x4 DC inside: 9->dc0 {(d[0] - st[2])[m0].mean():.2f} dc0->dc1 (sum) {(d[1] - d[0])[m0].mean():.2f} "
              f"dc1->dc2 (put) {(d[2] - d[1])[m0].mean():.2f} dc2->10 {(st[3] - d[2])[m0].mean():.2f}")
        print(f"  fetch (2->7) mean {(g7 - us[:, 2]).mean():.2f}, pred 4x4 mode 0 filt {ep[(m == 13) & (sz == 16)].mean() if ((m == 13) & (sz == 16)).any() else 0:.2f}")
    # critical path
    c = int(np.argmax(us[:, 4]))
    hops, xfer, itx, late, wl, pred = 0, 0.0, 0.0, 0.0, 0, 0.0
    sizes = []
    while True:
        d = deps[ds[c]:ds[c + 1]]
        itx += us[c, 4] - us[c, 3]
        if len(d) == 0:
            break
        p = int(d[np.argmax(us[d, 4])])
        if us[p, 4] < us[c, 1]:
            # the consumer was not waiting: its own worker (dequeue, row pass) was later
            wl += 1
            late += us[c, 1] - us[p, 4]
        xfer += us[c, 3] - max(us[p, 4], us[c, 1])
        if gran:
            pred += us[c, 3] - g7[c]
        sizes.append(int(b[c]["w"]) * int(b[c]["h"]))
        hops += 1
        c = p
    print(f"  critical path {hops} hops from {us[c, 0]:.1f} us: hand-off+edges+pred {xfer:.0f} us "
          f"({xfer / max(hops, 1):.2f}/hop), column pass {itx:.0f} us ({itx / max(hops, 1):.2f}/hop), "
          f"worker-late {wl} hops {late:.0f} us; 4x4 hops {sum(1 for s in sizes if s == 16)}; "
          f"of the hand-off: edges->pred done {pred:.0f} us ({pred / max(hops, 1):.2f}/hop)")
