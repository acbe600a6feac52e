"""Every reference MD5 vector through the device path (front-end -> mi_frame_run -> output copy
-> product md5 muxer), on the GPU box.

    python tools/gpu_sweep.py prepare DIR     # container: copy the vectors + expected MD5s into DIR
    python tools/gpu_sweep.py run DIR OUT     # GPU box: decode them all, one JSON line per vector

DIR is scratch (gitignored): the vectors are the reference's test data
(tests/dav1d-test-data/**/meson.build) and travel to the box only for this sweep.
"""
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def prepare(d):
    from tools.make_stream_fixtures import GRAIN
    from tools.scan_vectors import vectors
    os.makedirs(d, exist_ok=True)
    base = "/root/reference/tests/dav1d-test-data"
    table = [(n, os.path.relpath(p, base), m, 0) for n, p, m in vectors()]
    table += [(n, rel, m, 1) for n, rel, m in GRAIN]
    out = []
    for name, rel, md5, fg in table:
        dst = rel.replace("/", "__")
        shutil.copyfile(os.path.join(base, rel), os.path.join(d, dst))
        out.append({"name": name, "file": dst, "md5": md5, "filmgrain": fg})
    json.dump(out, open(os.path.join(d, "vectors.json"), "w"))
    print(len(out), "vectors")


def run(d, out_path):
    from rav1d_amd.frame import Context
    from rav1d_amd.output import Muxer
    from rav1d_amd.stream import decode_to_muxer
    ctx = Context(0)
    table = json.load(open(os.path.join(d, "vectors.json")))
    ok = bad = err = 0
    with open(out_path, "w") as f:
        for v in table:
            data = open(os.path.join(d, v["file"]), "rb").read()
            m = Muxer("md5")
            t = time.time()
            try:
                n = decode_to_muxer(ctx, data, m, apply_grain=bool(v["filmgrain"]))
                got = m.digest()
                st = "ok" if got == v["md5"] else "MISMATCH"
            except Exception as e:  # noqa: BLE001 - record and continue
                n, got, st = 0, str(e)[:100], "error"
            m.close()
            ok += st == "ok"
            bad += st == "MISMATCH"
            err += st == "error"
            f.write(json.dumps({"name": v["name"], "file": v["file"], "status": st, "frames": n, "md5": got,
                                "s": round(time.time() - t, 3)}) + "\n")
            f.flush()
            print(st, v["name"], n, flush=True)
    print(json.dumps({"ok": ok, "mismatch": bad, "error": err, "total": len(table)}))


if __name__ == "__main__":
    if sys.argv[1] == "prepare":
        prepare(sys.argv[2])
    else:
        run(sys.argv[2], sys.argv[3])
