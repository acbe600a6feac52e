"""Decode the reference's MD5 test vectors through front-end + oracle (container only: reads
/root/reference/tests/dav1d-test-data). Prints one line per vector: ok / MISMATCH / error.

    python tools/scan_vectors.py [substring ...]
"""
import os
import re
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DATA = "/root/reference/tests/dav1d-test-data"


def vectors():
    out = []
    for d, _, files in os.walk(DATA):
        if "meson.build" not in files:
            continue
        txt = open(os.path.join(d, "meson.build")).read()
        for name, f, md5 in re.findall(r"\['([^']+)',\s*files\('([^']+)'\),\s*'([0-9a-f]{32})'\]", txt):
            out.append((name, os.path.join(d, f), md5))
    return sorted(out)


def run(v):
    name, path, md5 = v
    from tests.stream_lib import decode_stream
    t = time.time()
    try:
        got, n = decode_stream(open(path, "rb").read())
    except Exception as e:  # noqa: BLE001 - report and continue
        return f"error    {name} {type(e).__name__}: {str(e)[:120]}"
    tag = "ok      " if got == md5 else "MISMATCH"
    return f"{tag} {name} frames={n} {time.time() - t:.1f}s {os.path.getsize(path)}B"


if __name__ == "__main__":
    vs = [v for v in vectors() if not sys.argv[1:] or any(s in v[0] or s in v[1] for s in sys.argv[1:])]
    with ProcessPoolExecutor(int(os.environ.get("JOBS", "6"))) as ex:
        for line in ex.map(run, vs):
            print(line, flush=True)
