"""Copy the reference's MD5 test vectors that the front-end decodes into tests/golden/streams/
(data only: the IVF inputs and the expected MD5 from tests/dav1d-test-data/**/meson.build), and
write tests/golden/streams/vectors.json. Run in the container (reads /root/reference)."""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.scan_vectors import vectors  # noqa: E402

# (meson name, path under tests/dav1d-test-data) of the vectors pinned so far
PINNED = [
    ("av1-1-b8-02-allintra", "8-bit/intra/av1-1-b8-02-allintra.ivf"),
    ("issue_320", "8-bit/issues/320_tennis.ivf"),
    ("issue_321", "8-bit/issues/321_tennis.ivf"),
    ("issue_322", "8-bit/issues/322_tennis.ivf"),
    ("issue_324", "8-bit/issues/324_tennis.ivf"),
    ("issue_325", "8-bit/issues/325_tennis.ivf"),
    ("itut_t35", "8-bit/features/itut_t35.ivf"),
    ("long_leb", "8-bit/features/long_leb.ivf"),
    ("00000791", "12-bit/data/00000791.ivf"),
    ("itut_t35", "10-bit/features/itut_t35.ivf", "itut_t35_10bit"),   # 4K 10-bit, intra block copy
]

if __name__ == "__main__":
    out = os.path.join(ROOT, "tests", "golden", "streams")
    os.makedirs(out, exist_ok=True)
    by_path = {os.path.relpath(p, "/root/reference/tests/dav1d-test-data"): (n, m) for n, p, m in vectors()}
    table = []
    for name, rel, *alias in PINNED:
        n, md5 = by_path[rel]
        assert n == name, (n, name)
        name = alias[0] if alias else name
        dst = rel.replace("/", "__")
        shutil.copyfile(os.path.join("/root/reference/tests/dav1d-test-data", rel), os.path.join(out, dst))
        table.append({"name": name, "file": dst, "md5": md5, "source": f"tests/dav1d-test-data/{rel}"})
    json.dump(table, open(os.path.join(out, "vectors.json"), "w"), indent=1)
    print(len(table), "vectors")
