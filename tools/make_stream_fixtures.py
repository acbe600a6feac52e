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
    # inter frames: the smallest vectors that together use every inter tool at 8, 10 and 12 bit
    # and every layout (compound avg / w_avg / wedge / seg, OBMC, local and global warp,
    # inter-intra, scaled references, sub-8x8 chroma), from tools/dev feature counts
    ("av1-1-b8-01-size-18x16", "8-bit/size/av1-1-b8-01-size-18x16.ivf"),
    ("av1-1-b8-01-size-18x18", "8-bit/size/av1-1-b8-01-size-18x18.ivf"),
    ("av1-1-b8-01-size-18x34", "8-bit/size/av1-1-b8-01-size-18x34.ivf"),
    ("00000623", "8-bit/data/00000623.ivf"),
    ("00000706", "8-bit/data/00000706.ivf"),
    ("00000711", "8-bit/data/00000711.ivf"),
    ("00000862", "8-bit/data/00000862.ivf"),
    ("00001105", "8-bit/data/00001105.ivf"),
    ("00001132", "8-bit/data/00001132.ivf"),
    ("00001137", "8-bit/data/00001137.ivf"),
    ("00001138", "8-bit/data/00001138.ivf"),
    ("00000716", "10-bit/data/00000716.ivf", "00000716_10bit"),
    ("00000721", "10-bit/data/00000721.ivf", "00000721_10bit"),
    ("00000726", "10-bit/data/00000726.ivf", "00000726_10bit"),
    ("00000831", "10-bit/data/00000831.ivf", "00000831_10bit"),
    ("00000943", "10-bit/data/00000943.ivf", "00000943_10bit"),
    ("av1-1-b10-00-quantizer-61", "10-bit/quantizer/av1-1-b10-00-quantizer-61.ivf"),
    ("av1-1-b10-00-quantizer-62", "10-bit/quantizer/av1-1-b10-00-quantizer-62.ivf"),
    ("av1-1-b10-00-quantizer-63", "10-bit/quantizer/av1-1-b10-00-quantizer-63.ivf"),
    ("test185_302", "10-bit/argon/test185_302.obu"),                  # Annex B, scaled refs
    ("00000732", "12-bit/data/00000732.ivf", "00000732_12bit"),
    ("00000736", "12-bit/data/00000736.ivf", "00000736_12bit"),
    ("00000741", "12-bit/data/00000741.ivf", "00000741_12bit"),
    ("test15240", "12-bit/argon/test15240.obu"),                      # 4:0:0, scaled refs
    ("annexb", "8-bit/features/annexb.obu"),
    ("section5", "8-bit/features/section5.obu"),
    # the largest inter vectors: bench.py's real-stream entries
    ("issue_318", "10-bit/issues/318_tx_4x4.ivf"),                    # 1920x1080 10-bit, 35 frames
    ("00001141", "8-bit/data/00001141.ivf"),                          # 3840x2160 8-bit, 3 frames
    ("issue_295", "8-bit/issues/295_adst_precision.ivf"),             # 2780x2136 8-bit, 25 frames
    # 12-bit identity32 residuals at the column clip (the fused intra kernel's int16 residual
    # wrapped there in round 3)
    ("test15549_5522_4902", "12-bit/argon/test15549_5522_4902.obu"),
]

# the reference's --filmgrain 1 tests (explicit test() entries in the meson files: film grain
# applied to the shown pictures before hashing)
GRAIN = [
    ("av1-1-b8-23-film_grain-50", "8-bit/film_grain/av1-1-b8-23-film_grain-50.ivf", "392a4adc567fa05b210eebe15bcbb491"),
    ("ccvb_film_grain-fg", "8-bit/features/ccvb_film_grain.ivf", "a934b6263b7009746cce5f5bd33224f1"),
    ("309_odd_width", "8-bit/issues/309_odd_width.ivf", "30d31f7c74575e58366898534a87841d"),
    ("av1-1-b10-23-film_grain-50", "10-bit/film_grain/av1-1-b10-23-film_grain-50.ivf",
     "be596f5921854b9a9a5be81c302a5327"),
    ("test5606", "10-bit/argon/test5606.obu", "0888c66e9ad2f6ebc7f6d6fd8b464dd8"),
]



def driver_suite(by_path):
    """The rest of the driver-run GPU suite: every vector of the meson lists (round 4 held every
    10-bit, 12-bit and multi-bit vector and an 8-bit subset; round 5 adds the remaining 8-bit
    data and vq_suite streams). Returns [(name, rel, md5)], names unique."""
    return [(by_path[rel][0], rel, by_path[rel][1]) for rel in sorted(by_path)]


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
        table.append({"name": name, "file": dst, "md5": md5, "cpu": 1, "source": f"tests/dav1d-test-data/{rel}"})
    have = {t["source"] for t in table}
    names = {t["name"] for t in table}
    for name, rel, md5 in driver_suite(by_path):
        if f"tests/dav1d-test-data/{rel}" in have:
            continue
        if name in names:
            name = f"{name}_{rel.split('/')[0].replace('-', '')}"
        assert name not in names, name
        names.add(name)
        dst = rel.replace("/", "__")
        shutil.copyfile(os.path.join("/root/reference/tests/dav1d-test-data", rel), os.path.join(out, dst))
        table.append({"name": name, "file": dst, "md5": md5, "source": f"tests/dav1d-test-data/{rel}"})
    for name, rel, md5 in GRAIN:
        dst = rel.replace("/", "__")
        shutil.copyfile(os.path.join("/root/reference/tests/dav1d-test-data", rel), os.path.join(out, dst))
        table.append({"name": name, "file": dst, "md5": md5, "filmgrain": 1, "cpu": 1,
                      "source": f"tests/dav1d-test-data/{rel} --filmgrain 1"})
    json.dump(table, open(os.path.join(out, "vectors.json"), "w"), indent=1)
    print(len(table), "vectors")
