"""Output muxers (libmi_av1dec.so, include/mi_av1out.h) against the reference's muxer rules
(tools/output/md5.rs:541-637, yuv.rs, y4m2.rs), on the CPU. The md5 muxer is also pinned by
the reference's own vectors in tests/test_streams.py (every stream's MD5 goes through it)."""
import hashlib
import os

import numpy as np
import pytest

from rav1d_amd.output import Muxer, host_picture_np
from tests.stream_lib import alloc_picture, md5_update_picture


def random_picture(rng, w, h, bpc, layout):
    planes = alloc_picture(w, h, bpc, layout)
    for p in planes:
        p[...] = rng.integers(0, 1 << bpc, size=p.shape)
    return planes


CASES = [(w, h, bpc, layout) for (w, h) in [(64, 48), (33, 17), (1, 1)] for bpc in (8, 10, 12) for layout in (0, 1, 2, 3)]


@pytest.mark.parametrize("w,h,bpc,layout", CASES)
def test_md5_muxer_matches_md5_write(w, h, bpc, layout):
    rng = np.random.default_rng(w * 1000 + h * 10 + bpc + layout)
    ref = hashlib.md5()
    m = Muxer("md5")
    for _ in range(3):
        planes = random_picture(rng, w, h, bpc, layout)
        md5_update_picture(ref, planes, w, h, layout)
        m.write(host_picture_np(planes, w, h, bpc, layout))
    assert m.digest() == ref.hexdigest()
    assert m.verify(ref.hexdigest()) == 0
    m.close()


def test_md5_verify_mismatch_and_short_string():
    rng = np.random.default_rng(5)
    planes = random_picture(rng, 16, 16, 8, 1)
    for s, want in (("0" * 32, 1), ("abc", -1)):
        m = Muxer("md5")
        m.write(host_picture_np(planes, 16, 16, 8, 1))
        assert m.verify(s) == want
        m.close()


def test_md5_muxer_file_trailer(tmp_path):
    rng = np.random.default_rng(6)
    planes = random_picture(rng, 40, 24, 10, 1)
    f = str(tmp_path / "out.md5")
    m = Muxer("md5", f)
    m.write(host_picture_np(planes, 40, 24, 10, 1))
    m.close()
    ref = hashlib.md5()
    md5_update_picture(ref, planes, 40, 24, 1)
    assert open(f).read() == ref.hexdigest() + "\n"


def rows_bytes(planes, w, h, layout):
    out = [np.ascontiguousarray(planes[0][:h, :w]).tobytes()]
    if layout:
        sh, sv = int(layout in (1, 2)), int(layout == 1)
        cw, ch = (w + sh) >> sh, (h + sv) >> sv
        out += [np.ascontiguousarray(planes[p][:ch, :cw]).tobytes() for p in (1, 2)]
    return b"".join(out)


@pytest.mark.parametrize("w,h,bpc,layout", [(33, 17, 8, 1), (64, 48, 10, 2), (20, 10, 12, 3), (16, 8, 8, 0)])
def test_yuv_muxer_writes_visible_rows(tmp_path, w, h, bpc, layout):
    rng = np.random.default_rng(7)
    f = str(tmp_path / "out.yuv")
    m = Muxer("yuv", f, w, h, bpc, layout)
    pics = [random_picture(rng, w, h, bpc, layout) for _ in range(2)]
    for planes in pics:
        m.write(host_picture_np(planes, w, h, bpc, layout))
    m.close()
    assert open(f, "rb").read() == b"".join(rows_bytes(p, w, h, layout) for p in pics)


def y4m_expected_header(w, h, bpc, layout, chr, render, fps):
    """write_header (tools/output/y4m2.rs): tag and reduced aspect ratio."""
    if layout == 1 and bpc == 8:
        tag = ["420jpeg", "420mpeg2", "420"][chr if 0 <= chr <= 2 else 0]
    else:
        tag = [["mono", "mono10", "mono12"], [None, "420p10", "420p12"], ["422", "422p10", "422p12"],
               ["444", "444p10", "444p12"]][layout][{8: 0, 10: 1, 12: 2}[bpc]]
    aw, ah = h * render[0], w * render[1]
    import math
    g = math.gcd(aw, ah)
    return f"YUV4MPEG2 W{w} H{h} F{fps[0]}:{fps[1]} Ip A{aw // g}:{ah // g} C{tag}\n".encode()


@pytest.mark.parametrize("w,h,bpc,layout,chr,render", [
    (64, 48, 8, 1, 0, (64, 48)), (64, 48, 8, 1, 1, (64, 48)), (64, 48, 8, 1, 2, (64, 48)),
    (1920, 1088, 8, 1, 0, (1920, 1080)), (40, 20, 10, 1, 0, (80, 20)), (16, 16, 12, 2, 0, (16, 16)),
    (16, 16, 8, 3, 0, (16, 16)), (16, 16, 10, 0, 0, (16, 16))])
def test_y4m2_muxer(tmp_path, w, h, bpc, layout, chr, render):
    rng = np.random.default_rng(8)
    f = str(tmp_path / "out.y4m")
    fps = (30000, 1001)
    m = Muxer("y4m2", f, w, h, bpc, layout, chr=chr, render=render, fps=fps)
    pics = [random_picture(rng, w, h, bpc, layout) for _ in range(2)]
    for planes in pics:
        m.write(host_picture_np(planes, w, h, bpc, layout))
    m.close()
    want = y4m_expected_header(w, h, bpc, layout, chr, render, fps)
    want += b"".join(b"FRAME\n" + rows_bytes(p, w, h, layout) for p in pics)
    assert open(f, "rb").read() == want


def test_null_and_unknown_muxers(tmp_path):
    m = Muxer("null")
    planes = random_picture(np.random.default_rng(9), 8, 8, 8, 1)
    m.write(host_picture_np(planes, 8, 8, 8, 1))
    m.close()
    from rav1d_amd import MiError
    with pytest.raises(MiError):
        Muxer("gif")
    with pytest.raises(MiError):
        Muxer("yuv", os.path.join(str(tmp_path), "no", "such", "dir.yuv"))
