"""Reference MD5 vectors through the front-end and the CPU restatement (the oracle's pin).

The vectors and their MD5s are the reference's own (tests/dav1d-test-data/**/meson.build, copied
into tests/golden/streams/ by tools/make_stream_fixtures.py); the MD5 is taken over the shown
frames exactly as the md5 muxer does (tools/output/md5.rs:541-637). A match pins the whole
oracle chain used by these streams — intra prediction (all modes, CfL, palette, filter intra,
edge filter / upsampling), inter prediction (single / compound / wedge / segmentation masks,
OBMC, local and global warp, inter-intra, scaled references, sub-8x8 chroma), itx, deblocking,
CDEF, loop restoration and (for the reference's --filmgrain 1 vectors) film grain — bit for bit
to rav1d. Inputs are IVF, Annex B or section-5 OBU streams, demuxed as the reference CLI does.
"""
import json
import os

import pytest

from tests.stream_lib import decode_stream

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "streams")
# the CPU suite decodes the "cpu" subset (every tool, layout and bit depth; a few minutes);
# test_streams_gpu.py runs all of them on the device
VECTORS = [v for v in json.load(open(os.path.join(GOLDEN, "vectors.json"))) if v.get("cpu")]


def load(v):
    return open(os.path.join(GOLDEN, v["file"]), "rb").read()


@pytest.mark.parametrize("threads", [1, 4], ids=["t1", "t4"])
@pytest.mark.parametrize("v", VECTORS, ids=[v["name"] for v in VECTORS])
def test_oracle_matches_reference_md5(v, threads):
    """threads 4: the front-end's frame threads (intra frames) and tile threads (every frame's
    tiles on their own decoders, work lists merged in tile order)."""
    md5, n = decode_stream(load(v), apply_grain=bool(v.get("filmgrain")), threads=threads)
    assert n > 0
    assert md5 == v["md5"], f"{v['name']}: {n} frames, md5 {md5} != {v['md5']}"


def test_front_end_rejects_garbage():
    from rav1d_amd.av1dec import Av1Decoder
    dec = Av1Decoder()
    with pytest.raises(RuntimeError):
        dec.send(bytes([0x12, 0x00, 0x0a, 0x0b, 0x00, 0x00, 0x00, 0x24, 0xff, 0xff, 0xff, 0xff, 0xff]))
        list(dec.events())


@pytest.mark.parametrize("threads", [2, 5])
def test_frame_threads_match_reference_md5(threads):
    """The front-end's frame threads (mi_dec_set_threads): intra frames decoded on worker
    threads, events in decode order, MD5 unchanged."""
    for name in ("av1-1-b8-02-allintra", "itut_t35", "00000791"):
        v = next(x for x in VECTORS if x["name"] == name)
        data = open(os.path.join(GOLDEN, v["file"]), "rb").read()
        md5, n = decode_stream(data, threads=threads)
        assert md5 == v["md5"], name
