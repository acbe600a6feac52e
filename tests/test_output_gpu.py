"""GPU: the output side (include/mi_av1out.h). mi_output_picture writes the displayed picture
into pinned host memory — a DMA copy of the visible area, or the film-grain kernel storing
straight into host memory — checked against the device picture and the oracle's
rav1d_apply_grain; whole streams decoded on the device and written through the product md5
muxer match the reference's MD5 vectors."""
import json
import os

import numpy as np
import pytest
import torch

from rav1d_amd.frame import Frame
from rav1d_amd.output import HostPicture, Muxer, output_picture
from rav1d_amd.synth import make_fg_params
from tests import oracle_lib
from tests.test_lr_gpu import to_frame
from tests.test_oracle_lf import pad_planes
from tests.test_oracle_lr import planes_for

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "streams")
VECTORS = json.load(open(os.path.join(GOLDEN, "vectors.json")))


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
def test_output_copy_is_the_picture(gpu, bpc, layout):
    w, h = 203, 131
    rng = np.random.default_rng(bpc * 10 + layout)
    planes = planes_for(w, h, bpc, layout, rng)
    src = to_frame(planes, w, h, bpc, layout)
    host = HostPicture(w, h, bpc, layout)
    output_picture(gpu, src, host)
    torch.cuda.synchronize()
    for p in range(len(planes)):
        assert np.array_equal(host.plane_np(p), src.plane_np(p)), f"plane {p}"


@pytest.mark.parametrize("bpc,layout,size,seed", [(10, 1, (256, 160), 1), (8, 1, (201, 133), 2),
                                                   (12, 3, (128, 96), 3), (10, 2, (160, 90), 4),
                                                   (8, 0, (96, 64), 5), (10, 1, (3840, 2160), 6)])
def test_output_with_grain_matches_oracle(gpu, bpc, layout, size, seed):
    """Film grain fused with the device-to-host copy (the grain kernel's stores land in host
    memory) equals rav1d_apply_grain on the same input."""
    w, h = size
    rng = np.random.default_rng(seed)
    planes = planes_for(w, h, bpc, layout, rng)
    fg = make_fg_params(rng, layout)
    src = to_frame(planes, w, h, bpc, layout)
    host = HostPicture(w, h, bpc, layout)
    output_picture(gpu, src, host, fg)
    torch.cuda.synchronize()
    ref = oracle_lib.film_grain(pad_planes(planes, w, h, bpc, layout), bpc, layout, w, h, fg, 0)
    for p in range(len(planes)):
        ph, pw = planes[p].shape
        assert np.array_equal(host.plane_np(p), ref[p][:ph, :pw]), f"plane {p}"
    # the device picture is untouched
    for p in range(len(planes)):
        assert np.array_equal(src.plane_np(p), planes[p])


def test_output_rejects_geometry_mismatch(gpu):
    import ctypes
    from rav1d_amd import lib
    src = Frame(64, 64, 10, 1)
    host = HostPicture(64, 48, 10, 1)
    pic = src.picture()
    assert lib().mi_output_picture(gpu.h, ctypes.byref(pic), ctypes.byref(host.pic), None, 0, None) == -22


@pytest.mark.parametrize("v", VECTORS, ids=[v["name"] for v in VECTORS])
def test_stream_to_md5_muxer_matches_reference(gpu, v):
    """Stream -> front-end -> device reconstruction and filters -> mi_output_picture -> md5 muxer:
    the reference CLI's `--muxer md5` result for the vector."""
    from rav1d_amd.stream import decode_to_muxer
    data = open(os.path.join(GOLDEN, v["file"]), "rb").read()
    m = Muxer("md5")
    # the reference's md5 muxer defaults to --filmgrain 0; its explicit --filmgrain 1 vectors
    # get the grain fused into the output copy (mi_output_picture)
    n = decode_to_muxer(gpu, data, m, apply_grain=bool(v.get("filmgrain")))
    assert n > 0
    assert m.verify(v["md5"]) == 0, f"{v['name']}: {m.digest()} != {v['md5']}"
    m.close()


def test_stream_to_md5_muxer_unpipelined_matches_reference(gpu):
    """The same chain with every frame checked by mi_frame_end before it is shown (no overlap of
    the front-end with the device)."""
    from rav1d_amd.stream import decode_to_muxer
    v = next(x for x in VECTORS if x["name"] == "av1-1-b8-02-allintra")
    data = open(os.path.join(GOLDEN, v["file"]), "rb").read()
    m = Muxer("md5")
    assert decode_to_muxer(gpu, data, m, pipelined=False) == 39
    assert m.verify(v["md5"]) == 0
    m.close()
