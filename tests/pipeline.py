"""The whole implemented DSP pipeline, once through the oracle (CPU) and once through the
C-ABI on the device: [MC ->] recon(itx) -> deblock -> CDEF -> LR [-> film grain].
Shared by the end-to-end parity test, smoke() and bench.py's cpu_baseline leg."""
import numpy as np

from tests import oracle_lib
from tests.test_oracle_lf import pad_planes


def oracle_pipeline(fr, sb128=1):
    w, h, bpc, layout = fr["w"], fr["h"], fr["bpc"], fr["layout"]
    A = pad_planes(fr["planes"], w, h, bpc, layout)
    if fr.get("mc") is not None:
        refs = [pad_planes(r, w, h, bpc, layout) for r in fr["refs"]]
        units, _, masks = fr["mc"]
        A, _ = oracle_lib.mc_frame(A, refs, bpc, layout, w, h, units, masks)
    A = oracle_lib.itx_frame(A, fr["blocks"], fr["coef"].copy(), bpc)
    A = oracle_lib.deblock_frame(A, bpc, layout, w, h, fr["lf"], sb128=sb128)
    B = oracle_lib.cdef_frame(A, bpc, layout, w, h, fr["lf"]["masks"], fr["cdef"])
    O = oracle_lib.lr_frame(B, A, bpc, layout, w, h, dict(fr["lr"], sb128=sb128))
    G = oracle_lib.film_grain(O, bpc, layout, w, h, fr["fg"]) if fr["fg"] else O
    return dict(recon_deblocked=A, cdef=B, lr=O, out=G)


class _BenchJob(__import__("ctypes").Structure):
    """oracle/cpu_bench.c OracleBenchJob."""
    import ctypes as _c
    _fields_ = [("w", _c.c_int), ("h", _c.c_int), ("bpc", _c.c_int), ("layout", _c.c_int),
                ("strides", _c.c_ssize_t * 3), ("plane_bytes", _c.c_size_t * 3),
                ("refs", (_c.c_void_p * 3) * 2), ("nrefs", _c.c_int),
                ("units", _c.c_void_p), ("n_units", _c.c_int), ("masks", _c.c_void_p), ("masks_bytes", _c.c_size_t),
                ("tx", _c.c_void_p), ("n_tx", _c.c_int), ("coef", _c.c_void_p), ("coef_bytes", _c.c_size_t),
                ("lf_level", _c.c_void_p), ("b4_stride", _c.c_ssize_t), ("lf_masks", _c.c_void_p), ("sb128w", _c.c_int),
                ("lim_e", _c.c_void_p), ("lim_i", _c.c_void_p), ("filter_y", _c.c_int), ("filter_uv", _c.c_int),
                ("cdef_damping", _c.c_int), ("cdef_y", _c.c_void_p), ("cdef_uv", _c.c_void_p),
                ("restore_planes", _c.c_int), ("unit_size_log2", _c.c_int * 2), ("lr_mask", _c.c_void_p),
                ("lr_sb128w", _c.c_int)]


def oracle_bench(fr, threads, frames):
    """Wall seconds for `threads` C threads each running `frames` whole frames of `fr` through the
    oracle pipeline (oracle/cpu_bench.c: no Python inside the timed loop)."""
    import ctypes
    o = oracle_lib.load_oracle()
    o.oracle_bench_frames.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    o.oracle_bench_frames.restype = ctypes.c_double
    w, h, bpc, layout = fr["w"], fr["h"], fr["bpc"], fr["layout"]
    keep = []
    P = lambda a: (keep.append(a), a.ctypes.data)[1]  # noqa: E731
    j = _BenchJob()
    j.w, j.h, j.bpc, j.layout = w, h, bpc, layout
    planes0 = pad_planes(fr["planes"], w, h, bpc, layout)
    for p in range(3):
        a = planes0[min(p, len(planes0) - 1)]
        j.strides[p] = a.strides[0]
        j.plane_bytes[p] = a.nbytes
    if fr.get("mc") is not None:
        refs = [pad_planes(r, w, h, bpc, layout) for r in fr["refs"]]
        j.nrefs = len(refs)
        for r, planes in enumerate(refs):
            for p in range(3):
                j.refs[r][p] = P(planes[min(p, len(planes) - 1)])
        units, _, masks = fr["mc"]
        units = np.ascontiguousarray(units)
        masks = np.ascontiguousarray(masks)
        j.units, j.n_units = P(units), len(units)
        j.masks, j.masks_bytes = P(masks), masks.nbytes
    else:
        m = np.zeros(1, np.uint8)
        j.masks, j.masks_bytes = P(m), 1
    tx = np.ascontiguousarray(fr["blocks"])
    coef = np.ascontiguousarray(fr["coef"])
    j.tx, j.n_tx, j.coef, j.coef_bytes = P(tx), len(tx), P(coef), coef.nbytes
    lf = fr["lf"]
    j.lf_level, j.b4_stride = P(np.ascontiguousarray(lf["level"])), lf["b4_stride"]
    lfm = np.ascontiguousarray(lf["masks"])
    j.lf_masks, j.sb128w = P(lfm), lf["sb128w"]
    j.lim_e, j.lim_i = P(np.ascontiguousarray(lf["lim_e"], np.uint8)), P(np.ascontiguousarray(lf["lim_i"], np.uint8))
    j.filter_y, j.filter_uv = lf["filter_y"], lf["filter_uv"]
    cd = fr["cdef"]
    j.cdef_damping = cd["damping"]
    j.cdef_y = P(np.ascontiguousarray(cd["y_strength"], np.uint8))
    j.cdef_uv = P(np.ascontiguousarray(cd["uv_strength"], np.uint8))
    lr = fr["lr"]
    j.restore_planes = lr["restore_planes"]
    j.unit_size_log2[0], j.unit_size_log2[1] = [int(v) for v in lr["unit_size_log2"]]
    lrm = np.ascontiguousarray(lr["lr_mask"])
    j.lr_mask, j.lr_sb128w = P(lrm), lrm.shape[1]
    t = o.oracle_bench_frames(ctypes.byref(j), threads, frames)
    if t <= 0:
        raise RuntimeError("oracle_bench_frames failed")
    return t
