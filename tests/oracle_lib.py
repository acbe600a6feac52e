"""ctypes binding of oracle/liboracle.so — the CPU restatement used as the parity checker.

TEST INFRASTRUCTURE ONLY (see oracle/oracle.h). Builds the oracle with make if needed.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

_o = None
_VP = ctypes.c_void_p


def load_oracle():
    global _o
    if _o is not None:
        return _o
    srcs = [f for f in os.listdir(ORACLE_DIR) if f.endswith((".c", ".h"))]
    if not os.path.exists(ORACLE_SO) or any(
            os.path.getmtime(os.path.join(ORACLE_DIR, f)) > os.path.getmtime(ORACLE_SO) for f in srcs):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    o = ctypes.CDLL(ORACLE_SO)
    o.oracle_itxfm_add.argtypes = [ctypes.c_int, ctypes.c_int, _VP, ctypes.c_ssize_t, _VP, ctypes.c_int, ctypes.c_int]
    o.oracle_itxfm_add.restype = None
    o.oracle_itx_frame.argtypes = [_VP, _VP, _VP, ctypes.c_int, _VP, ctypes.c_int]
    o.oracle_itx_frame.restype = None
    o.oracle_itx_1d.argtypes = [ctypes.c_int, ctypes.c_int, _VP, ctypes.c_ssize_t, ctypes.c_int, ctypes.c_int]
    o.oracle_itx_1d.restype = None
    _o = o
    return o


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def itx_1d(kind, n, vec, lo=-(1 << 20), hi=(1 << 20) - 1):
    c = np.ascontiguousarray(vec, dtype=np.int32).copy()
    load_oracle().oracle_itx_1d(kind, n, ptr(c), 1, lo, hi)
    return c


def itx_frame(planes, blocks, coef, bpc):
    """Run the oracle over numpy planes (list of 2-D arrays, modified in place) and arena."""
    o = load_oracle()
    arrs = [np.ascontiguousarray(p) for p in planes]
    while len(arrs) < 3:
        arrs.append(arrs[0])
    pp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in arrs])
    st = (ctypes.c_ssize_t * 3)(*[a.strides[0] for a in arrs])
    b = np.ascontiguousarray(blocks)
    o.oracle_itx_frame(pp, st, ptr(b), len(b), ptr(coef), (1 << bpc) - 1)
    return arrs[:len(planes)]


def deblock_frame(planes, bpc, layout, w, h, lf, sb128=1):
    """Oracle whole-frame deblock in the reference's sbrow order; planes modified in place."""
    o = load_oracle()
    f = o.oracle_deblock_frame
    f.restype = None
    f.argtypes = [_VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _VP,
                  ctypes.c_ssize_t, _VP, ctypes.c_int, ctypes.c_int, _VP, _VP, ctypes.c_int, ctypes.c_int]
    arrs = [np.ascontiguousarray(p) for p in planes]
    while len(arrs) < 3:
        arrs.append(arrs[0])
    pp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in arrs])
    st = (ctypes.c_ssize_t * 3)(*[a.strides[0] for a in arrs])
    level = np.ascontiguousarray(lf["level"])
    masks = np.ascontiguousarray(lf["masks"])
    e = np.ascontiguousarray(lf["lim_e"]); i = np.ascontiguousarray(lf["lim_i"])
    f(pp, st, w, h, layout, bpc, ptr(level), lf["b4_stride"], ptr(masks), lf["sb128w"], sb128,
      ptr(e), ptr(i), lf["filter_y"], lf["filter_uv"])
    return arrs[:len(planes)]


def cdef_frame(src_planes, bpc, layout, w, h, masks, cdef):
    """Oracle whole-frame CDEF: returns new planes (src untouched). Planes must be 128-aligned."""
    o = load_oracle()
    f = o.oracle_cdef_frame
    f.restype = None
    f.argtypes = [_VP, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _VP,
                  ctypes.c_int, ctypes.c_int, _VP, _VP]
    srcs = [np.ascontiguousarray(p) for p in src_planes]
    dsts = [np.zeros_like(p) for p in srcs]
    while len(srcs) < 3:
        srcs.append(srcs[0]); dsts.append(dsts[0])
    sp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in srcs])
    dp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in dsts])
    st = (ctypes.c_ssize_t * 3)(*[a.strides[0] for a in srcs])
    m = np.ascontiguousarray(masks)
    ys = np.ascontiguousarray(cdef["y_strength"], np.uint8)
    uvs = np.ascontiguousarray(cdef["uv_strength"], np.uint8)
    f(dp, sp, st, w, h, layout, bpc, ptr(m), m.shape[1], cdef["damping"], ptr(ys), ptr(uvs))
    return dsts[:len(src_planes)]


def lr_frame(cdef_planes, deblocked_planes, bpc, layout, w, h, lr):
    """Oracle whole-frame loop restoration (in-place reference algorithm on a copy)."""
    o = load_oracle()
    f = o.oracle_lr_frame
    f.restype = None
    f.argtypes = [_VP, _VP, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int, ctypes.c_int, _VP, _VP, ctypes.c_int]
    c = [np.ascontiguousarray(p) for p in cdef_planes]
    d = [np.ascontiguousarray(p) for p in deblocked_planes]
    o_ = [np.zeros_like(p) for p in c]
    while len(c) < 3:
        c.append(c[0]); d.append(d[0]); o_.append(o_[0])
    arr = lambda L: (ctypes.c_void_p * 3)(*[a.ctypes.data for a in L])
    st = (ctypes.c_ssize_t * 3)(*[a.strides[0] for a in c])
    ul = np.array(lr["unit_size_log2"], np.int32)
    m = np.ascontiguousarray(lr["lr_mask"])
    f(arr(o_), arr(c), arr(d), st, w, h, layout, bpc, lr["sb128"], lr["restore_planes"], ptr(ul),
      ptr(m), m.shape[1])
    return o_[:len(cdef_planes)]


def film_grain(in_planes, bpc, layout, w, h, fg, is_id=0):
    """Oracle rav1d_apply_grain: returns output planes (input untouched). 128-aligned planes."""
    from rav1d_amd.frame import film_grain_data
    o = load_oracle()
    f = o.oracle_fg_apply
    f.restype = None
    f.argtypes = [_VP, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _VP, ctypes.c_int]
    src = [np.ascontiguousarray(p) for p in in_planes]
    dst = [np.zeros_like(p) for p in src]
    while len(src) < 3:
        src.append(src[0]); dst.append(dst[0])
    arr = lambda L: (ctypes.c_void_p * 3)(*[a.ctypes.data for a in L])
    st = (ctypes.c_ssize_t * 3)(*[a.strides[0] for a in src])
    d = film_grain_data(fg)
    f(arr(dst), arr(src), st, w, h, layout, bpc, ctypes.byref(d), is_id)
    return dst[:len(in_planes)]


def fg_grain_y(fg, bpc):
    from rav1d_amd.frame import film_grain_data
    o = load_oracle()
    o.oracle_fg_generate_grain_y.restype = None
    o.oracle_fg_generate_grain_y.argtypes = [_VP, _VP, ctypes.c_int]
    buf = np.zeros((73, 82), np.int16)
    d = film_grain_data(fg)
    o.oracle_fg_generate_grain_y(ptr(buf), ctypes.byref(d), (1 << bpc) - 1)
    return buf


def _mc_sigs(o):
    if getattr(o, "_mc_ready", False):
        return
    o.oracle_mc_frame.argtypes = [_VP, _VP, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP, _VP, ctypes.c_int, _VP, _VP]
    o.oracle_mc_frame.restype = None
    o.oracle_mc_scaled_frame.argtypes = [_VP, _VP] + [ctypes.c_int] * 4 + [_VP, _VP, _VP, _VP, ctypes.c_int, _VP]
    o.oracle_mc_warp_frame.argtypes = [_VP, _VP, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP, _VP, ctypes.c_int, _VP]
    o.oracle_mc_combine_frame.argtypes = [_VP, _VP, ctypes.c_int, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP]
    o.oracle_superres_frame.argtypes = [_VP, _VP, _VP, _VP] + [ctypes.c_int] * 5
    o.oracle_mc_blend.argtypes = [_VP, ctypes.c_ssize_t, _VP, ctypes.c_int, ctypes.c_int, _VP, ctypes.c_int]
    for n in ("oracle_mc_scaled_frame", "oracle_mc_warp_frame", "oracle_mc_combine_frame", "oracle_superres_frame",
              "oracle_mc_blend"):
        getattr(o, n).restype = None
    o.oracle_mc_put.argtypes = [ctypes.c_int, _VP, ctypes.c_ssize_t, _VP, ctypes.c_ssize_t] + [ctypes.c_int] * 5
    o.oracle_mc_prep.argtypes = [ctypes.c_int, _VP, _VP, ctypes.c_ssize_t] + [ctypes.c_int] * 5
    o.oracle_mc_emu_edge.argtypes = [ctypes.c_int] * 6 + [_VP, ctypes.c_ssize_t, _VP, ctypes.c_ssize_t, ctypes.c_int]
    o.oracle_mc_avg.argtypes = [_VP, ctypes.c_ssize_t, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    o.oracle_mc_w_mask.argtypes = [_VP, ctypes.c_ssize_t, _VP, _VP] + [ctypes.c_int] * 2 + [_VP] + [ctypes.c_int] * 4
    for n in ("oracle_mc_put", "oracle_mc_prep", "oracle_mc_emu_edge", "oracle_mc_avg", "oracle_mc_w_mask"):
        getattr(o, n).restype = None
    o._mc_ready = True


class _McFrameArgs:
    """ctypes views of padded current / reference planes for the oracle's MC frame drivers."""

    def __init__(self, cur_planes, ref_frames, ref_wh):
        self.cur = [np.ascontiguousarray(p).copy() for p in cur_planes]
        while len(self.cur) < 3:
            self.cur.append(self.cur[0])
        self.refs = [[np.ascontiguousarray(p) for p in f] for f in ref_frames]
        for f in self.refs:
            while len(f) < 3:
                f.append(f[0])
        self.cp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in self.cur])
        self.cs = (ctypes.c_ssize_t * 2)(self.cur[0].strides[0], self.cur[1].strides[0])
        refs = self.refs
        self.rp = (ctypes.c_void_p * max(1, 3 * len(refs)))(*[a.ctypes.data for f in refs for a in f])
        self.rs = (ctypes.c_ssize_t * max(1, 2 * len(refs)))(*[s for f in refs for s in (f[0].strides[0], f[1].strides[0])])
        self.rwh = (ctypes.c_int * max(1, 2 * len(refs)))(*[v for wh in ref_wh for v in wh])


def mc_frame(cur_planes, ref_frames, bpc, layout, w, h, units, masks, tmp=None):
    """Oracle frame MC. cur_planes: padded planes (modified copies returned); ref_frames: list
    of padded plane lists; units: MCBLOCK_DTYPE array (luma first); masks: uint8 buffer; tmp:
    int16 arena for MI_MC_PREP units (modified copy returned as the third value if given)."""
    o = load_oracle()
    _mc_sigs(o)
    fa = _McFrameArgs(cur_planes, ref_frames, [(w, h)] * len(ref_frames))
    u = np.ascontiguousarray(units)
    m = np.ascontiguousarray(masks).copy()
    t = np.zeros(1, np.int16) if tmp is None else np.ascontiguousarray(tmp, dtype=np.int16).copy()
    o.oracle_mc_frame(fa.cp, fa.cs, layout, bpc, fa.rp, fa.rs, fa.rwh, ptr(u), len(u), ptr(m), ptr(t))
    n = 3 if layout else 1
    if tmp is None:
        return fa.cur[:n], m
    return fa.cur[:n], m, t


def mc_scaled_frame(cur_planes, ref_frames, ref_wh, bpc, layout, w, h, units, tmp):
    o = load_oracle()
    _mc_sigs(o)
    fa = _McFrameArgs(cur_planes, ref_frames, ref_wh)
    u = np.ascontiguousarray(units)
    t = np.ascontiguousarray(tmp, dtype=np.int16).copy()
    o.oracle_mc_scaled_frame(fa.cp, fa.cs, layout, bpc, w, h, fa.rp, fa.rs, fa.rwh, ptr(u), len(u), ptr(t))
    return fa.cur[:3 if layout else 1], t


def mc_warp_frame(cur_planes, ref_frames, bpc, layout, w, h, blocks, tmp):
    o = load_oracle()
    _mc_sigs(o)
    fa = _McFrameArgs(cur_planes, ref_frames, [(w, h)] * len(ref_frames))
    b = np.ascontiguousarray(blocks)
    t = np.ascontiguousarray(tmp, dtype=np.int16).copy()
    o.oracle_mc_warp_frame(fa.cp, fa.cs, layout, bpc, fa.rp, fa.rs, fa.rwh, ptr(b), len(b), ptr(t))
    return fa.cur[:3 if layout else 1], t


def mc_combine_frame(cur_planes, bpc, layout, units, tmp, masks):
    o = load_oracle()
    _mc_sigs(o)
    fa = _McFrameArgs(cur_planes, [], [])
    u = np.ascontiguousarray(units)
    t = np.ascontiguousarray(tmp, dtype=np.int16)
    m = np.ascontiguousarray(masks).copy()
    o.oracle_mc_combine_frame(fa.cp, fa.cs, layout, bpc, ptr(u), len(u), ptr(t), ptr(m))
    return fa.cur[:3 if layout else 1], m


def superres_frame(src_planes, dst_planes, bpc, layout, src_w, dst_w, h):
    o = load_oracle()
    _mc_sigs(o)
    src = [np.ascontiguousarray(p) for p in src_planes]
    dst = [np.ascontiguousarray(p).copy() for p in dst_planes]
    while len(src) < 3:
        src.append(src[0])
        dst.append(dst[0])
    sp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in src])
    ss = (ctypes.c_ssize_t * 2)(src[0].strides[0], src[1].strides[0])
    dp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in dst])
    dss = (ctypes.c_ssize_t * 2)(dst[0].strides[0], dst[1].strides[0])
    o.oracle_superres_frame(sp, ss, dp, dss, layout, bpc, src_w, dst_w, h)
    return dst[:3 if layout else 1]


def mc_blend(dst, tmp, mask, bpc):
    """mc.blend (inter-intra): dst (h, w) pixels blended with tmp under mask, in a copy."""
    o = load_oracle()
    _mc_sigs(o)
    d = np.ascontiguousarray(dst).copy()
    t = np.ascontiguousarray(tmp, dtype=d.dtype)
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    h, w = d.shape
    o.oracle_mc_blend(ptr(d), d.strides[0], ptr(t), w, h, ptr(m), bpc)
    return d


def _ipred_sigs(o):
    if getattr(o, "_ipred_ready", False):
        return
    o.oracle_intra_pred.argtypes = [ctypes.c_int, _VP, ctypes.c_ssize_t, _VP] + [ctypes.c_int] * 6
    o.oracle_cfl_pred.argtypes = [ctypes.c_int, _VP, ctypes.c_ssize_t, _VP, ctypes.c_int, ctypes.c_int, _VP,
                                  ctypes.c_int, ctypes.c_int]
    o.oracle_cfl_ac.argtypes = [_VP, _VP, ctypes.c_ssize_t] + [ctypes.c_int] * 7
    o.oracle_pal_pred.argtypes = [_VP, ctypes.c_ssize_t, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    o.oracle_intra_blocks.argtypes = [_VP, _VP, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP, _VP]
    for n in ("oracle_intra_pred", "oracle_cfl_pred", "oracle_cfl_ac", "oracle_pal_pred", "oracle_intra_blocks"):
        getattr(o, n).restype = None
    o._ipred_ready = True


def intra_pred(mode, edges, tl_index, w, h, angle, max_w, max_h, bpc):
    """Oracle intra_pred[mode] on a 1-D edge array (pixels) with topleft at tl_index."""
    o = load_oracle()
    _ipred_sigs(o)
    dt = np.uint8 if bpc == 8 else np.uint16
    e = np.ascontiguousarray(edges, dtype=dt)
    dst = np.zeros((h, w), dt)
    o.oracle_intra_pred(mode, ptr(dst), dst.strides[0], ctypes.c_void_p(e.ctypes.data + tl_index * e.itemsize),
                        w, h, angle, max_w, max_h, bpc)
    return dst


def cfl_pred(mode, edges, tl_index, w, h, ac, alpha, bpc):
    o = load_oracle()
    _ipred_sigs(o)
    dt = np.uint8 if bpc == 8 else np.uint16
    e = np.ascontiguousarray(edges, dtype=dt)
    dst = np.zeros((h, w), dt)
    a = np.ascontiguousarray(ac, dtype=np.int16)
    o.oracle_cfl_pred(mode, ptr(dst), dst.strides[0], ctypes.c_void_p(e.ctypes.data + tl_index * e.itemsize),
                      w, h, ptr(a), alpha, bpc)
    return dst


def pal_pred(pal, idx, w, h, bpc):
    o = load_oracle()
    _ipred_sigs(o)
    dt = np.uint8 if bpc == 8 else np.uint16
    p = np.ascontiguousarray(pal, dtype=dt)
    i = np.ascontiguousarray(idx, dtype=np.uint8)
    dst = np.zeros((h, w), dt)
    o.oracle_pal_pred(ptr(dst), dst.strides[0], ptr(p), ptr(i), w, h, bpc)
    return dst


def intra_blocks(planes, bpc, blocks, ac, idx, pal):
    """Oracle recon_b_intra step over MiIntraBlock records in order (edges gathered from the
    planes as they are being written). planes: padded plane buffers (copies returned)."""
    o = load_oracle()
    _ipred_sigs(o)
    pl = [np.ascontiguousarray(p).copy() for p in planes]
    while len(pl) < 3:
        pl.append(pl[0])
    pp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in pl])
    ps = (ctypes.c_ssize_t * 2)(pl[0].strides[0], pl[1].strides[0])
    b = np.ascontiguousarray(blocks)
    a_, i_, p_ = (np.ascontiguousarray(x) for x in (ac, idx, pal))
    o.oracle_intra_blocks(pp, ps, bpc, ptr(b), len(b), ptr(a_), ptr(i_), ptr(p_))
    return pl[:len(planes)]


def intra_recon(planes, bpc, blocks, tx_blocks, ac, idx, pal, coef):
    """Oracle decode-order intra reconstruction: per block prediction then its residual
    (tx_blocks[k] belongs to blocks[k]); returns (planes, arena after zeroing), copies."""
    o = load_oracle()
    _ipred_sigs(o)
    f = o.oracle_intra_recon
    f.restype = None
    f.argtypes = [_VP, _VP, ctypes.c_int, _VP, _VP, ctypes.c_int, _VP, _VP, _VP, _VP]
    pl = [np.ascontiguousarray(p).copy() for p in planes]
    while len(pl) < 3:
        pl.append(pl[0])
    pp = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in pl])
    ps = (ctypes.c_ssize_t * 2)(pl[0].strides[0], pl[1].strides[0])
    b, t = np.ascontiguousarray(blocks), np.ascontiguousarray(tx_blocks)
    assert len(b) == len(t)
    a_, i_, p_ = (np.ascontiguousarray(x) for x in (ac, idx, pal))
    c = np.ascontiguousarray(coef).copy()
    f(pp, ps, bpc, ptr(b), ptr(t), len(b), ptr(a_), ptr(i_), ptr(p_), ptr(c))
    return pl[:len(planes)], c
