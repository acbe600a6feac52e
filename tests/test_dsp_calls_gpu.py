"""GPU parity of the remaining table-compatible per-call entries (cfl_pred, pal_pred, cfl_ac,
loop_filter_sb, cdef.fb, cdef.dir) vs the oracle's per-call restatements, host buffers in
and out as a rav1d DSP-table caller would pass them. Bit-exact."""
import ctypes

import numpy as np
import pytest

from rav1d_amd import lib
from rav1d_amd.synth import calc_eih, make_texture
from tests import oracle_lib

pytestmark = pytest.mark.gpu
_VP, _SS = ctypes.c_void_p, ctypes.c_ssize_t


def _o():
    o = oracle_lib.load_oracle()
    o.oracle_cfl_ac.argtypes = [_VP, _VP, _SS] + [ctypes.c_int] * 7
    o.oracle_cfl_ac.restype = None
    o.oracle_lf_sb.argtypes = [ctypes.c_int, ctypes.c_int, _VP, _SS, _VP, _VP, _SS, _VP, _VP, ctypes.c_int,
                               ctypes.c_int]
    o.oracle_lf_sb.restype = None
    o.oracle_cdef_filter_block.argtypes = [_VP, _SS, _VP, _SS, _VP, _VP, _VP] + [ctypes.c_int] * 8
    o.oracle_cdef_filter_block.restype = None
    o.oracle_cdef_find_dir.argtypes = [_VP, _SS, _VP, ctypes.c_int]
    o.oracle_cdef_find_dir.restype = ctypes.c_int
    return o


def P(a, off=0):
    return ctypes.c_void_p(a.ctypes.data + off * a.itemsize)


def _dt(bpc):
    return np.uint8 if bpc == 8 else np.uint16


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_cfl_pred_pal_pred(gpu, bpc):
    rng = np.random.default_rng(bpc)
    bdmax = (1 << bpc) - 1
    for _ in range(60):
        w, h = (int(v) for v in rng.choice([4, 8, 16, 32], 2))
        mode = int(rng.choice([0, 3, 4, 5]))
        edges = rng.integers(0, bdmax + 1, size=2 * 64 + 1).astype(_dt(bpc))
        ac = rng.integers(-(bdmax << 3), (bdmax << 3) + 1, size=w * h).astype(np.int16)
        alpha = int(rng.integers(-16, 17))
        exp = oracle_lib.cfl_pred(mode, edges, 64, w, h, ac, alpha, bpc)
        got = np.zeros((h, w), _dt(bpc))
        assert lib().mi_dsp_cfl_pred(mode, P(got), got.strides[0], P(edges, 64), w, h, P(ac), alpha, bdmax) == 0
        assert np.array_equal(got, exp), (mode, w, h)
        w, h = (int(v) for v in rng.choice([4, 8, 16, 32, 64], 2))
        pal = rng.integers(0, bdmax + 1, size=8).astype(_dt(bpc))
        idx = rng.integers(0, 8, size=w * h).astype(np.uint8)
        exp = oracle_lib.pal_pred(pal, idx, w, h, bpc)
        got = np.zeros((h, w + 3), _dt(bpc))     # a wider destination: the stride is honoured
        assert lib().mi_dsp_pal_pred(P(got), got.strides[0], P(pal), P(idx), w, h, bdmax) == 0
        assert np.array_equal(got[:, :w], exp) and not got[:, w:].any()


@pytest.mark.parametrize("bpc", [8, 10])
@pytest.mark.parametrize("layout", [1, 2, 3])
def test_cfl_ac(gpu, bpc, layout):
    o = _o()
    rng = np.random.default_rng(layout * 3 + bpc)
    ss_hor, ss_ver = int(layout != 3), int(layout == 1)
    for _ in range(40):
        cw, ch = (int(v) for v in rng.choice([4, 8, 16, 32], 2))
        w_pad, h_pad = int(rng.integers(0, cw // 4)), int(rng.integers(0, ch // 4))
        y = rng.integers(0, 1 << bpc, size=(ch << ss_ver, (cw << ss_hor) + 5)).astype(_dt(bpc))
        exp = np.zeros(cw * ch, np.int16)
        o.oracle_cfl_ac(P(exp), P(y), y.strides[0], w_pad, h_pad, cw, ch, ss_hor, ss_ver, bpc)
        got = np.zeros(cw * ch, np.int16)
        assert lib().mi_dsp_cfl_ac(layout, P(got), P(y), y.strides[0], w_pad, h_pad, cw, ch, (1 << bpc) - 1) == 0
        assert np.array_equal(got, exp), (cw, ch, w_pad, h_pad)


@pytest.mark.parametrize("bpc", [8, 10, 12])
@pytest.mark.parametrize("cls,dir", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_loop_filter_sb(gpu, bpc, cls, dir):
    o = _o()
    rng = np.random.default_rng(bpc * 10 + cls * 2 + dir)
    bdmax = (1 << bpc) - 1
    for it in range(12):
        pic = make_texture(rng, 160, 160, bpc)
        # flat regions so that the wide filters fire
        pic[rng.random(pic.shape) < 0.3] = pic[0, 0]
        b4_stride = 48
        lvl = rng.integers(0, 64, size=(40, b4_stride, 4)).astype(np.uint8)
        lvl[rng.random(lvl.shape) < 0.15] = 0
        vm = rng.integers(0, 1 << 32, size=3, dtype=np.uint64).astype(np.uint32)
        if cls:
            vm[2] = 0
        vm[1] &= ~vm[2]
        vm[0] &= ~(vm[1] | vm[2])
        vm[0] |= rng.integers(0, 1 << 32, dtype=np.uint64).astype(np.uint32) & ~(vm[1] | vm[2])
        e, i = calc_eih(int(rng.integers(0, 8)))
        lut = np.zeros(144, np.uint8)
        lut[:64], lut[64:128] = e, i
        x0, y0 = 16, 16
        slot = 0 if cls == 0 else 2               # run start: level entry (2, 3), neighbours valid
        ref = pic.copy()
        o.oracle_lf_sb(cls, dir, P(ref, y0 * 160 + x0), ref.strides[0], P(vm),
                       ctypes.c_void_p(lvl.ctypes.data + (2 * b4_stride + 3) * 4 + slot), b4_stride,
                       P(lut), P(lut, 64), 32, bdmax)
        got = pic.copy()
        rc = lib().mi_dsp_loop_filter_sb(cls, dir, P(got, y0 * 160 + x0), got.strides[0], P(vm),
                                         ctypes.c_void_p(lvl.ctypes.data + (2 * b4_stride + 3) * 4 + slot),
                                         b4_stride, P(lut), 32, bdmax)
        assert rc == 0
        assert np.array_equal(got, ref), f"iteration {it}: {np.argwhere(got != ref)[:4]}"


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_cdef_filter_and_dir(gpu, bpc):
    o = _o()
    rng = np.random.default_rng(77 + bpc)
    bdmax = (1 << bpc) - 1
    bdm8 = bpc - 8
    for it in range(80):
        fb = int(rng.integers(0, 3))
        w, h = (8 if fb == 0 else 4), (4 if fb == 2 else 8)
        pic = make_texture(rng, 32, 32, bpc)
        x0, y0 = 8, 8
        left = np.ascontiguousarray(pic[y0:y0 + h, x0 - 2:x0])
        edges = int(rng.integers(0, 16))
        pri = int(rng.integers(0, 16)) << bdm8
        sec = int(rng.choice([0, 1, 2, 4])) << bdm8
        d = int(rng.integers(0, 8))
        damping = int(rng.integers(3, 7)) + bdm8 - (fb > 0)
        src = pic.copy()
        ref = pic.copy()
        o.oracle_cdef_filter_block(P(ref, y0 * 32 + x0), ref.strides[0], P(src, y0 * 32 + x0), src.strides[0],
                                   P(left), P(src, (y0 - 2) * 32 + x0), P(src, (y0 + h) * 32 + x0),
                                   pri, sec, d, damping, w, h, edges, bdmax)
        got = pic.copy()
        rc = lib().mi_dsp_cdef_filter(fb, P(got, y0 * 32 + x0), got.strides[0], P(left),
                                      P(src, (y0 - 2) * 32 + x0), P(src, (y0 + h) * 32 + x0),
                                      pri, sec, d, damping, edges, bdmax)
        assert rc == 0
        assert np.array_equal(got, ref), (it, fb, edges, pri, sec, d)
        var_o, var_g = ctypes.c_uint(0), ctypes.c_uint(0)
        d_o = o.oracle_cdef_find_dir(P(pic, y0 * 32 + x0), pic.strides[0], ctypes.byref(var_o), bdmax)
        d_g = lib().mi_dsp_cdef_dir(P(pic, y0 * 32 + x0), pic.strides[0], ctypes.byref(var_g), bdmax)
        assert (d_g, var_g.value) == (d_o, var_o.value)


def _mc_sigs(o):
    I = ctypes.c_int
    o.oracle_mc_put.argtypes = [I, _VP, _SS, _VP, _SS, I, I, I, I, I]
    o.oracle_mc_prep.argtypes = [I, _VP, _VP, _SS, I, I, I, I, I]
    o.oracle_mc_avg.argtypes = [_VP, _SS, _VP, _VP, I, I, I]
    o.oracle_mc_w_avg.argtypes = [_VP, _SS, _VP, _VP, I, I, I, I]
    o.oracle_mc_mask.argtypes = [_VP, _SS, _VP, _VP, I, I, _VP, I]
    o.oracle_mc_w_mask.argtypes = [_VP, _SS, _VP, _VP, I, I, _VP, I, I, I, I]
    o.oracle_mc_blend.argtypes = [_VP, _SS, _VP, I, I, _VP, I]
    o.oracle_mc_blend_v.argtypes = [_VP, _SS, _VP, I, I, I]
    o.oracle_mc_blend_h.argtypes = [_VP, _SS, _VP, I, I, I]
    o.oracle_mc_emu_edge.argtypes = [I, I, I, I, I, I, _VP, _SS, _VP, _SS, I]
    for f in ("put", "prep", "avg", "w_avg", "mask", "w_mask", "blend", "blend_v", "blend_h", "emu_edge"):
        getattr(o, "oracle_mc_" + f).restype = None
    return o


SIZES = [2, 4, 8, 16, 32, 64, 128]


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_mc_put_prep(gpu, bpc):
    o = _mc_sigs(_o())
    rng = np.random.default_rng(500 + bpc)
    bdmax = (1 << bpc) - 1
    for it in range(60):
        w, h = int(rng.choice(SIZES)), int(rng.choice(SIZES))
        f2d = int(rng.integers(0, 10))
        mx, my = int(rng.integers(0, 16)) * int(rng.random() < 0.8), int(rng.integers(0, 16)) * int(rng.random() < 0.8)
        src = make_texture(rng, 144, 144, bpc)
        off = 8 * 144 + 8
        ref = np.zeros((h, w + 2), _dt(bpc))
        got = np.zeros((h, w + 2), _dt(bpc))
        o.oracle_mc_put(f2d, P(ref), ref.strides[0], P(src, off), src.strides[0], w, h, mx, my, bpc)
        assert lib().mi_dsp_mc_put(f2d, P(got), got.strides[0], P(src, off), src.strides[0], w, h, mx, my, bdmax) == 0
        assert np.array_equal(got, ref), ("put", it, f2d, w, h, mx, my)
        rt = np.zeros(w * h, np.int16)
        gt = np.zeros(w * h, np.int16)
        o.oracle_mc_prep(f2d, P(rt), P(src, off), src.strides[0], w, h, mx, my, bpc)
        assert lib().mi_dsp_mc_prep(f2d, P(gt), P(src, off), src.strides[0], w, h, mx, my, bdmax) == 0
        assert np.array_equal(gt, rt), ("prep", it, f2d, w, h, mx, my)


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_mc_combine_blend_emu(gpu, bpc):
    o = _mc_sigs(_o())
    rng = np.random.default_rng(600 + bpc)
    bdmax = (1 << bpc) - 1
    for it in range(40):
        w, h = int(rng.choice(SIZES[1:])), int(rng.choice(SIZES[1:]))
        t = [np.zeros(w * h, np.int16) for _ in range(2)]
        for k in range(2):
            src = make_texture(rng, w + 16, h + 16, bpc)
            o.oracle_mc_prep(int(rng.integers(0, 10)), P(t[k]), P(src, 4 * (w + 16) + 4), src.strides[0], w, h,
                             int(rng.integers(0, 16)), int(rng.integers(0, 16)), bpc)
        m = rng.integers(0, 65, size=w * h).astype(np.uint8)
        weight = int(rng.integers(1, 16))
        for name in ("avg", "w_avg", "mask"):
            ref = np.zeros((h, w), _dt(bpc))
            got = np.zeros((h, w), _dt(bpc))
            extra = {"avg": [], "w_avg": [weight], "mask": [P(m)]}[name]
            getattr(o, "oracle_mc_" + name)(P(ref), ref.strides[0], P(t[0]), P(t[1]), w, h, *extra, bpc)
            assert getattr(lib(), "mi_dsp_mc_" + name)(P(got), got.strides[0], P(t[0]), P(t[1]), w, h, *extra,
                                                        bdmax) == 0
            assert np.array_equal(got, ref), (name, w, h)
        for layout, (sh, sv) in ((1, (1, 1)), (2, (1, 0)), (3, (0, 0))):
            sign = int(rng.integers(0, 2))
            ref = np.zeros((h, w), _dt(bpc))
            got = np.zeros((h, w), _dt(bpc))
            rm = np.zeros((h >> sv) * (w >> sh), np.uint8)
            gm = np.zeros_like(rm)
            o.oracle_mc_w_mask(P(ref), ref.strides[0], P(t[0]), P(t[1]), w, h, P(rm), sign, sh, sv, bpc)
            assert lib().mi_dsp_mc_w_mask(layout, P(got), got.strides[0], P(t[0]), P(t[1]), w, h, P(gm), sign,
                                          bdmax) == 0
            assert np.array_equal(got, ref) and np.array_equal(gm, rm), ("w_mask", layout, w, h)
        dst0 = make_texture(rng, w, h, bpc)
        tmp = make_texture(rng, w, h, bpc)
        for name, extra in (("blend", [P(m)]), ("blend_v", []), ("blend_h", [])):
            if name != "blend" and (w > 32 if name == "blend_v" else h > 32):
                continue
            ref, got = dst0.copy(), dst0.copy()
            getattr(o, "oracle_mc_" + name)(P(ref), ref.strides[0], P(tmp), w, h, *extra, bpc)
            assert getattr(lib(), "mi_dsp_mc_" + name)(P(got), got.strides[0], P(tmp), w, h, *extra, bdmax) == 0
            assert np.array_equal(got, ref), (name, w, h)
        # emu_edge: blocks straddling every border of a small reference
        iw, ih = int(rng.integers(8, 40)), int(rng.integers(8, 40))
        refpic = make_texture(rng, iw, ih, bpc)
        bw, bh = int(rng.integers(1, 48)), int(rng.integers(1, 48))
        x, y = int(rng.integers(-bw - 4, iw + 4)), int(rng.integers(-bh - 4, ih + 4))
        r = np.zeros((bh, bw), _dt(bpc))
        g = np.zeros((bh, bw), _dt(bpc))
        o.oracle_mc_emu_edge(bw, bh, iw, ih, x, y, P(r), r.strides[0], P(refpic), refpic.strides[0], bpc)
        assert lib().mi_dsp_mc_emu_edge(bw, bh, iw, ih, x, y, P(g), g.strides[0], P(refpic), refpic.strides[0],
                                        bdmax) == 0
        assert np.array_equal(g, r), ("emu_edge", bw, bh, iw, ih, x, y)


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_mc_warp8x8_resize(gpu, bpc):
    o = _mc_sigs(_o())
    I = ctypes.c_int
    o.oracle_mc_warp8x8.argtypes = [I, _VP, _SS, _VP, _SS, _VP, _SS, _VP, I, I, I]
    o.oracle_mc_warp8x8.restype = None
    o.oracle_mc_resize.argtypes = [_VP, _SS, _VP, _SS, I, I, I, I, I, I]
    o.oracle_mc_resize.restype = None
    rng = np.random.default_rng(700 + bpc)
    bdmax = (1 << bpc) - 1
    for it in range(50):
        src = make_texture(rng, 32, 32, bpc)
        off = 8 * 32 + 8
        abcd = rng.integers(-2000, 2001, size=4).astype(np.int16)
        mx, my = int(rng.integers(-16384, 65537)), int(rng.integers(-16384, 65537))
        ref = np.zeros((8, 8), _dt(bpc))
        got = np.zeros((8, 8), _dt(bpc))
        o.oracle_mc_warp8x8(0, P(ref), ref.strides[0], None, 0, P(src, off), src.strides[0], P(abcd), mx, my, bpc)
        assert lib().mi_dsp_mc_warp8x8(0, P(got), got.strides[0], P(src, off), src.strides[0], P(abcd), mx, my,
                                       bdmax) == 0
        assert np.array_equal(got, ref), ("warp8x8", it)
        rt = np.zeros((8, 12), np.int16)
        gt = np.zeros((8, 12), np.int16)
        o.oracle_mc_warp8x8(1, None, 0, P(rt), 12, P(src, off), src.strides[0], P(abcd), mx, my, bpc)
        assert lib().mi_dsp_mc_warp8x8(1, P(gt), 12, P(src, off), src.strides[0], P(abcd), mx, my, bdmax) == 0
        assert np.array_equal(gt, rt), ("warp8x8t", it)
        # resize: a row band upscaled as superres does (dx = step, mx0 = initial phase)
        src_w, h = int(rng.integers(16, 200)), int(rng.integers(1, 9))
        dst_w = int(src_w * rng.uniform(1.0, 2.0))
        dx = ((src_w << 14) + (dst_w >> 1)) // dst_w
        mx0 = int(rng.integers(0, 1 << 14))
        s = make_texture(rng, src_w, h, bpc)
        r = np.zeros((h, dst_w), _dt(bpc))
        g = np.zeros((h, dst_w), _dt(bpc))
        o.oracle_mc_resize(P(r), r.strides[0], P(s), s.strides[0], dst_w, h, src_w, dx, mx0, bpc)
        assert lib().mi_dsp_mc_resize(P(g), g.strides[0], P(s), s.strides[0], dst_w, h, src_w, dx, mx0, bdmax) == 0
        assert np.array_equal(g, r), ("resize", src_w, dst_w, mx0)


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_mc_scaled(gpu, bpc):
    o = _mc_sigs(_o())
    I = ctypes.c_int
    o.oracle_mc_scaled.argtypes = [I, I, _VP, _SS, _VP, _VP, _SS] + [I] * 7
    o.oracle_mc_scaled.restype = None
    rng = np.random.default_rng(800 + bpc)
    bdmax = (1 << bpc) - 1
    for it in range(60):
        w, h = int(rng.choice(SIZES[:6])), int(rng.choice(SIZES[:6]))
        f2d = int(rng.integers(0, 10))
        mx, my = int(rng.integers(0, 1024)), int(rng.integers(0, 1024))
        dx, dy = int(rng.integers(512, 2049)), int(rng.integers(512, 2049))
        src = make_texture(rng, 160, 160, bpc)
        off = 8 * 160 + 8
        for prep in (0, 1):
            if prep:
                ref, got = np.zeros(w * h, np.int16), np.zeros(w * h, np.int16)
                o.oracle_mc_scaled(f2d, 1, None, 0, P(ref), P(src, off), src.strides[0], w, h, mx, my, dx, dy, bpc)
                rc = lib().mi_dsp_mc_scaled(1, f2d, P(got), 0, P(src, off), src.strides[0], w, h, mx, my, dx, dy, bdmax)
            else:
                ref, got = np.zeros((h, w), _dt(bpc)), np.zeros((h, w), _dt(bpc))
                o.oracle_mc_scaled(f2d, 0, P(ref), ref.strides[0], None, P(src, off), src.strides[0], w, h, mx, my,
                                   dx, dy, bpc)
                rc = lib().mi_dsp_mc_scaled(0, f2d, P(got), got.strides[0], P(src, off), src.strides[0], w, h, mx, my,
                                            dx, dy, bdmax)
            assert rc == 0
            assert np.array_equal(got, ref), ("scaled", prep, f2d, w, h, mx, my, dx, dy)


_SGR = [(140, 3236), (112, 2158), (93, 1618), (80, 1438), (70, 1295), (58, 1177), (47, 1079), (37, 996),
        (30, 925), (25, 863), (0, 2589), (0, 1618), (0, 1177), (0, 925), (56, 0), (22, 0)]


def _lr_case(rng, bpc):
    """One unit at (8, 8) of a 400 x 80 picture: random size (w <= 384, h <= 64), edges, and
    left / lpf pixels independent of the picture as the reference's callers may pass them."""
    w = int(rng.choice([384, 64, 65, int(rng.integers(1, 385))]))
    h = int(rng.choice([64, int(rng.integers(1, 65))]))
    pic = make_texture(rng, 400, 80, bpc)
    left = make_texture(rng, 4, h, bpc)
    lpf = make_texture(rng, 400, 8, bpc)
    return w, h, int(rng.integers(0, 16)), pic, left, lpf


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_lr_wiener_sgr(gpu, bpc):
    o = _o()
    I = ctypes.c_int
    o.oracle_lr_wiener.argtypes = [_VP, _SS, _VP, _VP, I, I, _VP, I, I]
    o.oracle_lr_wiener.restype = None
    o.oracle_lr_sgr.argtypes = [I, _VP, _SS, _VP, _VP, I, I, ctypes.c_uint, ctypes.c_uint, I, I, I, I]
    o.oracle_lr_sgr.restype = None
    rng = np.random.default_rng(900 + bpc)
    bdmax = (1 << bpc) - 1
    off = 8 * 400 + 8
    for it in range(30):
        w, h, edges, pic, left, lpf = _lr_case(rng, bpc)
        # LooprestorationParams.filter as lr_apply builds it: symmetric taps in the AV1 ranges
        f = np.zeros((2, 8), np.int16)
        for k in range(2):
            t = [int(rng.integers(-5, 11)), int(rng.integers(-23, 9)), int(rng.integers(-17, 47))]
            c = -2 * sum(t) + (128 if (k == 1 or bpc > 8) else 0)
            f[k, :7] = [t[0], t[1], t[2], c, t[2], t[1], t[0]]
        ref, got = pic.copy(), pic.copy()
        o.oracle_lr_wiener(P(ref, off), ref.strides[0], P(left), P(lpf, 8), w, h, P(f), edges, bdmax)
        rc = lib().mi_dsp_lr_wiener(P(got, off), got.strides[0], P(left), P(lpf, 8), w, h, P(f), edges, bdmax)
        assert rc == 0
        assert np.array_equal(got, ref), ("wiener", it, w, h, edges, np.argwhere(got != ref)[:4])
    for it in range(45):
        w, h, edges, pic, left, lpf = _lr_case(rng, bpc)
        s0, s1 = _SGR[int(rng.integers(0, 16))]
        kind = (s0 != 0) + 2 * (s1 != 0) - 1
        wt0, wt1 = int(rng.integers(-96, 32)), int(rng.integers(-32, 96))
        w0, w1 = wt0, 128 - (wt0 + wt1)
        prm = np.zeros(6, np.int16)
        prm.view(np.uint32)[:2] = [s0, s1]
        prm[4:6] = [w0, w1]
        ref, got = pic.copy(), pic.copy()
        o.oracle_lr_sgr(kind, P(ref, off), ref.strides[0], P(left), P(lpf, 8), w, h, s0, s1, w0, w1, edges, bdmax)
        rc = lib().mi_dsp_lr_sgr(kind, P(got, off), got.strides[0], P(left), P(lpf, 8), w, h, P(prm), edges, bdmax)
        assert rc == 0
        assert np.array_equal(got, ref), ("sgr", kind, it, w, h, edges, np.argwhere(got != ref)[:4])


def _fg_sigs(o):
    I = ctypes.c_int
    o.oracle_fg_generate_grain_y.argtypes = [_VP, _VP, I]
    o.oracle_fg_generate_grain_y.restype = None
    o.oracle_fg_generate_grain_uv.argtypes = [_VP, _VP, _VP, I, I, I, I]
    o.oracle_fg_generate_grain_uv.restype = None
    o.oracle_fg_32x32xn.argtypes = [I, I, _VP, _VP, _SS, _VP, I, _VP, _VP, I, I, _VP, _SS, I, I]
    o.oracle_fg_32x32xn.restype = None
    return o


def _entry(bpc):
    return np.int8 if bpc == 8 else np.int16


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_fg_generate_grain(gpu, bpc):
    from rav1d_amd.frame import film_grain_data
    from rav1d_amd.synth import make_fg_params
    o = _fg_sigs(_o())
    rng = np.random.default_rng(1000 + bpc)
    bdmax = (1 << bpc) - 1
    for it in range(12):
        layout = int(rng.integers(1, 4))
        d = film_grain_data(make_fg_params(rng, layout))
        ref_y = np.zeros((73, 82), np.int16)
        o.oracle_fg_generate_grain_y(P(ref_y), ctypes.byref(d), bdmax)
        got_y = np.zeros((74, 82), _entry(bpc))
        assert lib().mi_dsp_fg_generate_grain_y(P(got_y), ctypes.byref(d), bdmax) == 0
        assert np.array_equal(got_y[:73].astype(np.int16), ref_y), ("y", it)
        sx, sy = int(layout != 3), int(layout == 1)
        for uv in (0, 1):
            fill = int(rng.integers(-100, 100))
            ref = np.full((74, 82), fill, np.int16)
            o.oracle_fg_generate_grain_uv(P(ref), P(ref_y), ctypes.byref(d), uv, sx, sy, bdmax)
            got = np.full((74, 82), fill, _entry(bpc))
            assert lib().mi_dsp_fg_generate_grain_uv(layout, P(got), P(got_y), ctypes.byref(d), uv, bdmax) == 0
            assert np.array_equal(got.astype(np.int16), ref), ("uv", it, layout, uv)


@pytest.mark.parametrize("bpc", [8, 10, 12])
def test_fg_32x32xn(gpu, bpc):
    from rav1d_amd.frame import film_grain_data
    from rav1d_amd.synth import make_fg_params
    o = _fg_sigs(_o())
    rng = np.random.default_rng(1100 + bpc)
    bdmax = (1 << bpc) - 1
    gctr = 128 << (bpc - 8)
    for it in range(40):
        layout = int(rng.integers(1, 4))
        pl = int(rng.integers(0, 3))
        sx, sy = (int(layout != 3), int(layout == 1)) if pl else (0, 0)
        d = film_grain_data(make_fg_params(rng, layout))
        pw = int(rng.choice([int(rng.integers(1, 300)), 1000, 32 >> sx, (32 >> sx) + 1]))
        bh = int(rng.integers(1, (32 >> sy) + 1))
        row_num = int(rng.integers(0, 6))
        is_id = int(rng.integers(0, 2))
        W = (pw + 63) // 32 * 32
        src = make_texture(rng, W, bh, bpc)
        luma = make_texture(rng, 2 * W, bh << sy, bpc)
        lut = rng.integers(-gctr, gctr, size=(74, 82)).astype(np.int16)
        scl = rng.integers(0, 256, size=1 << bpc).astype(np.uint8)
        ref = np.zeros_like(src)
        o.oracle_fg_32x32xn(pl, layout, P(ref), P(src), src.strides[0], ctypes.byref(d), pw, P(scl), P(lut), bh,
                            row_num, P(luma), luma.strides[0], is_id, bdmax)
        got = np.zeros_like(src)
        glut = lut.astype(_entry(bpc))
        if pl == 0:
            rc = lib().mi_dsp_fgy_32x32xn(P(got), P(src), src.strides[0], ctypes.byref(d), pw, P(scl), P(glut), bh,
                                          row_num, bdmax)
        else:
            rc = lib().mi_dsp_fguv_32x32xn(layout, P(got), P(src), src.strides[0], ctypes.byref(d), pw, P(scl),
                                           P(glut), bh, row_num, P(luma), luma.strides[0], pl - 1, is_id, bdmax)
        assert rc == 0
        assert np.array_equal(got[:, :pw], ref[:, :pw]), ("fg", it, pl, layout, pw, bh, row_num,
                                                           np.argwhere(got[:, :pw] != ref[:, :pw])[:4])
