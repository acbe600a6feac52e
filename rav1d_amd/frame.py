"""Device-resident pictures and the batched per-frame calls.

Pictures follow dav1d's default allocator layout (rav1d src/picture.rs:98-115): width and
height aligned to 128, a luma stride of the aligned row bytes (+64 B when it is a multiple
of 1024, to break cache-set aliasing), chroma planes subsampled per layout. Each plane is a
torch uint8 tensor of shape (rows, stride_bytes) on the device; 16-bit pictures are the same
bytes viewed as little-endian uint16. torch is only the allocator/stream provider here.
"""
import ctypes

import numpy as np
import torch

from . import MC_NCLASS, MiCdef, MiFilmGrainData, MiLoopFilter, MiLr, MiPicture, MiError, check, lib

LAYOUT_I400, LAYOUT_I420, LAYOUT_I422, LAYOUT_I444 = 0, 1, 2, 3


def _align(v, a):
    return (v + a - 1) // a * a


def plane_geometry(w, h, layout, bpc):
    """(luma (rows, stride), chroma (rows, stride), chroma (w, h)) in bytes, as the reference."""
    pxb = 1 if bpc == 8 else 2
    aw, ah = _align(w, 128), _align(h, 128)
    ss_hor = layout in (LAYOUT_I420, LAYOUT_I422)
    ss_ver = layout == LAYOUT_I420
    y_stride = aw * pxb
    if y_stride % 1024 == 0:
        y_stride += 64
    uv_stride = (aw >> ss_hor) * pxb
    if uv_stride % 1024 == 0:
        uv_stride += 64
    cw, ch = (w + ss_hor) >> ss_hor, (h + ss_ver) >> ss_ver
    return (ah, y_stride), (ah >> ss_ver, uv_stride), (cw, ch)


class Frame:
    """A picture whose three planes live in device (or host) memory."""

    def __init__(self, w, h, bpc=10, layout=LAYOUT_I420, device="cuda"):
        self.w, self.h, self.bpc, self.layout = w, h, bpc, layout
        (yr, ys), (cr, cs), (cw, ch) = plane_geometry(w, h, layout, bpc)
        self.cw, self.ch = cw, ch
        self.pxb = 1 if bpc == 8 else 2
        self.strides = [ys, cs, cs]
        rows = [yr, cr, cr]
        n = 1 if layout == LAYOUT_I400 else 3
        self.planes = [torch.zeros((rows[p], self.strides[p]), dtype=torch.uint8, device=device)
                       for p in range(n)]

    def dims(self, p):
        return (self.w, self.h) if p == 0 else (self.cw, self.ch)

    def picture(self):
        pic = MiPicture()
        for p in range(3):
            pic.data[p] = self.planes[min(p, len(self.planes) - 1)].data_ptr()
        pic.stride[0], pic.stride[1] = self.strides[0], self.strides[1]
        pic.w, pic.h, pic.layout, pic.bpc = self.w, self.h, self.layout, self.bpc
        return pic

    # numpy views (copies across the device boundary)
    def buffer_np(self, p):
        """The whole allocated plane (aligned rows x stride) as pixels."""
        b = self.planes[p].cpu().numpy()
        return b.view("<u2").copy() if self.pxb == 2 else b.copy()

    def set_buffer_np(self, p, arr):
        a = np.ascontiguousarray(arr, dtype=np.uint16 if self.pxb == 2 else np.uint8)
        self.planes[p].copy_(torch.from_numpy(a.view(np.uint8).reshape(self.planes[p].shape)))

    def plane_np(self, p):
        b = self.planes[p].cpu().numpy()
        w, h = self.dims(p)
        if self.pxb == 2:
            return b.view("<u2")[:h, :w].copy()
        return b[:h, :w].copy()

    def set_plane_np(self, p, arr):
        w, h = self.dims(p)
        dt = np.uint16 if self.pxb == 2 else np.uint8
        host = self.planes[p].cpu().numpy().copy()
        view = host.view("<u2") if self.pxb == 2 else host
        view[:h, :w] = np.asarray(arr, dtype=dt)[:h, :w]
        self.planes[p].copy_(torch.from_numpy(host))

    def raw_np(self, p):
        """Whole plane including padding, as bytes (rows, stride)."""
        return self.planes[p].cpu().numpy()

    def clone(self):
        f = Frame.__new__(Frame)
        f.__dict__.update(self.__dict__)
        f.planes = [t.clone() for t in self.planes]
        return f


class Context:
    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().mi_ctx_create(device, ctypes.byref(h)), "mi_ctx_create")
        self.h = h

    def close(self):
        if self.h:
            lib().mi_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _stream_ptr(stream):
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def itx_frame(ctx, frame, blocks_dev, size_start, coef_dev, flags=0, stream=None, band_start=None, dc_end=None):
    """mi_itx_frame: inverse transform + add for all blocks of a frame (device tensors).
    band_start ([19][9], synth.itx_band_order): the blocks are also grouped by picture band
    and run through mi_itx_frame_banded (one XCD per band); with dc_end ([19][8],
    synth.itx_dc_runs) through mi_itx_frame_runs (each band's leading DC-only run on the DC path)."""
    pic = frame.picture()
    if blocks_dev.dtype != torch.uint8 or not blocks_dev.is_cuda:
        raise MiError("blocks must be a device uint8 tensor holding MiTxBlock records")
    if band_start is not None and dc_end is not None:
        bs = (ctypes.c_uint32 * (19 * 9))(*[int(v) for v in np.asarray(band_start).reshape(-1)])
        de = (ctypes.c_uint32 * (19 * 8))(*[int(v) for v in np.asarray(dc_end).reshape(-1)])
        rc = lib().mi_itx_frame_runs(ctx.h, ctypes.byref(pic), ctypes.c_void_p(blocks_dev.data_ptr()), bs, de,
                                     ctypes.c_void_p(coef_dev.data_ptr()), flags, _stream_ptr(stream))
        check(rc, "mi_itx_frame_runs")
        return
    if band_start is not None:
        bs = (ctypes.c_uint32 * (19 * 9))(*[int(v) for v in np.asarray(band_start).reshape(-1)])
        rc = lib().mi_itx_frame_banded(ctx.h, ctypes.byref(pic), ctypes.c_void_p(blocks_dev.data_ptr()), bs,
                                       ctypes.c_void_p(coef_dev.data_ptr()), flags, _stream_ptr(stream))
        check(rc, "mi_itx_frame_banded")
        return
    ss = (ctypes.c_uint32 * 20)(*[int(v) for v in size_start])
    rc = lib().mi_itx_frame(ctx.h, ctypes.byref(pic), ctypes.c_void_p(blocks_dev.data_ptr()), ss,
                            ctypes.c_void_p(coef_dev.data_ptr()), flags, _stream_ptr(stream))
    check(rc, "mi_itx_frame")


class McMeta:
    """Device copies of a frame's MC units (MiMcBlock, bucketed by plane group and shape
    class; see mc_sort_units) and mask buffer."""

    def __init__(self, units, class_start, masks):
        self.n = len(units)
        # no chroma MASK unit (which may read a mask a SEG luma unit of the call writes): both
        # plane groups can run in one grid (mi_mc_frame_ex, MI_MC_ONE_GRID)
        self.one_grid = not bool(((units["plane"] > 0) & (units["ref"][:, 1] >= 0) & (units["comp"] == 2)).any())
        self.blocks = torch.from_numpy(np.ascontiguousarray(units).view(np.uint8).copy()).cuda()
        self.masks = torch.from_numpy(np.ascontiguousarray(masks).copy()).cuda()
        self.class_start = (ctypes.c_uint32 * (2 * MC_NCLASS + 1))(*[int(v) for v in class_start])


class McSplitMeta:
    """A frame's MC units split for mi_mc_frame_ex(MI_MC_ONE_GRID) (synth.mc_split_one_grid):
    `a` runs luma and most chroma in one grid, `b` the chroma MASK units after it; both use
    one device mask buffer."""

    def __init__(self, units, masks):
        from .synth import mc_split_one_grid
        ua, ca, ub, cb = mc_split_one_grid(units)
        self.n = len(units)
        self.a = McMeta(ua, ca, masks)
        self.b = McMeta(ub, cb, masks[:0])
        self.masks = self.b.masks = self.a.masks


def mc_frame_one_grid(ctx, cur, refs, split, stream=None, tmp=None):
    """mi_mc_frame_ex(MI_MC_ONE_GRID) over split.a, then mi_mc_frame over split.b."""
    pics = (MiPicture * len(refs))(*[r.picture() for r in refs])
    L, pc, sp = lib(), ctypes.byref(cur.picture()), _stream_ptr(stream)
    check(L.mi_mc_frame_ex(ctx.h, pc, pics, len(refs), ctypes.c_void_p(split.a.blocks.data_ptr()),
                           split.a.class_start, ctypes.c_void_p(split.masks.data_ptr()), _dptr(tmp),
                           MI_MC_ONE_GRID, sp), "mi_mc_frame_ex")
    if split.b.n:
        check(L.mi_mc_frame(ctx.h, pc, pics, len(refs), ctypes.c_void_p(split.b.blocks.data_ptr()),
                            split.b.class_start, ctypes.c_void_p(split.masks.data_ptr()), _dptr(tmp), sp),
              "mi_mc_frame")


MI_MC_ONE_GRID = 1


def mc_frame_sync(ctx, cur, refs, meta, stream=None, tmp=None):
    """mi_mc_frame_sync: one grid; chroma units flagged MI_MC_AFTER_SEG wait inside the launch
    for the SEG unit that writes their mask."""
    pics = (MiPicture * len(refs))(*[r.picture() for r in refs])
    check(lib().mi_mc_frame_sync(ctx.h, ctypes.byref(cur.picture()), pics, len(refs),
                                 ctypes.c_void_p(meta.blocks.data_ptr()), meta.class_start,
                                 ctypes.c_void_p(meta.masks.data_ptr()), meta.masks.numel(), _dptr(tmp),
                                 _stream_ptr(stream)), "mi_mc_frame_sync")


def _dptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def mc_frame(ctx, cur, refs, meta, stream=None, tmp=None):
    """mi_mc_frame: inter prediction of every unit into `cur` from the reference Frames.
    tmp: optional int16 device tensor (arena for MI_MC_PREP units)."""
    pics = (MiPicture * len(refs))(*[r.picture() for r in refs])
    rc = lib().mi_mc_frame_ex(ctx.h, ctypes.byref(cur.picture()), pics, len(refs),
                              ctypes.c_void_p(meta.blocks.data_ptr()), meta.class_start,
                              ctypes.c_void_p(meta.masks.data_ptr()), _dptr(tmp),
                              MI_MC_ONE_GRID if meta.one_grid else 0, _stream_ptr(stream))
    check(rc, "mi_mc_frame_ex")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


def mc_scaled(ctx, cur, refs, units, tmp, stream=None):
    """mi_mc_scaled over MiMcBlock units (numpy) whose references differ in size from cur."""
    pics = (MiPicture * len(refs))(*[r.picture() for r in refs])
    u = _dev(units)
    check(lib().mi_mc_scaled(ctx.h, ctypes.byref(cur.picture()), pics, len(refs), ctypes.c_void_p(u.data_ptr()),
                             len(units), _dptr(tmp), _stream_ptr(stream)), "mi_mc_scaled")
    return u


def mc_warp(ctx, cur, refs, blocks, tmp, stream=None):
    pics = (MiPicture * len(refs))(*[r.picture() for r in refs])
    b = _dev(blocks)
    check(lib().mi_mc_warp(ctx.h, ctypes.byref(cur.picture()), pics, len(refs), ctypes.c_void_p(b.data_ptr()),
                           len(blocks), _dptr(tmp), _stream_ptr(stream)), "mi_mc_warp")
    return b


def mc_combine(ctx, cur, units, tmp, masks, stream=None):
    u = _dev(units)
    check(lib().mi_mc_combine(ctx.h, ctypes.byref(cur.picture()), ctypes.c_void_p(u.data_ptr()), len(units),
                              _dptr(tmp), _dptr(masks), _stream_ptr(stream)), "mi_mc_combine")
    return u


def superres_frame(ctx, src, dst, stream=None):
    check(lib().mi_superres_frame(ctx.h, ctypes.byref(src.picture()), ctypes.byref(dst.picture()),
                                  _stream_ptr(stream)), "mi_superres_frame")


class LoopFilterMeta:
    """Device copies of the deblocking inputs (MiLoopFilter)."""

    def __init__(self, lf):
        self.level = torch.from_numpy(np.ascontiguousarray(lf["level"]).reshape(-1)).cuda()
        self.masks = torch.from_numpy(np.ascontiguousarray(lf["masks"]).view(np.uint8).reshape(-1)).cuda()
        s = MiLoopFilter()
        s.level = self.level.data_ptr()
        s.b4_stride = int(lf["b4_stride"])
        s.masks = self.masks.data_ptr()
        s.sb128w = int(lf["sb128w"])
        s.filter_y = int(lf["filter_y"])
        s.filter_uv = int(lf["filter_uv"])
        s.lim_e[:] = [int(v) for v in lf["lim_e"]]
        s.lim_i[:] = [int(v) for v in lf["lim_i"]]
        self.s = s


def deblock_frame(ctx, frame, meta, stream=None, dst=None):
    """In place (two launches: column edges, row edges) or, with `dst`, out of place (one
    fused launch of 64x64 tiles)."""
    pic = frame.picture()
    if dst is None:
        check(lib().mi_deblock_frame(ctx.h, ctypes.byref(pic), ctypes.byref(meta.s), _stream_ptr(stream)),
              "mi_deblock_frame")
    else:
        check(lib().mi_deblock_frame_to(ctx.h, ctypes.byref(pic), ctypes.byref(dst.picture()),
                                        ctypes.byref(meta.s), _stream_ptr(stream)), "mi_deblock_frame_to")


class CdefMeta:
    """Device copy of the Av1Filter array + frame CDEF params (MiCdef). With the picture's
    (w, h, layout), also the workgroup order mi_cdef_tile_order computes on the host (costliest
    units first), as the frame executor passes it."""

    def __init__(self, masks, cdef, masks_dev=None, geometry=None):
        self.masks = masks_dev if masks_dev is not None else \
            torch.from_numpy(np.ascontiguousarray(masks).view(np.uint8).reshape(-1)).cuda()
        s = MiCdef()
        s.masks = self.masks.data_ptr()
        s.sb128w = int(masks.shape[1])
        s.damping = int(cdef["damping"])
        s.y_strength[:] = [int(v) for v in cdef["y_strength"]]
        s.uv_strength[:] = [int(v) for v in cdef["uv_strength"]]
        self.s = s
        self.order = None
        if geometry is not None:
            w, h, layout = geometry
            m = np.ascontiguousarray(masks)
            cap = ((w + 63) // 64 + 1) * ((h + 63) // 64 + 1)
            buf = (ctypes.c_int32 * cap)()
            n = lib().mi_cdef_tile_order(m.ctypes.data_as(ctypes.c_void_p), w, h, layout, ctypes.byref(s), buf, cap)
            check(n if n < 0 else 0, "mi_cdef_tile_order")
            self.order = torch.tensor(list(buf[:n]), dtype=torch.int32).cuda()
            s.order = self.order.data_ptr()


def cdef_frame(ctx, src, dst, meta, stream=None):
    ps, pd = src.picture(), dst.picture()
    check(lib().mi_cdef_frame(ctx.h, ctypes.byref(ps), ctypes.byref(pd), ctypes.byref(meta.s),
                              _stream_ptr(stream)), "mi_cdef_frame")


class LrMeta:
    """Device copy of the Av1Restoration array + frame LR params (MiLr). With the picture's
    (w, h, layout), also the workgroup order mi_lr_tile_order computes on the host (longest
    tiles first), as the frame executor passes it."""

    def __init__(self, lr, geometry=None):
        m = np.ascontiguousarray(lr["lr_mask"])
        self.mask = torch.from_numpy(m.view(np.uint8).reshape(-1)).cuda()
        s = MiLr()
        s.lr_mask = self.mask.data_ptr()
        s.sb128w = int(m.shape[1])
        s.restore_planes = int(lr["restore_planes"])
        s.unit_size_log2[0], s.unit_size_log2[1] = [int(v) for v in lr["unit_size_log2"]]
        self.s = s
        self.order = None
        if geometry is not None:
            w, h, layout = geometry
            cap = 3 * ((h + 63) // 64 + 1) * ((w + 31) // 32 + 1)
            buf = (ctypes.c_int32 * cap)()
            n = lib().mi_lr_tile_order(m.ctypes.data_as(ctypes.c_void_p), w, h, layout, ctypes.byref(s), buf, cap)
            check(n if n < 0 else 0, "mi_lr_tile_order")
            self.order = torch.tensor(list(buf[:n]), dtype=torch.int32).cuda()
            s.order = self.order.data_ptr()


def lr_frame(ctx, cdef, deblocked, dst, meta, stream=None):
    pc, pd, po = cdef.picture(), deblocked.picture(), dst.picture()
    check(lib().mi_lr_frame(ctx.h, ctypes.byref(pc), ctypes.byref(pd), ctypes.byref(po),
                            ctypes.byref(meta.s), _stream_ptr(stream)), "mi_lr_frame")


def film_grain_data(fg):
    """dict (rav1d_amd.synth.make_fg_params) -> MiFilmGrainData (a MiFilmGrainData is returned as is)"""
    if isinstance(fg, MiFilmGrainData):
        return fg
    d = MiFilmGrainData()
    d.seed = fg["seed"]
    d.num_y_points = fg["num_y_points"]
    for i, (a, b) in enumerate(fg["y_points"]):
        d.y_points[i][0], d.y_points[i][1] = a, b
    d.chroma_scaling_from_luma = fg["chroma_scaling_from_luma"]
    for pl in range(2):
        d.num_uv_points[pl] = fg["num_uv_points"][pl]
        for i, (a, b) in enumerate(fg["uv_points"][pl]):
            d.uv_points[pl][i][0], d.uv_points[pl][i][1] = a, b
        for i, v in enumerate(fg["ar_coeffs_uv"][pl]):
            d.ar_coeffs_uv[pl][i] = v
        d.uv_mult[pl], d.uv_luma_mult[pl], d.uv_offset[pl] = fg["uv_mult"][pl], fg["uv_luma_mult"][pl], fg["uv_offset"][pl]
    d.scaling_shift = fg["scaling_shift"]
    d.ar_coeff_lag = fg["ar_coeff_lag"]
    for i, v in enumerate(fg["ar_coeffs_y"]):
        d.ar_coeffs_y[i] = v
    d.ar_coeff_shift = fg["ar_coeff_shift"]
    d.grain_scale_shift = fg["grain_scale_shift"]
    d.overlap_flag = fg["overlap_flag"]
    d.clip_to_restricted_range = fg["clip_to_restricted_range"]
    return d


def film_grain_frame(ctx, src, dst, fg, is_id=0, stream=None):
    d = film_grain_data(fg)
    ps, pd = src.picture(), dst.picture()
    check(lib().mi_film_grain_frame(ctx.h, ctypes.byref(ps), ctypes.byref(pd), ctypes.byref(d), is_id,
                                    _stream_ptr(stream)), "mi_film_grain_frame")
