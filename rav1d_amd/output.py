"""Output side (include/mi_av1out.h): displayed pictures from HBM into pinned host memory (film
grain fused with the copy, librav1d_amd.so) and the reference CLI's muxers md5 / yuv / y4m2 /
null (tools/output/*.rs, implemented in C++ in libmi_av1dec.so)."""
import ctypes

import numpy as np

from . import MiFilmGrainData, MiPicture, check, lib
from .av1dec import dec_lib

_VP = ctypes.c_void_p


class MiOutParams(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int32), ("h", ctypes.c_int32), ("bpc", ctypes.c_int32), ("layout", ctypes.c_int32),
                ("chr", ctypes.c_int32), ("render_w", ctypes.c_int32), ("render_h", ctypes.c_int32)]


def _mux_lib():
    d = dec_lib()
    if not getattr(d, "_mux_bound", False):
        d.mi_muxer_open.argtypes = [ctypes.POINTER(_VP), ctypes.c_char_p, ctypes.c_char_p,
                                    ctypes.POINTER(MiOutParams), ctypes.POINTER(ctypes.c_uint * 2)]
        d.mi_muxer_write.argtypes = [_VP, ctypes.POINTER(MiPicture)]
        d.mi_muxer_verify.argtypes = [_VP, ctypes.c_char_p]
        d.mi_muxer_digest.argtypes = [_VP, ctypes.c_char_p]
        d.mi_muxer_close.argtypes = [_VP]
        d.mi_muxer_close.restype = None
        d._mux_bound = True
    return d


class Muxer:
    """One output muxer (tools/output/output.rs): name "md5" | "yuv" | "y4m2" | "null"; file a
    path, "-" (stdout) or None (md5 kept in memory for digest() / verify())."""

    def __init__(self, name, file=None, w=0, h=0, bpc=8, layout=1, chr=0, render=None, fps=(25, 1)):
        d = _mux_lib()
        p = MiOutParams(w, h, bpc, layout, chr, *(render or (w, h)))
        f = (ctypes.c_uint * 2)(*fps)
        self.h = _VP()
        check(d.mi_muxer_open(ctypes.byref(self.h), name.encode(), file.encode() if file else None,
                              ctypes.byref(p), ctypes.byref(f)), f"mi_muxer_open({name})")

    def write(self, pic):
        check(_mux_lib().mi_muxer_write(self.h, ctypes.byref(pic)), "mi_muxer_write")

    def digest(self):
        buf = ctypes.create_string_buffer(33)
        check(_mux_lib().mi_muxer_digest(self.h, buf), "mi_muxer_digest")
        return buf.value.decode()

    def verify(self, md5_hex):
        return _mux_lib().mi_muxer_verify(self.h, md5_hex.encode())

    def close(self):
        if self.h:
            _mux_lib().mi_muxer_close(self.h)
            self.h = None

    def __del__(self):
        self.close()


def host_picture_np(planes, w, h, bpc, layout):
    """MiPicture over numpy planes (host memory: for the muxers)."""
    pic = MiPicture()
    for p in range(3):
        pic.data[p] = planes[min(p, len(planes) - 1)].ctypes.data
    pic.stride[0] = planes[0].strides[0]
    pic.stride[1] = planes[1].strides[0] if len(planes) > 1 else planes[0].strides[0]
    pic.w, pic.h, pic.bpc, pic.layout = w, h, bpc, layout
    return pic


class HostPicture:
    """A pinned, device-mapped host picture (mi_host_picture_alloc) with numpy views."""

    def __init__(self, w, h, bpc, layout):
        self.pic = MiPicture()
        check(lib().mi_host_picture_alloc(w, h, layout, bpc, ctypes.byref(self.pic)), "mi_host_picture_alloc")

    def plane_np(self, p):
        """Visible area of plane p (a copy)."""
        pic = self.pic
        ss_hor, ss_ver = int(pic.layout in (1, 2)), int(pic.layout == 1)
        w, h = (pic.w, pic.h) if p == 0 else ((pic.w + ss_hor) >> ss_hor, (pic.h + ss_ver) >> ss_ver)
        st = pic.stride[1 if p else 0]
        pxb = 1 if pic.bpc == 8 else 2
        raw = np.ctypeslib.as_array((ctypes.c_uint8 * (st * h)).from_address(pic.data[p])).reshape(h, st)
        rows = raw[:, :w * pxb].copy()
        return rows.view("<u2") if pxb == 2 else rows

    def free(self):
        if self.pic.data[0]:
            lib().mi_host_picture_free(ctypes.byref(self.pic))

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def output_picture(ctx, frame, host, fg=None, is_id=0, stream=None):
    """Enqueue the output of a device Frame into a HostPicture (+ film grain when fg, a
    MiFilmGrainData or a make_fg_params dict)."""
    from .frame import _stream_ptr, film_grain_data
    src = frame.picture()
    if fg is not None and not isinstance(fg, MiFilmGrainData):
        fg = film_grain_data(fg)
    check(lib().mi_output_picture(ctx.h, ctypes.byref(src), ctypes.byref(host.pic),
                                  ctypes.byref(fg) if fg is not None else None, is_id, _stream_ptr(stream)),
          "mi_output_picture")
