"""rav1d_amd — MI355X-native AV1 decode-DSP path behind rav1d's DSP tables.

The product is the C-ABI library ``librav1d_amd.so`` (header ``include/mi_av1dsp.h``),
built from the gfx950 HIP sources in ``csrc/``. This package is the host-side mirror used
by tests and the benchmark: it loads the library, describes its structs for ctypes/numpy,
and wraps the entry points. There is no CPU fallback: if the library is missing or has no
GPU, calls fail loudly.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MI_LIB") or os.path.join(HERE, "librav1d_amd.so")

_lib = None


class MiError(RuntimeError):
    pass


# --- struct mirrors (include/mi_av1dsp.h) ---------------------------------------------

class MiPicture(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p * 3), ("stride", ctypes.c_ssize_t * 2),
                ("w", ctypes.c_int32), ("h", ctypes.c_int32),
                ("layout", ctypes.c_int32), ("bpc", ctypes.c_int32)]


class MiFramePictures(ctypes.Structure):
    """include/mi_av1dec.h: the pictures of one frame's pass 2 (recon, deblocked, cdef, restored)."""
    _fields_ = [("pics", MiPicture * 4), ("refs", MiPicture * 7)]


class MiFrameTiming(ctypes.Structure):
    """include/mi_av1dec.h: per-stage timing of mi_frame_run (mi_ctx_set_timing / mi_ctx_timing)."""
    _fields_ = [("frames", ctypes.c_int32), ("reserved", ctypes.c_int32), ("host_ms", ctypes.c_double),
                ("upload_ms", ctypes.c_double), ("inter_ms", ctypes.c_double), ("intra_ms", ctypes.c_double),
                ("filter_ms", ctypes.c_double), ("upload_bytes", ctypes.c_int64), ("stage_ms", ctypes.c_double),
                ("strips_ms", ctypes.c_double)]


class MiIntraFrame(ctypes.Structure):
    _fields_ = [("pic", MiPicture), ("blocks", ctypes.c_void_p), ("tx", ctypes.c_void_p),
                ("dep_start", ctypes.c_void_p), ("deps", ctypes.c_void_p), ("ac", ctypes.c_void_p),
                ("idx", ctypes.c_void_p), ("pal", ctypes.c_void_p), ("coef", ctypes.c_void_p), ("n", ctypes.c_int32)]


class MiLoopFilter(ctypes.Structure):
    _fields_ = [("level", ctypes.c_void_p), ("b4_stride", ctypes.c_ssize_t), ("masks", ctypes.c_void_p),
                ("sb128w", ctypes.c_int32), ("filter_y", ctypes.c_int32), ("filter_uv", ctypes.c_int32),
                ("lim_e", ctypes.c_uint8 * 64), ("lim_i", ctypes.c_uint8 * 64)]


class MiCdef(ctypes.Structure):
    _fields_ = [("masks", ctypes.c_void_p), ("sb128w", ctypes.c_int32), ("damping", ctypes.c_int32),
                ("y_strength", ctypes.c_uint8 * 8), ("uv_strength", ctypes.c_uint8 * 8), ("order", ctypes.c_void_p)]


class MiLr(ctypes.Structure):
    _fields_ = [("lr_mask", ctypes.c_void_p), ("sb128w", ctypes.c_int32), ("restore_planes", ctypes.c_int32),
                ("unit_size_log2", ctypes.c_int32 * 2), ("order", ctypes.c_void_p)]


class MiFilmGrainData(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint), ("num_y_points", ctypes.c_int), ("y_points", (ctypes.c_uint8 * 2) * 14),
                ("chroma_scaling_from_luma", ctypes.c_int), ("num_uv_points", ctypes.c_int * 2),
                ("uv_points", ((ctypes.c_uint8 * 2) * 10) * 2), ("scaling_shift", ctypes.c_int),
                ("ar_coeff_lag", ctypes.c_int), ("ar_coeffs_y", ctypes.c_int8 * 24),
                ("ar_coeffs_uv", (ctypes.c_int8 * 28) * 2), ("ar_coeff_shift", ctypes.c_uint64),
                ("grain_scale_shift", ctypes.c_int), ("uv_mult", ctypes.c_int * 2), ("uv_luma_mult", ctypes.c_int * 2),
                ("uv_offset", ctypes.c_int * 2), ("overlap_flag", ctypes.c_int), ("clip_to_restricted_range", ctypes.c_int)]


assert ctypes.sizeof(MiFilmGrainData) == 224


TXBLOCK_DTYPE = np.dtype([("coef_off", "<u4"), ("x", "<u2"), ("y", "<u2"), ("plane", "u1"),
                          ("tx", "u1"), ("txtp", "u1"), ("flags", "u1"), ("eob", "<i4")])
assert TXBLOCK_DTYPE.itemsize == 16

MCBLOCK_DTYPE = np.dtype([("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"), ("plane", "u1"),
                          ("filter2d", "u1"), ("mvx", "<i2", 2), ("mvy", "<i2", 2), ("ref", "i1", 2),
                          ("comp", "u1"), ("param", "u1"), ("mask_off", "<u4")])
assert MCBLOCK_DTYPE.itemsize == 24
IPRED_DTYPE = np.dtype([("edge_off", "<u4"), ("aux_off", "<u4"), ("x", "<u2"), ("y", "<u2"), ("w", "u1"),
                        ("h", "u1"), ("plane", "u1"), ("mode", "u1"), ("angle", "<u2"), ("max_w", "<u2"),
                        ("max_h", "<u2"), ("alpha", "i1"), ("pad", "u1")])
assert IPRED_DTYPE.itemsize == 24
IPRED_CFL, IPRED_PAL = 32, 64
INTRA_DTYPE = np.dtype([("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"), ("plane", "u1"), ("mode", "u1"),
                        ("angle", "i1"), ("flags", "u1"), ("filt_idx", "u1"), ("alpha", "i1"), ("tile_w", "<u2"),
                        ("tile_h", "<u2"), ("max_w", "<u2"), ("max_h", "<u2"), ("aux_off", "<u4"),
                        ("pal_off", "<u4"), ("reserved", "<u4")])
assert INTRA_DTYPE.itemsize == 32
INTRA_HAVE_LEFT, INTRA_HAVE_TOP, INTRA_TOP_RIGHT, INTRA_BOTTOM_LEFT = 1, 2, 4, 8
INTRA_SMOOTH_NB, INTRA_EDGE_FILTER, INTRA_II, INTRA_CFL_AC = 16, 32, 64, 128

MC_AVG, MC_WAVG, MC_MASK, MC_SEG = 0, 1, 2, 3
MC_OBMC_H, MC_OBMC_V, MC_PREP = 4, 5, 6
WARP_DTYPE = np.dtype([("x", "<u2"), ("y", "<u2"), ("plane", "u1"), ("ref", "i1"), ("prep", "u1"), ("pad0", "u1"),
                       ("dx", "<i4"), ("dy", "<i4"), ("mx", "<i4"), ("my", "<i4"), ("abcd", "<i2", 4),
                       ("tmp_off", "<u4"), ("tmp_stride", "<u2"), ("pad1", "<u2")])
assert WARP_DTYPE.itemsize == 40
COMBINE_DTYPE = np.dtype([("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"), ("plane", "u1"), ("comp", "u1"),
                          ("param", "u1"), ("pad", "u1", 3), ("tmp_off", "<u4", 2), ("mask_off", "<u4")])
assert COMBINE_DTYPE.itemsize == 24
IPRED_II = 128
MC_NCLASS = 64

N_RECT_TX_SIZES = 19
ITX_KEEP_COEFS = 1
ITX_DC_DEFER = 2       # mi_itx_frame_runs: DC runs deferred to mi_deblock_frame_dc

_VP = ctypes.c_void_p


def _sig(lib, name, res, args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args
    return f


def lib():
    """Load librav1d_amd.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MiError(f"{LIB_PATH} missing: run `python -m rav1d_amd.build` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    _sig(L, "mi_version", ctypes.c_char_p, [])
    _sig(L, "mi_ctx_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_VP)])
    _sig(L, "mi_ctx_destroy", None, [_VP])
    _sig(L, "mi_ctx_last_error", ctypes.c_int, [_VP])
    _sig(L, "mi_itx_frame", ctypes.c_int,
         [_VP, ctypes.POINTER(MiPicture), _VP, ctypes.POINTER(ctypes.c_uint32), _VP, ctypes.c_uint, _VP])
    _sig(L, "mi_itx_frame_banded", ctypes.c_int,
         [_VP, ctypes.POINTER(MiPicture), _VP, ctypes.POINTER(ctypes.c_uint32), _VP, ctypes.c_uint, _VP])
    _sig(L, "mi_itx_frame_runs", ctypes.c_int,
         [_VP, ctypes.POINTER(MiPicture), _VP, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), _VP,
          ctypes.c_uint, _VP])
    _sig(L, "mi_dsp_itxfm_add", ctypes.c_int,
         [ctypes.c_int, ctypes.c_int, _VP, ctypes.c_ssize_t, _VP, ctypes.c_int, ctypes.c_int])
    _sig(L, "mi_mc_frame", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture), ctypes.c_int,
                                          _VP, ctypes.POINTER(ctypes.c_uint32), _VP, _VP, _VP])
    _sig(L, "mi_mc_frame_ex", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture), ctypes.c_int,
                                             _VP, ctypes.POINTER(ctypes.c_uint32), _VP, _VP, ctypes.c_uint, _VP])
    _sig(L, "mi_mc_frame_sync", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture), ctypes.c_int,
                                               _VP, ctypes.POINTER(ctypes.c_uint32), _VP, ctypes.c_size_t, _VP, _VP])
    _sig(L, "mi_mc_sync_status", ctypes.c_int, [_VP, _VP])
    for n in ("mi_mc_scaled", "mi_mc_warp"):
        _sig(L, n, ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture), ctypes.c_int,
                                  _VP, ctypes.c_int, _VP, _VP])
    _sig(L, "mi_mc_combine", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), _VP, ctypes.c_int, _VP, _VP, _VP])
    _sig(L, "mi_superres_frame", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture), _VP])
    _sig(L, "mi_intra_blocks", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), _VP, ctypes.c_int, _VP, _VP, _VP, _VP])
    _sig(L, "mi_intra_recon", ctypes.c_int, [_VP, ctypes.POINTER(MiIntraFrame), ctypes.c_int, ctypes.c_uint, _VP])
    _sig(L, "mi_ctx_device_status", ctypes.c_int, [_VP, _VP])
    _sig(L, "mi_ipred_blocks", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), _VP, ctypes.c_int, _VP, _VP, _VP, _VP])
    _sig(L, "mi_dsp_intra_pred", ctypes.c_int, [ctypes.c_int, _VP, ctypes.c_ssize_t, _VP] + [ctypes.c_int] * 6)
    _SS = ctypes.c_ssize_t
    _sig(L, "mi_dsp_cfl_pred", ctypes.c_int, [ctypes.c_int, _VP, _SS, _VP, ctypes.c_int, ctypes.c_int, _VP,
                                              ctypes.c_int, ctypes.c_int])
    _sig(L, "mi_dsp_pal_pred", ctypes.c_int, [_VP, _SS, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int])
    _sig(L, "mi_dsp_cfl_ac", ctypes.c_int, [ctypes.c_int, _VP, _VP, _SS] + [ctypes.c_int] * 5)
    _sig(L, "mi_dsp_loop_filter_sb", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _VP, _SS, _VP, _VP, _SS, _VP,
                                                    ctypes.c_int, ctypes.c_int])
    _sig(L, "mi_dsp_cdef_filter", ctypes.c_int, [ctypes.c_int, _VP, _SS, _VP, _VP, _VP] + [ctypes.c_int] * 6)
    _sig(L, "mi_dsp_cdef_dir", ctypes.c_int, [_VP, _SS, _VP, ctypes.c_int])
    _I = ctypes.c_int
    _sig(L, "mi_dsp_mc_put", _I, [_I, _VP, _SS, _VP, _SS, _I, _I, _I, _I, _I])
    _sig(L, "mi_dsp_mc_prep", _I, [_I, _VP, _VP, _SS, _I, _I, _I, _I, _I])
    _sig(L, "mi_dsp_mc_avg", _I, [_VP, _SS, _VP, _VP, _I, _I, _I])
    _sig(L, "mi_dsp_mc_w_avg", _I, [_VP, _SS, _VP, _VP, _I, _I, _I, _I])
    _sig(L, "mi_dsp_mc_mask", _I, [_VP, _SS, _VP, _VP, _I, _I, _VP, _I])
    _sig(L, "mi_dsp_mc_w_mask", _I, [_I, _VP, _SS, _VP, _VP, _I, _I, _VP, _I, _I])
    _sig(L, "mi_dsp_mc_blend", _I, [_VP, _SS, _VP, _I, _I, _VP, _I])
    for n in ("mi_dsp_mc_blend_v", "mi_dsp_mc_blend_h"):
        _sig(L, n, _I, [_VP, _SS, _VP, _I, _I, _I])
    _sig(L, "mi_dsp_mc_emu_edge", _I, [_I, _I, _I, _I, _I, _I, _VP, _SS, _VP, _SS, _I])
    _sig(L, "mi_dsp_mc_warp8x8", _I, [_I, _VP, _SS, _VP, _SS, _VP, _I, _I, _I])
    _sig(L, "mi_dsp_mc_resize", _I, [_VP, _SS, _VP, _SS, _I, _I, _I, _I, _I, _I])
    _sig(L, "mi_dsp_mc_scaled", _I, [_I, _I, _VP, _SS, _VP, _SS] + [_I] * 7)
    _sig(L, "mi_dsp_lr_wiener", _I, [_VP, _SS, _VP, _VP, _I, _I, _VP, _I, _I])
    _sig(L, "mi_dsp_lr_sgr", _I, [_I, _VP, _SS, _VP, _VP, _I, _I, _VP, _I, _I])
    _sig(L, "mi_dsp_fg_generate_grain_y", _I, [_VP, _VP, _I])
    _sig(L, "mi_dsp_fg_generate_grain_uv", _I, [_I, _VP, _VP, _VP, _I, _I])
    _sig(L, "mi_dsp_fgy_32x32xn", _I, [_VP, _VP, _SS, _VP, ctypes.c_size_t, _VP, _VP, _I, _I, _I])
    _sig(L, "mi_dsp_fguv_32x32xn", _I, [_I, _VP, _VP, _SS, _VP, ctypes.c_size_t, _VP, _VP, _I, _I, _VP, _SS, _I, _I,
                                        _I])
    _sig(L, "mi_deblock_frame", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiLoopFilter), _VP])
    _sig(L, "mi_deblock_frame_to", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture),
                                                  ctypes.POINTER(MiLoopFilter), _VP])
    _sig(L, "mi_deblock_frame_dc", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture),
                                                  ctypes.POINTER(MiLoopFilter), _VP])
    _sig(L, "mi_cdef_frame", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture),
                                            ctypes.POINTER(MiCdef), _VP])
    _sig(L, "mi_lr_frame", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture),
                                          ctypes.POINTER(MiPicture), ctypes.POINTER(MiLr), _VP])
    _sig(L, "mi_cdef_tile_order", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(MiCdef),
                                                 ctypes.POINTER(ctypes.c_int32), ctypes.c_int])
    _sig(L, "mi_lr_tile_order", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(MiLr),
                                               ctypes.POINTER(ctypes.c_int32), ctypes.c_int])
    for n in ("mi_film_grain_frame", "mi_film_grain_apply"):
        _sig(L, n, ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture),
                                  ctypes.POINTER(MiFilmGrainData), ctypes.c_int, _VP])
    _sig(L, "mi_film_grain_prep", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiFilmGrainData), _VP])
    _sig(L, "mi_frame_run", ctypes.c_int, [_VP, _VP, ctypes.POINTER(MiFramePictures), ctypes.POINTER(ctypes.c_int), _VP])
    _sig(L, "mi_frame_plan_ms", ctypes.c_double, [_VP, ctypes.c_int])
    _sig(L, "mi_frame_end", ctypes.c_int, [_VP, _VP])
    _sig(L, "mi_frame_validate", ctypes.c_int, [_VP, ctypes.POINTER(MiFramePictures), ctypes.POINTER(ctypes.c_char_p)])
    _sig(L, "mi_ctx_set_timing", ctypes.c_int, [_VP, ctypes.c_int])
    _sig(L, "mi_ctx_timing", ctypes.c_int, [_VP, ctypes.POINTER(MiFrameTiming)])
    # output side (include/mi_av1out.h)
    _sig(L, "mi_host_picture_alloc", ctypes.c_int, [_I, _I, _I, _I, ctypes.POINTER(MiPicture)])
    _sig(L, "mi_host_picture_free", None, [ctypes.POINTER(MiPicture)])
    _sig(L, "mi_output_picture", ctypes.c_int, [_VP, ctypes.POINTER(MiPicture), ctypes.POINTER(MiPicture),
                                                ctypes.POINTER(MiFilmGrainData), ctypes.c_int, _VP])
    _lib = L
    return L


# Every symbol include/mi_av1dsp.h declares (checked by tests/test_abi.py).
EXPORTED = ["mi_version", "mi_ctx_create", "mi_ctx_destroy", "mi_ctx_last_error",
            "mi_itx_frame", "mi_itx_frame_banded", "mi_itx_frame_runs", "mi_mc_frame", "mi_mc_frame_ex", "mi_mc_frame_sync", "mi_mc_sync_status", "mi_mc_scaled", "mi_mc_warp", "mi_mc_combine", "mi_superres_frame",
            "mi_ipred_blocks", "mi_intra_blocks", "mi_intra_recon", "mi_ctx_device_status", "mi_deblock_frame", "mi_deblock_frame_to", "mi_deblock_frame_dc", "mi_cdef_frame", "mi_lr_frame", "mi_lr_tile_order", "mi_cdef_tile_order",
            "mi_film_grain_frame", "mi_film_grain_prep", "mi_film_grain_apply", "mi_frame_run", "mi_frame_end", "mi_frame_validate", "mi_frame_plan_ms",
            "mi_ctx_set_timing", "mi_ctx_timing",
            "mi_dsp_itxfm_add", "mi_dsp_intra_pred", "mi_dsp_cfl_pred", "mi_dsp_pal_pred", "mi_dsp_cfl_ac",
            "mi_dsp_loop_filter_sb", "mi_dsp_cdef_filter", "mi_dsp_cdef_dir", "mi_dsp_mc_put", "mi_dsp_mc_prep",
            "mi_dsp_mc_avg", "mi_dsp_mc_w_avg", "mi_dsp_mc_mask", "mi_dsp_mc_w_mask", "mi_dsp_mc_blend",
            "mi_dsp_mc_blend_v", "mi_dsp_mc_blend_h", "mi_dsp_mc_emu_edge", "mi_dsp_mc_warp8x8", "mi_dsp_mc_resize",
            "mi_dsp_mc_scaled", "mi_dsp_lr_wiener", "mi_dsp_lr_sgr",
            "mi_dsp_fg_generate_grain_y", "mi_dsp_fg_generate_grain_uv", "mi_dsp_fgy_32x32xn", "mi_dsp_fguv_32x32xn",
            "mi_host_picture_alloc", "mi_host_picture_free", "mi_output_picture"]


def check(rc, what):
    if rc != 0:
        raise MiError(f"{what} failed: {rc} ({os.strerror(-rc) if rc < 0 else rc})")
    return rc
