"""Host front-end binding: IVF demux (tools/input/ivf.rs) and the C-ABI of
rav1d_amd/libmi_av1dec.so (include/mi_av1dec.h), which parses AV1 OBUs into per-frame work
lists for the gfx950 kernels. No pixels are produced here."""
import ctypes
import os
import struct
import subprocess

from . import MiFilmGrainData

HERE = os.path.dirname(os.path.abspath(__file__))
DEC_PATH = os.environ.get("MI_DEC_LIB") or os.path.join(HERE, "libmi_av1dec.so")

_dec = None


class MiDecFrame(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int32), ("h", ctypes.c_int32), ("up_w", ctypes.c_int32),
                ("render_w", ctypes.c_int32), ("render_h", ctypes.c_int32),
                ("bpc", ctypes.c_int32), ("layout", ctypes.c_int32), ("sb128", ctypes.c_int32),
                ("intra", ctypes.c_void_p), ("intra_tx", ctypes.c_void_p), ("n_intra", ctypes.c_int32),
                ("dep_start", ctypes.c_void_p), ("deps", ctypes.c_void_p), ("n_deps", ctypes.c_int32),
                ("inter_tx", ctypes.c_void_p), ("n_inter_tx", ctypes.c_int32),
                ("coef", ctypes.c_void_p), ("ncoef", ctypes.c_size_t),
                ("idx", ctypes.c_void_p), ("nidx", ctypes.c_size_t),
                ("pal", ctypes.c_void_p), ("npal", ctypes.c_size_t),
                ("filter_y", ctypes.c_int32), ("filter_uv", ctypes.c_int32),
                ("lf_level", ctypes.c_void_p), ("b4_stride", ctypes.c_int32),
                ("lf_masks", ctypes.c_void_p), ("sb128w", ctypes.c_int32), ("sb128h", ctypes.c_int32),
                ("lim_e", ctypes.c_uint8 * 64), ("lim_i", ctypes.c_uint8 * 64),
                ("cdef_on", ctypes.c_int32), ("cdef_damping", ctypes.c_int32),
                ("cdef_y", ctypes.c_uint8 * 8), ("cdef_uv", ctypes.c_uint8 * 8),
                ("lr_mask", ctypes.c_void_p), ("lr_sb128w", ctypes.c_int32), ("restore_planes", ctypes.c_int32),
                ("lr_unit_size", ctypes.c_int32 * 2),
                ("mc", ctypes.c_void_p), ("n_mc", ctypes.c_int32),
                ("obmc_h", ctypes.c_void_p), ("n_obmc_h", ctypes.c_int32),
                ("obmc_v", ctypes.c_void_p), ("n_obmc_v", ctypes.c_int32),
                ("warp", ctypes.c_void_p), ("n_warp", ctypes.c_int32),
                ("scaled", ctypes.c_void_p), ("n_scaled", ctypes.c_int32),
                ("combine_y", ctypes.c_void_p), ("n_combine_y", ctypes.c_int32),
                ("combine_uv", ctypes.c_void_p), ("n_combine_uv", ctypes.c_int32),
                ("masks", ctypes.c_void_p), ("nmasks", ctypes.c_size_t),
                ("ntmp", ctypes.c_size_t),
                ("q_intra", ctypes.c_void_p), ("q_intra_tx", ctypes.c_void_p), ("q_dep_start", ctypes.c_void_p),
                ("q_deps", ctypes.c_void_p), ("q_n_deps", ctypes.c_int32), ("q_strip_start", ctypes.c_void_p),
                ("q_nstrips", ctypes.c_int32), ("q_granules", ctypes.c_int32)]


class MiDecEvent(ctypes.Structure):
    _fields_ = [("frame", ctypes.POINTER(MiDecFrame)), ("pic_id", ctypes.c_int32),
                ("ref_pic", ctypes.c_int32 * 7), ("show_pic", ctypes.c_int32),
                ("fg_present", ctypes.c_int32), ("fg", MiFilmGrainData),
                ("release", ctypes.POINTER(ctypes.c_int32)), ("n_release", ctypes.c_int32),
                ("mtrx_identity", ctypes.c_int32)]


def build_dec():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "host")], check=True)


def dec_lib():
    global _dec
    if _dec is None:
        if not os.path.exists(DEC_PATH):
            raise RuntimeError(f"{DEC_PATH} missing: build it with `make -C rav1d_amd/host`")
        d = ctypes.CDLL(DEC_PATH)
        d.mi_dec_create.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        d.mi_dec_destroy.argtypes = [ctypes.c_void_p]
        d.mi_dec_destroy.restype = None
        d.mi_dec_send.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        d.mi_dec_next.argtypes = [ctypes.c_void_p, ctypes.POINTER(MiDecEvent)]
        d.mi_dec_set_threads.argtypes = [ctypes.c_void_p, ctypes.c_int]
        d.mi_dec_set_inloop_filters.argtypes = [ctypes.c_void_p, ctypes.c_int]
        d.mi_dec_error.argtypes = [ctypes.c_void_p]
        d.mi_dec_error.restype = ctypes.c_char_p
        _dec = d
    return _dec


def ivf_frames(path_or_bytes):
    """Yield the frame payloads of an IVF file (32-byte header, then 12-byte frame headers:
    u32 size, u64 timestamp; tools/input/ivf.rs:224)."""
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    if data[:4] != b"DKIF":
        raise ValueError("not an IVF file")
    hdr_len = struct.unpack_from("<H", data, 6)[0]
    off = hdr_len
    while off + 12 <= len(data):
        size = struct.unpack_from("<I", data, off)[0]
        off += 12
        if off + size > len(data):
            break
        yield bytes(data[off:off + size])
        off += size


def _leb128(data, off):
    v, n = 0, 0
    while True:
        if off + n >= len(data) or n >= 8:
            raise ValueError("truncated leb128")
        b = data[off + n]
        v |= (b & 0x7f) << (7 * n)
        n += 1
        if not b & 0x80:
            return v, n


def _obu_type(b):
    return (b >> 3) & 0xf


def _is_annexb(data):
    """annexb_probe (tools/input/annexb.rs; C tools/input/annexb.c): temporal unit, frame unit and
    OBU sizes nest, and the first OBU is an empty temporal delimiter."""
    try:
        tu, n0 = _leb128(data, 0)
        fu, n1 = _leb128(data, n0)
        ou, n2 = _leb128(data, n0 + n1)
    except ValueError:
        return False
    o = n0 + n1 + n2
    if fu + n1 > tu or ou + n2 >= fu or o >= len(data):
        return False
    return _obu_type(data[o]) == 2


def annexb_units(data):
    """Annex B demuxer (tools/input/annexb.rs): temporal_unit(size) > frame_unit(size) >
    obu_length + OBU; yields one OBU at a time, as the reference hands each to the decoder."""
    off = 0
    while off < len(data):
        tu, n = _leb128(data, off)
        off += n
        end_tu = off + tu
        while off < end_tu:
            fu, n = _leb128(data, off)
            off += n
            end_fu = off + fu
            while off < end_fu:
                ln, n = _leb128(data, off)
                off += n
                yield bytes(data[off:off + ln])
                off += ln


def section5_units(data):
    """Low-overhead OBU stream (section 5; tools/input/section5.rs): temporal units split at
    temporal delimiters, every OBU carrying its size field."""
    off, start = 0, 0
    while off < len(data):
        h = data[off]
        if not h & 0x2:
            raise ValueError("section 5 OBU without a size field")
        if _obu_type(h) == 2 and off > start:
            yield bytes(data[start:off])
            start = off
        ext = 1 if h & 0x4 else 0
        ln, n = _leb128(data, off + 1 + ext)
        off += 1 + ext + n + ln
    if off > start:
        yield bytes(data[start:off])


def stream_units(data):
    """The decoder inputs of a file in any of the reference CLI's demuxer formats (IVF, Annex B,
    section 5; tools/input/input.rs probes them in that order)."""
    if data[:4] == b"DKIF":
        return ivf_frames(data)
    if _is_annexb(data):
        return annexb_units(data)
    return section5_units(data)


# Dav1dSettings.inloop_filters bits (include/dav1d/dav1d.rs:28-35; include/mi_av1dec.h)
INLOOPFILTER_NONE, INLOOPFILTER_DEBLOCK, INLOOPFILTER_CDEF, INLOOPFILTER_RESTORATION = 0, 2, 4, 8
INLOOPFILTER_ALL = INLOOPFILTER_DEBLOCK | INLOOPFILTER_CDEF | INLOOPFILTER_RESTORATION
# the CLI's --inloopfilters values (inloop_filters_tbl, tools/dav1d_cli_parse.rs:479-530)
INLOOPFILTER_NAMES = {"none": 0, "deblock": 2, "nodeblock": 12, "cdef": 4, "nocdef": 10,
                      "restoration": 8, "norestoration": 6, "all": 14}


class Av1Decoder:
    """One stream. send() one temporal unit, then drain events()."""

    def __init__(self, threads=1, inloop_filters=INLOOPFILTER_ALL):
        """threads > 1: intra frames are decoded on that many worker threads (mi_dec_set_threads);
        send a few temporal units ahead of draining events() to overlap them. inloop_filters:
        Dav1dSettings.inloop_filters (an int of INLOOPFILTER_* bits or a CLI name)."""
        self.lib = dec_lib()
        self.h = ctypes.c_void_p()
        r = self.lib.mi_dec_create(ctypes.byref(self.h))
        if r:
            raise RuntimeError(f"mi_dec_create: {r}")
        if threads > 1:
            self.lib.mi_dec_set_threads(self.h, threads)
        if isinstance(inloop_filters, str):
            inloop_filters = INLOOPFILTER_NAMES[inloop_filters]
        if inloop_filters != INLOOPFILTER_ALL:
            r = self.lib.mi_dec_set_inloop_filters(self.h, int(inloop_filters))
            if r:
                raise ValueError(f"mi_dec_set_inloop_filters({inloop_filters}): {r}")

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.mi_dec_destroy(self.h)
            self.h = None

    def error(self):
        return self.lib.mi_dec_error(self.h).decode()

    def send(self, data):
        r = self.lib.mi_dec_send(self.h, data, len(data))
        if r < 0:
            raise RuntimeError(f"mi_dec_send: {r} ({self.error()})")

    def events(self):
        """Yield MiDecEvent structs; each is valid only until the next one is requested."""
        ev = MiDecEvent()
        while True:
            r = self.lib.mi_dec_next(self.h, ctypes.byref(ev))
            if r < 0:
                raise RuntimeError(f"mi_dec_next: {r} ({self.error()})")
            if r == 0:
                return
            yield ev


def stream_events(data, threads=1, lookahead=None, inloop_filters=INLOOPFILTER_ALL):
    """Decoder events of a stream (IVF, Annex B or section 5) in decode order. With threads > 1 the front-end keeps
    `lookahead` (default 2 * threads) temporal units ahead of the events handed out, so that
    frames decode on the worker threads while the caller consumes earlier ones. Each event is
    valid until the next one is requested."""
    dec = Av1Decoder(threads, inloop_filters)
    la = 0 if threads <= 1 else (lookahead if lookahead is not None else 2 * threads)
    # (threads > 1 with lookahead 0: one temporal unit at a time, its frame's tiles in parallel)
    sent = 0
    for tu in stream_units(data):
        dec.send(tu)
        sent += 1
        if sent <= la:
            continue
        gen = dec.events()
        if la:
            ev = next(gen, None)     # one event per temporal unit sent: the queue stays `la` deep
            if ev is not None:
                yield ev
        else:
            yield from gen
    yield from dec.events()
