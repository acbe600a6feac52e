"""Whole-frame intra reconstruction on the device: the batched replacement of recon_b_intra's
per-transform-block loop (rav1d src/recon.rs:2402-3160: prepare_intra_edges + intra_pred /
cfl_pred / pal_pred, then itxfm_add).

Transform blocks are grouped by dependency level (ipred_synth.make_intra_frame computes the
levels a decoder's block walk implies). Each level is two launches on one stream:
mi_intra_blocks (edges gathered on the device from the picture, then prediction) and
mi_itx_frame over the same blocks' residuals (grouped by transform size within the level).
Level L + 1 reads only pixels that levels <= L finished.

IntraFrame.recon / intra_recon use the persistent fused path instead (mi_intra_recon): one
launch for up to 8 frames, prediction + residual per block, per-block dependency waits.
"""
import ctypes

import numpy as np
import torch

from . import ITX_KEEP_COEFS, N_RECT_TX_SIZES, TXBLOCK_DTYPE
from . import frame as F
from .synth import TX_BY_DIMS, make_coefs, tx_types


def make_intra_residuals(fr, bpc, rng, dc_frac=0.5, full_frac=0.1):
    """One MiTxBlock + coefficients per intra transform block of `fr` (make_intra_frame),
    laid out level by level and, within a level, grouped by transform size. Adds to fr:
    tx_blocks, tx_size_start (levels x 20, relative to the level's first record), tx_level_off,
    coef, tx_of_block (decode-order block index -> its MiTxBlock row)."""
    blocks, order, ls = fr["blocks"], fr["order"], fr["level_start"]
    recs, chunks, off = [], [], 0
    per_block = {}
    for k in order:
        b = blocks[k]
        tx = TX_BY_DIMS[(int(b["w"]), int(b["h"]))]
        if rng.random() < dc_frac:
            txtp, regime = 0, 0
        else:
            types = tx_types(tx)
            txtp = types[int(rng.integers(len(types)))]
            regime = 2 if rng.random() < full_frac / (1 - dc_frac) else 1
        c, eob = make_coefs(rng, tx, txtp, regime, bpc)
        per_block[int(k)] = (off, int(b["x"]), int(b["y"]), int(b["plane"]), tx, txtp, 0, eob)
        chunks.append(c)
        off += c.size
    rows, size_start, level_off, tx_of_block = [], [], [], np.zeros(len(blocks), np.int64)
    for lv in range(len(ls) - 1):
        ks = [int(k) for k in order[ls[lv]:ls[lv + 1]]]
        ks.sort(key=lambda k: (per_block[k][4], per_block[k][5]))
        level_off.append(len(rows))
        txs = [per_block[k][4] for k in ks]
        size_start.append(np.searchsorted(np.array(txs, np.int64), np.arange(N_RECT_TX_SIZES + 1)).astype(np.uint32))
        for k in ks:
            tx_of_block[k] = len(rows)
            rows.append(per_block[k])
    fr["tx_blocks"] = np.array(rows, dtype=TXBLOCK_DTYPE)
    fr["tx_size_start"] = np.array(size_start, np.uint32)
    fr["tx_level_off"] = np.array(level_off, np.int64)
    fr["coef"] = np.concatenate(chunks).astype(np.int16 if bpc == 8 else np.int32)
    fr["tx_of_block"] = tx_of_block
    return fr


class IntraFrame:
    """Device copies of one intra frame's descriptors; step() reconstructs it into `pic`."""

    def __init__(self, ctx, fr):
        self.ctx, self.fr = ctx, fr
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()  # noqa: E731
        self.blocks = dev(fr["blocks"][fr["order"]])
        self.ac = torch.from_numpy(fr["ac"].copy()).cuda()
        self.idx = torch.from_numpy(fr["idx"].copy()).cuda()
        self.pal = dev(fr["pal"])
        self.tx = dev(fr["tx_blocks"])
        self.coef = torch.from_numpy(fr["coef"].copy()).cuda()
        ls = fr["level_start"]
        self.levels = [(int(ls[i]), int(ls[i + 1])) for i in range(len(ls) - 1)]
        # fused path: blocks in level order, their residual records in the same order, and the
        # dependency lists as positions in that order
        order = fr["order"]
        pos = np.empty(len(order), np.int64)
        pos[order] = np.arange(len(order))
        dl = [pos[fr["deps"][k]] for k in order]
        self.dep_start = torch.from_numpy(np.concatenate([[0], np.cumsum([len(d) for d in dl])]).astype(np.int32)).cuda()
        deps = np.concatenate(dl).astype(np.int32) if sum(len(d) for d in dl) else np.zeros(1, np.int32)
        self.deps = torch.from_numpy(deps).cuda()
        self.tx_ord = dev(fr["tx_blocks"][fr["tx_of_block"][order]])
        self.ss = [(ctypes.c_uint32 * (N_RECT_TX_SIZES + 1))(*[int(v) for v in row]) for row in fr["tx_size_start"]]

    def step(self, pic, stream=None, keep_coefs=True):
        lib = F.lib()
        sp = F._stream_ptr(stream)
        h = self.ctx.h
        ac, idx, pal = (ctypes.c_void_p(t.data_ptr()) for t in (self.ac, self.idx, self.pal))
        coef = ctypes.c_void_p(self.coef.data_ptr())
        flags = ITX_KEEP_COEFS if keep_coefs else 0
        for lv, (a, b) in enumerate(self.levels):
            F.check(lib.mi_intra_blocks(h, ctypes.byref(pic), ctypes.c_void_p(self.blocks.data_ptr() + 32 * a), b - a,
                                        ac, idx, pal, sp), "mi_intra_blocks")
            t0 = int(self.fr["tx_level_off"][lv])
            F.check(lib.mi_itx_frame(h, ctypes.byref(pic), ctypes.c_void_p(self.tx.data_ptr() + 16 * t0), self.ss[lv],
                                     coef, flags, sp), "mi_itx_frame")

    def frame_desc(self, pic):
        """MiIntraFrame for the fused path (pic: MiPicture)."""
        from . import MiIntraFrame
        d = MiIntraFrame()
        d.pic = pic
        d.blocks, d.tx = self.blocks.data_ptr(), self.tx_ord.data_ptr()
        d.dep_start, d.deps = self.dep_start.data_ptr(), self.deps.data_ptr()
        d.ac, d.idx, d.pal = self.ac.data_ptr(), self.idx.data_ptr(), self.pal.data_ptr()
        d.coef = self.coef.data_ptr()
        d.n = len(self.fr["blocks"])
        return d

    def recon(self, pic, stream=None, keep_coefs=True, granules=False):
        """Whole-frame reconstruction in one persistent launch (mi_intra_recon)."""
        intra_recon(self.ctx, [(self, pic)], stream, keep_coefs, granules)


IR_EDGE_GRANULES = 2   # mi_av1dsp.h MI_IR_EDGE_GRANULES


def intra_recon(ctx, frames, stream=None, keep_coefs=True, granules=False):
    """Reconstruct up to 24 independent intra frames in one launch: frames = [(IntraFrame,
    MiPicture)], frame f on XCD f % 8. granules: MI_IR_EDGE_GRANULES (every pixel an edge reads
    is reconstructed by this call: intra-only frames)."""
    from . import MiIntraFrame
    descs = (MiIntraFrame * len(frames))(*[f.frame_desc(p) for f, p in frames])
    flags = (ITX_KEEP_COEFS if keep_coefs else 0) | (IR_EDGE_GRANULES if granules else 0)
    F.check(F.lib().mi_intra_recon(ctx.h, descs, len(frames), flags, F._stream_ptr(stream)), "mi_intra_recon")


def device_status(ctx, stream=None):
    """Synchronise and raise if a persistent launch reported a failed dependency wait."""
    F.check(F.lib().mi_ctx_device_status(ctx.h, F._stream_ptr(stream)), "mi_ctx_device_status")
