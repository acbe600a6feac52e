"""The oracle is re-entrant: the CPU baseline (oracle/cpu_bench.c) and the parity checkers run it
from several threads at once. Each thread decodes its own copy of one synthetic frame through
the itx and loop-restoration restatements (the stages that keep per-call scratch) while the
others run, and every thread's output must equal a single-threaded run. ctypes releases the
GIL for the duration of each oracle call, so the calls genuinely overlap.
"""
import threading

import numpy as np

from rav1d_amd.synth import make_frame
from tests import oracle_lib

W, H, BPC, LAYOUT = 256, 256, 10, 1      # the LR restatement expects 128-aligned planes


def _decode(fr):
    planes = oracle_lib.itx_frame([p.copy() for p in fr["planes"]], fr["blocks"], fr["coef"].copy(), BPC)
    return oracle_lib.lr_frame(planes, planes, BPC, LAYOUT, W, H, fr["lr"])


def test_oracle_itx_and_lr_are_thread_safe():
    frames = [make_frame(W, H, BPC, LAYOUT, seed=0x7E5 + k, with_fg=False) for k in range(4)]
    want = [_decode(fr) for fr in frames]
    got = [[None] * 3 for _ in frames]

    def work(k):
        for it in range(3):
            got[k][it] = _decode(frames[k])

    threads = [threading.Thread(target=work, args=(k,)) for k in range(len(frames))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for k in range(len(frames)):
        for it in range(3):
            for p in range(3):
                assert np.array_equal(got[k][it][p], want[k][p]), (k, it, p)
