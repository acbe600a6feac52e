"""configs[3]'s film-grain measurement alone (bench.film_grain_8k), for quick A/B runs."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
from rav1d_amd import frame as F
ctx = F.Context(0)
s = torch.cuda.Stream()
for _ in range(2):
    print(bench.film_grain_8k(ctx, s), flush=True)
