"""GPU time of a launch sequence without host overhead: the calls are captured into a HIP graph
(torch.cuda.graph; the library launches on the capture stream) and the graph is replayed."""
import torch


def gtime(fn, reps=20, replays=10):
    """Mean device time (us) of one fn() call; fn(stream) enqueues on `stream`."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * replays)
