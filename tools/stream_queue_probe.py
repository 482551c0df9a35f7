"""Which stream pairs run concurrently on this box (GPU_MAX_HW_QUEUES hardware queues, HIP maps streams onto them
round-robin): two ~1 ms busy kernels (torch.cuda._sleep) on a pair of streams, wall time ~1 ms when they overlap,
~2 ms when the streams share a hardware queue."""
import time

import torch

dev = torch.device("cuda", 0)
torch.cuda.init()
CYC = 2_000_000


def pair(a, b, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(a):
            torch.cuda._sleep(CYC)
        with torch.cuda.stream(b):
            torch.cuda._sleep(CYC)
        torch.cuda.synchronize(dev)
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


null = torch.cuda.current_stream(dev)
with torch.cuda.stream(null):
    torch.cuda._sleep(CYC)
torch.cuda.synchronize(dev)
t0 = time.perf_counter()
torch.cuda._sleep(CYC)
torch.cuda.synchronize(dev)
print("one sleep kernel: %.3f ms" % ((time.perf_counter() - t0) * 1e3))
pool = [torch.cuda.Stream(dev) for _ in range(6)]
hi = [torch.cuda.Stream(dev, priority=-1) for _ in range(3)]
ext = [torch.cuda.ExternalStream(torch.cuda.Stream(dev).cuda_stream) for _ in range(1)]
print("null + pool[i]:", ["%.2f" % pair(null, s) for s in pool])
print("pool[0] + pool[i]:", ["%.2f" % pair(pool[0], s) for s in pool[1:]])
print("null + hi[i]:", ["%.2f" % pair(null, s) for s in hi])
print("pool[0] + hi[i]:", ["%.2f" % pair(pool[0], s) for s in hi])
print("hi[0] + hi[i]:", ["%.2f" % pair(hi[0], s) for s in hi[1:]])
more = [torch.cuda.Stream(dev, priority=-1) for _ in range(8)]
print("hi[0] + more[i]:", ["%.2f" % pair(hi[0], s) for s in more])
print("null + more[i]:", ["%.2f" % pair(null, s) for s in more])
lo, hi_ = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (None, None)
print("priority range", torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else "n/a")
