"""Per-launch floor of a chain of trivial dependent kernels, eager and HIP
graph (prints us per launch).  Run under different env settings."""
import os
import time

import torch

n = 200
x = torch.zeros(1024, device="cuda")
y = torch.zeros(64 * 1024 * 16, device="cuda")


def chain(t):
    for _ in range(n):
        t.add_(1.0)


for name, t in (("tiny", x), ("1MB", y)):
    for _ in range(3):
        chain(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        chain(t)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / (5 * n) * 1e6
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain(t)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        chain(t)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    gr = (time.perf_counter() - t0) / (10 * n) * 1e6
    print("%-5s eager %.2f us/launch  graph %.2f us/launch  env=%s" % (
        name, eager, gr, {k: v for k, v in os.environ.items() if k.startswith(("HIP_", "DEBUG_HIP", "GPU_", "AMD_"))}),
        flush=True)
