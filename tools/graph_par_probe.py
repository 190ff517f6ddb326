"""Do the independent branches of a captured HIP graph run concurrently?
Two chains of small launches captured on one stream vs forked onto two
streams (event fork / join inside the capture); replay time per launch."""
import time

import torch

dev = torch.device("cuda", 0)
n = 60
x = [torch.randn(64, 64, device=dev) for _ in range(4)]


def chain(t, k):
    for _ in range(k):
        t = torch.tanh(t @ t * 0.01)
    return t


def capture(parallel):
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    ws = torch.cuda.Stream()
    ws.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(ws):
        chain(x[0], 2)
    torch.cuda.current_stream().wait_stream(ws)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        if parallel:
            side.wait_stream(cur)
            chain(x[0], n)
            with torch.cuda.stream(side):
                chain(x[1], n)
            cur.wait_stream(side)
        else:
            chain(x[2], n)
            chain(x[3], n)
    return g


for par in (False, True, False, True):
    g = capture(par)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20 * 1e6
    print("parallel=%d  %.1f us per replay, %.2f us per launch (%d launches)" % (par, dt, dt / (6 * n), 6 * n),
          flush=True)
