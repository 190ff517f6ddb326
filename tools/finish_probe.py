"""Time sgg_grad_finish on the D-step's job list (synthetic slabs) inside a
HIP graph: the whole list, the pooling slab alone, and torch's column sum of
the same slab for an achievable-bandwidth reference.  GPU only."""
import ctypes
import sys
import os

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "group-gan-gcn-gat_amd"))
from sgan import _native as N  # noqa: E402

DEV = "cuda"
lib = N.load()
D_JOBS = [(40, 3072), (40, 64), (40, 64), (40, 1), (256, 24576), (256, 48), (40, 24576), (40, 512), (160, 9216),
          (160, 192)]


def graph_time(fn, reps=20, iters=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / (reps * iters)


def run(jobs, label, bce=False):
    srcs = [torch.randn(r, c, device=DEV) for r, c in jobs]
    outs = [torch.empty(c, device=DEV) for _, c in jobs]
    reds = (N.Red * len(jobs))(*[N.Red(N.ptr(s), s.shape[0], s.shape[1], 0, s.shape[1], N.ptr(o), 0, 0, 0, 0)
                                 for s, o in zip(srcs, outs)])
    scratch = torch.empty(16, device=DEV)

    x = torch.randn(2560, device=DEV)
    ys = torch.tensor([0.0, 0.9], device=DEV)
    lo = torch.zeros(2, device=DEV)
    bj = (N.BceJob * 1)(N.BceJob(N.ptr(x), 2560, 1280, N.ptr(ys), ctypes.c_void_p(ys.data_ptr() + 4), 1.0, N.ptr(lo),
                                 None, None, None))

    def fn():
        N.check(lib.sgg_grad_finish_losses(reds, len(jobs), None, 0, N.ptr(scratch), 64, None, 0,
                                           bj if bce else None, 1 if bce else 0, N.stream_ptr()), "finish")
    us = graph_time(fn)
    mb = sum(r * c for r, c in jobs) * 4 / 1e6
    ok = all(torch.allclose(o, s.sum(0), rtol=1e-4, atol=1e-4) for s, o in zip(srcs, outs))
    print("%-22s %8.2f us  %7.2f MB  %6.2f TB/s  ok=%s" % (label, us, mb, mb / us, ok), flush=True)
    return srcs


if __name__ == "__main__":
    run(D_JOBS, "D-step list")
    run(D_JOBS, "D-step list + BCE", bce=True)
    run([(16, 64)], "tiny + BCE", bce=True)
    srcs = run([(256, 24576)], "pool slab 256x24576")
    run([(64, 24576)], "pool slab 64x24576")
    run([(16, 64)], "tiny (launch floor)")
    x = srcs[0]
    out = torch.empty(24576, device=DEV)
    us = graph_time(lambda: torch.sum(x, 0, out=out))
    print("%-22s %8.2f us  %6.2f TB/s" % ("torch.sum(dim 0)", us, x.numel() * 4 / 1e6 / us), flush=True)
