"""Device time of the node-transform kernel (sgg_xw) over launch shapes:
HIP events around 200 back-to-back launches (graph-captured, so host launch
cost is out).  usage: python tools/xw_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "group-gan-gcn-gat_amd")]
from sgan import kernels as K  # noqa: E402


def time_it(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        for _ in range(reps):
            fn()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = "cuda"
    for M, Kd, N, tw in ((1280, 32, 512, True), (128, 32, 512, True), (64, 32, 64, True), (2560, 48, 512, True),
                         (2560, 48, 64, True), (25600, 32, 512, True), (1280, 64, 48, False)):
        x = torch.randn(M, Kd, device=dev)
        w = torch.randn(N, Kd, device=dev) if tw else torch.randn(Kd, N, device=dev)
        b = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev)
        us = time_it(lambda: K.xw_raw(x, w, b, trans_w=tw, act=1, out=y, prec="fp32"))
        mb = 4.0 * (M * Kd + Kd * N + M * N) / 1e6
        print("M %6d K %3d N %4d trans %d: %7.2f us  (%.2f MB, %.0f GB/s)" % (M, Kd, N, tw, us, mb, mb * 1e3 / us))
    # an empty-ish launch for the floor
    z = torch.zeros(1, device=dev)
    print("torch add_ (1 elem): %.2f us" % time_it(lambda: z.add_(1.0)))


if __name__ == "__main__":
    main()
