"""Device time of the step's small glue kernels at the bench shape (64 scenes
x 20 peds, T 12, best_k 20), each replayed 50x from a HIP graph.
usage: python tools/glue_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sgan import kernels as K  # noqa: E402
from sgan.scene import SceneIndex  # noqa: E402


def graph_time(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = "cuda"
    S, n, T, k = 64, 20, 12, 20
    B = S * n
    sc = SceneIndex(np.arange(0, B + 1, n), dev)
    gt = torch.randn(T, B, 2, device=dev)
    pred = torch.randn(T, k * B, 2, device=dev)
    mask = (torch.rand(B, T, device=dev) > 0.1).float()
    p = torch.randn(T, B, 2, device=dev)
    with torch.no_grad():
        print("l2_select   %6.2f us" % graph_time(lambda: K.l2_select(pred, gt, mask, sc, k)))
        print("l2_loss fwd %6.2f us" % graph_time(lambda: K.l2_loss(p, gt, mask, sc, 1.0)))
    for R, E in ((512, 64), (192, 16)):
        W, We, be = torch.randn(R, E, device=dev), torch.randn(E, 2, device=dev), torch.randn(E, device=dev)
        dA, db = torch.randn(R, 2, device=dev), torch.randn(R, device=dev)
        print("fold_bwd R=%d E=%d %6.2f us" % (R, E, graph_time(lambda: K.fold_bwd(W, We, be, dA, db))))
    sys.path.insert(0, ROOT)
    import bench
    g, d = bench.build_models(0)
    for name, mod, clip in (("G", g, 2.0), ("D", d, 0.0)):
        mod = mod.to(dev)
        ps = [q for q in mod.parameters() if q.requires_grad]
        for q in ps:
            q.grad = torch.randn_like(q) * 1e-2
        opt = K.ClipAdam(ps, lr=1e-4)
        opt.step(clip)   # state
        print("adam %s (%d tensors, %d floats, clip %.1f) %6.2f us" % (
            name, len(ps), sum(q.numel() for q in ps), clip, graph_time(lambda: opt.step(clip), reps=20)))
    x = torch.empty(1, device=dev)
    print("empty fill  %6.2f us" % graph_time(lambda: x.fill_(1.0)))


if __name__ == "__main__":
    main()
