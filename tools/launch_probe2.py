"""Which node kinds raise the per-launch floor inside a captured HIP graph."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
from sgan import kernels as K  # noqa: E402

n = 200
dev = "cuda"
x = torch.zeros(1024, device=dev)
z = torch.zeros(1024, device=dev)
xa = torch.randn(64, 32, device=dev)
wa = torch.randn(32, 16, device=dev)
ya = torch.empty(64, 16, device=dev)
pinned = torch.zeros(1024).pin_memory()


def add_chain():
    for _ in range(n):
        x.add_(1.0)


def alloc_chain():
    for _ in range(n):
        torch.zeros(1024, device=dev)


def copy_mix():
    for i in range(n):
        if i % 10 == 0:
            z.copy_(x)
        else:
            x.add_(1.0)


def sgg_chain():
    for _ in range(n):
        K.xw_raw(xa, wa, None, out=ya)


def cat_chain():
    for _ in range(n):
        torch.cat([x, z])


def mixed():
    for i in range(n // 4):
        x.add_(1.0)
        K.xw_raw(xa, wa, None, out=ya)
        torch.cat([x, z])
        torch.zeros(64, device=dev)


for name, f in (("add", add_chain), ("alloc", alloc_chain), ("copy_mix", copy_mix), ("sgg_xw", sgg_chain),
                ("cat", cat_chain), ("mixed", mixed)):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / (5 * n) * 1e6
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        f()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    gr = (time.perf_counter() - t0) / (10 * n) * 1e6
    print("%-9s eager %.2f us/launch  graph %.2f us/launch" % (name, eager, gr), flush=True)
