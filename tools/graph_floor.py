"""Time the captured training iteration: full GraphedTrainer.step() (host RNG
draws + staging copies + replay) against bare graph.replay() back to back."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from sgan.data.synthetic import synthetic_batch  # noqa: E402
from sgan.scene import SceneIndex  # noqa: E402
from sgan.train_step import GanTrainer, GraphedTrainer  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
g, d = bench.build_models(0)
g, d = g.to(dev), d.to(dev)
tr = GanTrainer(g, d, capturable=True)
b1 = synthetic_batch([20] * S, seed=1, device=dev)
b2 = synthetic_batch([20] * S, seed=2, device=dev)
sc1 = SceneIndex.from_seq_start_end(b1[-1], dev)
sc2 = SceneIndex.from_seq_start_end(b2[-1], dev)
gt = GraphedTrainer(tr, b1, sc1, warmup=2, batch_g=b2, sc_g=sc2)
for _ in range(5):
    gt.step()
torch.cuda.synchronize()
n = 30
t0 = time.perf_counter()
for _ in range(n):
    gt.step()
torch.cuda.synchronize()
full = (time.perf_counter() - t0) / n * 1e3
t0 = time.perf_counter()
for _ in range(n):
    gt.graph.replay()
torch.cuda.synchronize()
bare = (time.perf_counter() - t0) / n * 1e3
t0 = time.perf_counter()
for _ in range(n):
    gt._load(*tr.draw_inputs(*gt.span))
torch.cuda.synchronize()
host = (time.perf_counter() - t0) / n * 1e3
print("S=%d  step %.3f ms  bare replay %.3f ms  host draw+stage %.3f ms  -> %.0f scenes/s" % (
    S, full, bare, host, S / full * 1e3), flush=True)
