"""Host-side cost of one GraphedTrainer step at configs[1]: the host RNG
draws, the staging copies, the graph replay call, and the device time of a
replay, to see whether the step is bound by the host or the device.
usage: python tools/replay_probe.py [steps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "group-gan-gcn-gat_amd")]
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    trainer, batch, sc, batch_g, sc_g, kw = bench.setup(64, 20, 0, 1, dev, "gat")
    from sgan.train_step import GraphedTrainer
    gt = GraphedTrainer(trainer, batch, sc, warmup=2, batch_g=batch_g, sc_g=sc_g, **kw)
    for _ in range(10):
        gt.step()
    torch.cuda.synchronize()
    td = tl = tr = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        a = time.perf_counter()
        ins = trainer.draw_inputs(*gt.span)
        b = time.perf_counter()
        if gt.pair:   # one rank: the input copy is a node of the graph (GraphedTrainer.step)
            i = gt.cur
            gt.cur ^= 1
            if gt.done_ev[i] is not None:
                gt.done_ev[i].synchronize()
            for dst, src in zip(gt.stage[i], ins):
                if src is not None:
                    dst.copy_(src)
            c = time.perf_counter()
            gt.pair[i][0].replay()
            ev = torch.cuda.Event()
            ev.record()
            gt.done_ev[i] = ev
        else:
            gt._load(*ins)
            c = time.perf_counter()
            for g, _ in gt.segments:
                g.replay()
        d = time.perf_counter()
        td += b - a
        tl += c - b
        tr += d - c
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    print("per step: draws %.1f us, staging %.1f us, replay call %.1f us, wall %.1f us"
          % (td / steps * 1e6, tl / steps * 1e6, tr / steps * 1e6, wall * 1e6))
    # device time of back-to-back replays (inputs unchanged)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graphs = [g for g, _ in gt.pair] or [g for g, _ in gt.segments]
    for k in range(steps):
        if gt.pair:
            graphs[k % 2].replay()
        else:
            for g in graphs:
                g.replay()
    e1.record()
    e1.synchronize()
    print("back-to-back replays only: %.1f us / step" % (e0.elapsed_time(e1) / steps * 1e3))


if __name__ == "__main__":
    main()
