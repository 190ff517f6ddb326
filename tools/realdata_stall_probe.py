"""Where a slow real-data iteration's host time goes: BucketedGraphTrainer
over zara1 train (one untimed epoch of bucket captures), then `iters` timed
iterations with BucketedGraphTrainer.step's phases and every
PaddedScenes.load timed, each with the thread's minor page faults (getrusage
RUSAGE_THREAD).  Prints every iteration over 2 ms.  (Round 5 found the ~7 ms
stall, 4105 faults, inside the host-issued scene-structure copy of load();
that copy is now a node of the replayed graph.)
usage: python tools/realdata_stall_probe.py [iters]"""
import os
import resource
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "group-gan-gcn-gat_amd")]
import bench  # noqa: E402


def flt():
    return resource.getrusage(resource.RUSAGE_THREAD).ru_minflt


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    dev = torch.device("cuda", 0)
    from sgan.data.device import DeviceLoader, DeviceTrajectoryDataset
    from sgan.data.trajectories_GCN import TrajectoryDataset
    from sgan import scene as SC
    from sgan.train_step import BucketedGraphTrainer, DataParallel, GanTrainer
    rec = []
    orig = SC.PaddedScenes.load

    def load(self, host_off_real, rows_real, graph_stage=None):
        t0, f0 = time.perf_counter(), flt()
        orig(self, host_off_real, rows_real, graph_stage=graph_stage)
        rec.append(((time.perf_counter() - t0) * 1e3, flt() - f0, graph_stage))

    SC.PaddedScenes.load = load
    dd = DeviceTrajectoryDataset(TrajectoryDataset(os.path.join(ROOT, "tests", "golden", "datasets_group", "zara1",
                                                                "train")), dev)
    g, d = bench.build_models(0)
    tr = GanTrainer(g.to(dev), d.to(dev), dp=DataParallel(), capturable=True)
    bt = BucketedGraphTrainer(tr, dd, batch_size=64)

    def batches():
        while True:
            yield from DeviceLoader(dd, batch_size=64, shuffle=True).scene_batches()
    it = batches()
    for _ in range(len(dd) // 64 + 1):
        bt.step(next(it), next(it))
    torch.cuda.synchronize()
    from sgan import kernels as K
    slow, host = [], []
    with K.gc_frozen():
        for n in range(iters):
            del rec[:]
            f0 = flt()
            t0 = time.perf_counter()
            bt.step(next(it), next(it))
            ms = (time.perf_counter() - t0) * 1e3
            host.append(ms)
            if ms > 2.0:
                slow.append((n, ms, flt() - f0, bt.phase_ms, [list(r) for r in rec]))
        torch.cuda.synchronize()
    host = np.array(host)
    print("iters %d host ms median %.3f max %.3f, %d over 2 ms"
          % (iters, np.median(host), host.max(), len(slow)), flush=True)
    for n, ms, fl, ph, r in slow:
        print("  it %3d %.2f ms faults %d phases %s" % (n, ms, fl, None if ph is None else [round(x, 2) for x in ph]))
        for k, (a, b, gs) in enumerate(r):
            print("     load %d (graph stage %s): %.2f ms, %d faults" % (k, gs, a, b))


if __name__ == "__main__":
    main()
