"""Graph-replayed real-data training (BucketedGraphTrainer) alone, for a
rocprofv3 kernel trace: one untimed epoch pass (bucket captures), then
`iters` timed iterations over zara1 train, per-bucket iteration counts.
usage: python tools/realdata_graph_probe.py [iters] [gran] [pad_scenes] [np_caps]"""
import collections
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "group-gan-gcn-gat_amd")]
import bench  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    gran = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    pad = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    caps = tuple(int(x) for x in sys.argv[4].split(",")) if len(sys.argv) > 4 else (48, 64)
    dev = torch.device("cuda", 0)
    from sgan.data.device import DeviceLoader, DeviceTrajectoryDataset
    from sgan.data.trajectories_GCN import TrajectoryDataset
    from sgan.train_step import BucketedGraphTrainer, DataParallel, GanTrainer
    dd = DeviceTrajectoryDataset(TrajectoryDataset(os.path.join(ROOT, "tests", "golden", "datasets_group", "zara1",
                                                                "train")), dev)
    g, d = bench.build_models(0)
    tr = GanTrainer(g.to(dev), d.to(dev), dp=DataParallel(), capturable=True)
    bt = BucketedGraphTrainer(tr, dd, batch_size=64, pad_scenes=pad, gran=gran, np_caps=caps)

    def batches():
        while True:
            yield from DeviceLoader(dd, batch_size=64, shuffle=True).scene_batches()
    it = batches()
    for _ in range(len(dd) // 64 + 1):
        bt.step(next(it), next(it))
    torch.cuda.synchronize()
    used = collections.Counter()
    import gc
    gcs = [0]
    gc.callbacks.append(lambda phase, info: gcs.__setitem__(0, gcs[0] + (phase == "start")))
    caps0 = len(bt.buckets)
    t0 = time.perf_counter()
    marks = [t0]
    mono = [time.monotonic_ns()]   # (CLOCK_MONOTONIC: the clock of rocprofv3's host traces)
    info = []
    for _ in range(iters):
        sd, sg = next(it), next(it)
        used[bt.bucket_of(dd.layout(sd)[0], dd.layout(sg)[0])] += 1
        bt.step(sd, sg)
        marks.append(time.perf_counter())
        mono.append(time.monotonic_ns())
        info.append(bt.last)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    host = np.diff(marks) * 1e3
    if os.environ.get("SGG_PROBE_MARKS"):   # per-iteration host windows (tools/systrace_stall.py)
        import json
        with open(os.environ["SGG_PROBE_MARKS"], "w") as f:
            json.dump([{"index": i, "start_ns": mono[i], "end_ns": mono[i + 1], "host_ms": float(host[i]),
                        "bucket": (list(info[i][0]) if info[i][0] is not None else "eager"),
                        "prior_replays": info[i][1]} for i in range(iters)], f)
    print("host ms per iteration: median %.3f max %.3f; gc collections %d; buckets captured in the loop %d"
          % (np.median(host), host.max(), gcs[0], len(bt.buckets) - caps0))
    print("gran %d pad %d caps %s: %.3f ms / iteration, %.0f D-step scenes/s; buckets used %s"
          % (gran, pad, caps, dt / iters * 1e3, 64 * iters / dt, dict(used)), flush=True)
    if os.environ.get("SGG_PROBE_CPROFILE"):   # where the host's share of an iteration goes
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(iters):
            bt.step(next(it), next(it))
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
