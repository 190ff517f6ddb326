"""Host-side profile (cProfile) of bench.py's real-data leg, device data path:
where an eager training iteration over zara1 train batches spends its time.
usage: python tools/realdata_profile.py [iters]"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "group-gan-gcn-gat_amd")]
import bench  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    from sgan.data.device import DeviceLoader, DeviceTrajectoryDataset
    from sgan.data.trajectories_GCN import TrajectoryDataset
    from sgan.train_step import DataParallel, GanTrainer
    dset = TrajectoryDataset(os.path.join(ROOT, "tests", "golden", "datasets_group", "zara1", "train"))
    dd = DeviceTrajectoryDataset(dset, dev)
    g, d = bench.build_models(0)
    tr = GanTrainer(g.to(dev), d.to(dev), dp=DataParallel(), capturable=True)

    def batches():
        while True:
            yield from DeviceLoader(dd, batch_size=64, shuffle=True)
    it = batches()
    from sgan import kernels as K
    for w in range(3):
        (bd, scd), (bg, scg) = next(it), next(it)
        K.GATENC_FUSED = w != 0 and os.environ.get("SGG_GATENC_FUSED", "1") != "0"   # warm the per-layer path too
        tr.d_step(bd, scd)
        tr.g_step(bg, scg)
    K.GATENC_FUSED = os.environ.get("SGG_GATENC_FUSED", "1") != "0"
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    st0 = torch.cuda.memory_stats()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(iters):
        (bd, scd), (bg, scg) = next(it), next(it)
        tr.d_step(bd, scd)
        tr.g_step(bg, scg)
    torch.cuda.synchronize()
    pr.disable()
    print("%.3f ms / iteration" % ((time.perf_counter() - t0) / iters * 1e3))
    st1 = torch.cuda.memory_stats()
    for k in ("num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams"):
        print("%s: %d" % (k, st1.get(k, 0) - st0.get(k, 0)))
    pstats.Stats(pr).sort_stats("tottime").print_stats(12)
    pstats.Stats(pr).sort_stats("cumtime").print_stats(30)


if __name__ == "__main__":
    main()
