"""Worker of test_gpu_configs.test_nccl_world1_dp_path (one process, launched
by the test with RANK=0 / WORLD_SIZE=1): the data-parallel code path on the
one GPU of a lease through RCCL (backend "nccl", device_id bound).

  eager     eager steps, DataParallel(exercise=True): one flat RCCL SUM
            all-reduce per optimizer step, world size 1
  captured  GraphedTrainer, the all-reduces CAPTURED in the HIP graph
            (DataParallel capture=True: one graph per replay, the
            all-reduce through sgan.rccl.RcclComm), 1- and 2-iteration
            graphs
  segmented GraphedTrainer cut at each all-reduce (capture=False: the
            collectives eager between graph segments, the form gloo needs)

An RCCL SUM over one rank is the identity, so each must equal the same
execution form without DP bitwise (losses and every parameter).  Prints "OK" and one JSON line with
the eager all-reduce time per iteration."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from _dp_graph_worker import models, weights  # noqa: E402

ITERS = 3


def run(dp_kind, graphed, iters, sizes):
    """dp_kind: "none" | "captured" | "segmented" (DP exercised at world 1)."""
    from sgan.data.synthetic import synthetic_batch
    from sgan.scene import SceneIndex
    from sgan.train_step import DataParallel, GanTrainer, GraphedTrainer
    g, d = models()
    if dp_kind == "none":
        dp = DataParallel()
        dp.on, dp.world, dp.rank, dp.exercise, dp.capture = False, 1, 0, False, False
    else:
        dp = DataParallel(exercise=True, capture=dp_kind == "captured")
        assert dp.collective and dist.get_backend() == "nccl"
    tr = GanTrainer(g, d, dp=dp, capturable=True)
    batch = synthetic_batch(sizes, seed=3, device="cuda")
    batch_g = synthetic_batch(sizes, seed=4, device="cuda")
    sc = SceneIndex(np.concatenate([[0], np.cumsum(sizes)]), "cuda")
    scg = SceneIndex(np.concatenate([[0], np.cumsum(sizes)]), "cuda")
    torch.manual_seed(9)
    random.seed(9)
    if not graphed:
        for _ in range(ITERS):
            ld, lg = tr.step(batch, sc, batch_g, scg)
    else:
        gt = GraphedTrainer(tr, batch, sc, warmup=1, batch_g=batch_g, sc_g=scg, iters=iters)
        if dp_kind == "segmented":
            assert len(gt.segments) == 3, len(gt.segments)
        else:
            assert gt.pair and not gt.segments, "collective not captured in the graph"
        for _ in range((ITERS - 1) // iters):
            ld, lg = gt.step()
    torch.cuda.synchronize()
    return {k: float(v) for k, v in list(ld.items()) + list(lg.items())}, weights(g, d), tr


def allreduce_us(tr, reps=20):
    """HIP events around the two flat buckets' all-reduces (G, D), eager."""
    nums = [sum(p.numel() for p in ps) + 3 for ps in (tr.g_params, tr.d_params)]
    bufs = [torch.ones(n, device="cuda") for n in nums]
    for b in bufs:
        dist.all_reduce(b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        for b in bufs:
            dist.all_reduce(b)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps, nums


def main():
    from sgan.train_step import DataParallel
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    assert DataParallel(exercise=True).capture, "nccl default is the captured form"
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    sizes = [20, 7, 13, 20, 2, 9]
    out = {}
    tr = None
    for graphed, iters, kinds in ((False, 1, ("captured",)), (True, 1, ("captured", "segmented")),
                                  (True, 2, ("captured",))):
        ref_l, ref_w, _ = run("none", graphed, iters, sizes)
        for kind in kinds:
            l, w, tr = run(kind, graphed, iters, sizes)
            name = "%s%s" % ("graph%d_" % iters if graphed else "eager_", kind if graphed else "dp")
            assert l == ref_l, (name, l, ref_l)
            for k in ref_w:
                assert torch.equal(w[k], ref_w[k]), (name, k, (w[k] - ref_w[k]).abs().max().item())
            out[name] = "bitwise == the same form without DP"
    us, nums = allreduce_us(tr)
    out["allreduce_us_per_iter"] = round(us, 2)
    out["bucket_floats"] = nums
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    print("rank 0 OK", flush=True)


if __name__ == "__main__":
    main()
