"""Worker of test_gpu_zz_multiprocess.test_rccl_world1_dp_path (one process,
launched by the test with RANK=0 / WORLD_SIZE=1): the data-parallel code path
on the one GPU of a lease through RCCL, set up exactly as bench.py sets up
N > 1 -- a gloo process group for host control (barrier, timing max) and the
gradient all-reduces on sgan.rccl's own communicator (transport "rccl", the
id exchanged through the rendezvous store).  No ProcessGroupNCCL exists in
the process, so no watchdog thread polls events while graphs are captured
(the round-5 abort).

  eager     eager steps, DataParallel(exercise=True): one flat RCCL SUM
            all-reduce per optimizer step, world size 1
  captured  GraphedTrainer, the all-reduces CAPTURED in the HIP graph
            (capture=True: one graph per replay), 1- and 2-iteration graphs
  segmented GraphedTrainer cut at each all-reduce (capture=False: the RCCL
            all-reduces eager between graph segments)

An RCCL SUM over one rank is the identity, so each must equal the same
execution form without DP bitwise (losses and every parameter).  The
sequence is run SGG_W1_ROUNDS times (default 3) in the one process, so a
hazard that depends on timing gets several chances to show.  Prints one JSON
line with the eager all-reduce time per iteration, then "rank 0 OK"."""
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
        dp = DataParallel(transport="pg")           # world 1, not exercised: no collective at all
        assert not dp.collective
    else:
        dp = DataParallel(exercise=True, transport="rccl", capture=dp_kind == "captured")
        assert dp.collective and dp.transport == "rccl"
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
    """HIP events around the two flat buckets' all-reduces (G, D), eager, on
    the communicator the steps use."""
    nums = [sum(p.numel() for p in ps) + 3 for ps in (tr.g_params, tr.d_params)]
    bufs = [torch.ones(n, device="cuda") for n in nums]
    comm = tr.dp.rccl
    for b in bufs:
        comm.allreduce_sum_(b)
    torch.cuda.synchronize()
    assert all(bool((b == 1).all()) for b in bufs), "an RCCL SUM over one rank is the identity"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        for b in bufs:
            comm.allreduce_sum_(b)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps, nums


def main():
    from sgan import rccl
    from sgan.train_step import DataParallel
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    assert dist.get_world_size() == 1 and dist.get_backend() == "gloo"
    dp0 = DataParallel(exercise=True, transport="rccl")
    assert dp0.capture, "the rccl transport's default is the captured form"
    sizes = [20, 7, 13, 20, 2, 9]
    out = {}
    tr = None
    for rnd in range(int(os.environ.get("SGG_W1_ROUNDS", "3"))):
        for graphed, iters, kinds in ((False, 1, ("captured",)), (True, 1, ("captured", "segmented")),
                                      (True, 2, ("captured",))):
            ref_l, ref_w, _ = run("none", graphed, iters, sizes)
            for kind in kinds:
                l, w, tr = run(kind, graphed, iters, sizes)
                name = "%s%s" % ("graph%d_" % iters if graphed else "eager_", kind if graphed else "dp")
                assert l == ref_l, (rnd, name, l, ref_l)
                for k in ref_w:
                    assert torch.equal(w[k], ref_w[k]), (rnd, name, k, (w[k] - ref_w[k]).abs().max().item())
                out[name] = "bitwise == the same form without DP"
        out["rounds"] = rnd + 1
    us, nums = allreduce_us(tr)
    out["allreduce_us_per_iter"] = round(us, 2)
    out["bucket_floats"] = nums
    del tr
    import gc
    gc.collect()                 # the graphs that captured the all-reduce are gone before the communicator
    torch.cuda.synchronize()
    dist.barrier()
    rccl.release()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    print("rank 0 OK", flush=True)


if __name__ == "__main__":
    main()
