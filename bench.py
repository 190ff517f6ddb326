"""Benchmark: train-scenes/s of the group-aware Social-GAN hot path on MI355X.

One step = one reference training iteration (scripts/train.py defaults, GAT
generator): D-step + G-step (best_k = 20) with Adam updates, on a batch of
`--batch` synthetic 20-ped scenes per GPU (obs 8 / pred 12), inputs resident
in HBM before the timed region.  Multi-GPU: one process per GPU launched by
torch.distributed.run, scenes sharded (weak scaling), RCCL all-reduce of the
G/D gradients once per optimizer step.

Prints ONE JSON line (rank 0).  Extra objects:
  roofline     the dominant kernel (by summed device time over the timed
               steps, measured with HIP events on its launch stream) against
               the fp32 peak; `achieved` = algorithmic FLOP per launch / avg
               launch time (FLOP model in DESIGN.md);
  cpu_baseline the CPU oracle (reference formulation, per-scene loops) timed
               on this host for a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "scenes/sec (obs8/pred12, 20 peds) at 1/2/4/8 GPUs; ADE/FDE vs ref"
FP32_PEAK_TFLOPS = 157.3   # MI355X fp32 dense (vector == f32 MFMA), MI355X_MICROARCH.md


def build_models(seed, graph="gat"):
    from sgan.models import TrajectoryDiscriminator, TrajectoryGenerator
    torch.manual_seed(seed)
    g = TrajectoryGenerator(8, 12, embedding_dim=16, encoder_h_dim=32, decoder_h_dim=32, mlp_dim=64, num_layers=1,
                            noise_dim=(8,), noise_type="gaussian", noise_mix_type="global", pooling_type="pool_net",
                            pool_every_timestep=False, dropout=0.0, bottleneck_dim=8, batch_norm=False,
                            n_units=[40, 16, 40], n_heads=1, dropout1=0.0, alpha=0.2, graph=graph)
    d = TrajectoryDiscriminator(8, 12, embedding_dim=16, h_dim=48, mlp_dim=64, num_layers=1, batch_norm=False,
                                dropout=0.0, d_type="global")
    for m in list(g.modules()) + list(d.modules()):   # train.py:127-130 init_weights
        if isinstance(m, torch.nn.Linear):
            torch.nn.init.kaiming_normal_(m.weight)
    return g, d


def cpu_baseline(batch_scenes, n_peds, iters=2, threads=None):
    """Oracle (reference formulation) D-step + G-step on the host cores."""
    from oracle import sgan_oracle as O
    from sgan.data.synthetic import synthetic_batch
    threads = threads or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    g, d = O.build_default("gat")
    og = torch.optim.Adam(g.parameters(), lr=1e-4)
    od = torch.optim.Adam(d.parameters(), lr=1e-3)
    b = synthetic_batch([n_peds] * batch_scenes, seed=123)
    O.discriminator_step(O.Args, b, g, d, od)          # warm-up (not timed)
    t0 = time.perf_counter()
    for _ in range(iters):
        O.discriminator_step(O.Args, b, g, d, od)
        O.generator_step(O.Args, b, g, d, og)
    dt = time.perf_counter() - t0
    return {"value": round(batch_scenes * iters / dt, 3), "unit": "scenes/s", "cores": threads, "kind": "port",
            "sample": "%d train iterations (D-step + G-step, best_k=20) on %d x %d-ped synthetic scenes, oracle/"
                      "sgan_oracle.py reference formulation, torch CPU fp32, %d threads (%.1f s)"
                      % (iters, batch_scenes, n_peds, threads, dt)}


def pool_flops(sc, bn):
    """Algorithmic FLOP of one sgg_pool_fwd launch: per (i, j) pair 512 hidden
    units x (2 FMA for A.r + bn FMA for layer 2) = 512 * (4 + 2 bn)."""
    sizes = np.diff(sc.host_off)
    return float((sizes.astype(np.float64) ** 2).sum()) * 512.0 * (4 + 2 * bn)


def pmc_traffic(kname, key):
    """HBM bytes per launch of the roofline kernel from the committed PMC
    passes (profiles/r01_pool_traffic.json, written by tools/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench, with the
    gfx950 FETCH_SIZE x2 correction of MI355X_MICROARCH.md), or None when that
    file holds no entry for this exact launch shape."""
    path = os.path.join(ROOT, "profiles", "r01_pool_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        tab = json.load(f)
    ent = tab.get("%s|%s" % (kname, list(key)))
    return None if ent is None else ent["hbm_bytes"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="scenes per GPU")
    ap.add_argument("--peds", type=int, default=20)
    ap.add_argument("--graph-kind", dest="graph_kind", default="gat", choices=["gat", "gcn"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", type=int, default=1, help="capture the iteration in a HIP graph (1) or run eager (0)")
    ap.add_argument("--cpu-iters", type=int, default=2)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; SGG_BENCH_BACKEND=gloo (and more ranks than GPUs,
    # ranks sharing a device) is only for rehearsing the multi-rank path on a
    # one-GPU box -- the driver's runs use nccl (RCCL over xGMI)
    backend = os.environ.get("SGG_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from sgan import kernels as K
    from sgan.data.synthetic import synthetic_batch
    from sgan.scene import SceneIndex
    from sgan.train_step import DataParallel, GanTrainer, GraphedTrainer

    g, d = build_models(0, args.graph_kind)
    g, d = g.to(dev), d.to(dev)
    trainer = GanTrainer(g, d, dp=DataParallel(), capturable=bool(args.graph))
    # the reference feeds consecutive loader batches to the D-step and the
    # G-step (scripts/train.py:279-297): two distinct synthetic batches
    batch = synthetic_batch([args.peds] * args.batch, seed=1000 + rank, device=dev)
    batch_g = synthetic_batch([args.peds] * args.batch, seed=5000 + rank, device=dev)
    sc = SceneIndex.from_seq_start_end(batch[-1], dev)
    sc_g = SceneIndex.from_seq_start_end(batch_g[-1], dev)
    S_glob, B_glob = sc.S * world, sc.B * world
    kw = dict(S_global=S_glob, B_global=B_glob, shard=(rank * sc.S, (rank + 1) * sc.S))

    graphed = False
    if args.graph:
        try:
            gt = GraphedTrainer(trainer, batch, sc, warmup=2, batch_g=batch_g, sc_g=sc_g, **kw)
            step = gt.step
            graphed = True
        except Exception as e:  # capture unsupported (e.g. a collective): eager
            print("bench: graph capture failed (%s: %s); running eager" % (type(e).__name__, e), file=sys.stderr)
            torch.cuda.synchronize()
    if not graphed:
        step = lambda: trainer.step(batch, sc, batch_g, sc_g, **kw)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    # roofline of the pooling kernel: every sgg_pool_fwd launch of a few
    # instrumented iterations on the same inputs is recorded (graph replays
    # carry no events), then each distinct launch is re-issued back to back
    # between HIP events on its launch stream (device-busy average duration);
    # rocprofv3's kernel trace of the same command is the cross-check (profiles/)
    n_it = max(1, min(args.steps, 3))
    K.pool_timer.start()
    for _ in range(n_it):
        trainer.step(batch, sc, batch_g, sc_g, **kw)
    timed = K.pool_timer.replay(K.pool_timer.stop())

    if rank == 0:
        # dominant kernel: the pool forward launch with the most device time per iteration
        key = max(timed, key=lambda k: timed[k][0] * timed[k][2])
        n, fl, ms = timed[key]
        kname = "sgg::pool_fwd_kernel<%d, %d, %d>" % key[:3]
        achieved = fl / (ms * 1e-3) / 1e12
        roofline = {"bound": "mfma", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": pmc_traffic(kname, key),
                    "kernel": kname, "launches_per_iteration": round(n / n_it, 2),
                    "avg_launch_us": round(ms * 1e3, 2), "flop_per_launch": fl,
                    "note": "fp32 (f32 MFMA, same peak as VALU FMA); all pool forward launches per iteration "
                            "[bn, gpw, unroll, scenes, peds]: %s" % {
                                "%s" % list(k): {"per_iter": round(v[0] / n_it, 2), "avg_us": round(v[2] * 1e3, 2),
                                                 "TFLOP/s": round(v[1] / (v[2] * 1e-3) / 1e12, 2)}
                                for k, v in timed.items()}}
        ms_step = elapsed / args.steps * 1e3
        value = world * args.batch / (elapsed / args.steps)
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(args.batch, args.peds, iters=args.cpu_iters)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "scenes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic (random-init weights, SURVEY.md 8d recipe)",
            "config": {"workload": "train iteration = D-step + G-step (best_k=20, Adam) of the GAT generator "
                                   "(scripts/train.py defaults)", "scenes_per_gpu": args.batch,
                       "global_batch": args.batch * world, "peds_per_scene": args.peds, "obs_len": 8, "pred_len": 12,
                       "generator": args.graph_kind, "hip_graph": graphed, "parallelism": "dp%d" % world},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
