"""Benchmark: train-scenes/s of the group-aware Social-GAN hot path on MI355X.

One step = one reference training iteration (scripts/train.py defaults, GAT
generator): D-step + G-step (best_k = 20) with Adam updates, on synthetic
20-ped scenes (obs 8 / pred 12), inputs resident in HBM before the timed
region.

  N = 1 (default): BASELINE configs[1]'s shape, 64 scenes on one GPU.
  N > 1: BASELINE configs[3], the 4096-scene global batch split over the N
         GPUs (4096 / N scenes per GPU, strong scaling): one process per GPU
         (`--gpus N` spawns them through torch.distributed.run when it is
         not already running under it), scenes sharded, RCCL all-reduce of the
         G / D gradients once per optimizer step.  The N = 1 line carries the
         same 4096-scene workload on one GPU as `scaling_reference`, the
         denominator of that strong-scaling curve.

Prints ONE JSON line (rank 0).  Extra objects:
  kernels      every instrumented kernel's device time per iteration
               (HIP events on its launch stream, LaunchTimer in sgan/kernels.py);
  roofline     the dominant one (most device time per iteration) against its
               bound: the fp32 MFMA peak when its arithmetic intensity is
               above the ridge, HBM otherwise; `achieved` = algorithmic FLOP
               (or bytes) per launch / average launch time (work models in
               DESIGN.md section 4); `traffic` = PMC-measured HBM bytes per
               launch of that kernel (profiles/, tools/pmc_traffic.py);
  cpu_baseline the CPU oracle (reference formulation) timed on this host for a
               bounded sample of the same workload, validated against the
               real reference in the build container (ref_cpu_timing.json);
               the host's core count and CPU model beside it;
  legs         (N = 1) the other BASELINE configurations on one GPU, each with
               its own dominant kernel and roofline: configs[2]'s GCN
               generator (fp32 and bf16), configs[4]'s sgangat generator on
               64-ped scenes (bf16), and configs[3]'s per-GPU shard at N = 8
               (512 scenes).
"""
import argparse
import glob
import json
import os
import socket
import subprocess
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
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E, MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0  # MI355X bf16 dense MFMA (no sparsity), MI355X_MICROARCH.md
RIDGE = FP32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)   # FLOP / byte
TRANSPORT = ["rccl"]       # DataParallel transport of the N > 1 runs (main)
CONFIG4_GLOBAL = 4096      # BASELINE configs[3]: synthetic 20-ped, batch 4096, 8 x MI355X
GRAPH_ITERS = int(os.environ.get("SGG_GRAPH_ITERS", "4"))   # iterations per HIP-graph replay (one rank)
# one rank: the G-step's prefix graph beside the D-step graph on a second
# stream (GraphedTrainer(overlap=True))
OVERLAP = os.environ.get("SGG_OVERLAP", "0") == "1"
# PMC traffic tables (tools/pmc_traffic.py), every round's, newest first
# (rNN[_x]_pmc_traffic.json sorts by round, then by the round's run letter)
TRAFFIC_TABLES = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_pmc_traffic.json")), reverse=True)
# the reference's CPU path, train iteration at batch 64, 8 threads (the survey container)
REFERENCE_CPU_SCENES_S = 13.9

# the BASELINE configurations measured beside the headline at N = 1 (one GPU each)
LEGS = {
    "configs1": dict(per_gpu=64, peds=20, graph="gat", prec="fp32",
                     what="BASELINE configs[1] shape: 64 synthetic 20-ped scenes, GAT generator, fp32"),
    "configs3_shard512": dict(per_gpu=512, peds=20, graph="gat", prec="fp32",
                              what="configs[3]'s per-GPU shard at N = 8 (4096 / 8 = 512 scenes), GAT, fp32"),
    "configs2_gcn_fp32": dict(per_gpu=64, peds=20, graph="gcn", prec="fp32",
                              what="configs[2]'s GCN generator (sgan-g-p family), 64 scenes, fp32"),
    "configs2_gcn_bf16": dict(per_gpu=64, peds=20, graph="gcn", prec="bf16",
                              what="configs[2]'s GCN generator, 64 scenes, bf16 node transforms (fp32 accumulate)"),
    "configs4_sgangat_bf16": dict(per_gpu=64, peds=64, graph="sgangat", prec="bf16",
                                  what="configs[4]'s sgangat generator (sgangat-g-p family) on 64-ped scenes, "
                                       "64 scenes, bf16 node transforms (fp32 accumulate)"),
}


def build_models(seed, graph="gat"):
    from sgan.models import TrajectoryDiscriminator, TrajectoryGenerator
    torch.manual_seed(seed)
    g = TrajectoryGenerator(8, 12, embedding_dim=16, encoder_h_dim=32, decoder_h_dim=32, mlp_dim=64, num_layers=1,
                            noise_dim=(8,), noise_type="gaussian", noise_mix_type="global", pooling_type="pool_net",
                            pool_every_timestep=False, dropout=0.0, bottleneck_dim=8, batch_norm=False,
                            n_units=[40, 16, 40], n_heads=[4, 1] if graph == "sgangat" else 1, dropout1=0.0,
                            alpha=0.2, graph=graph)
    d = TrajectoryDiscriminator(8, 12, embedding_dim=16, h_dim=48, mlp_dim=64, num_layers=1, batch_norm=False,
                                dropout=0.0, d_type="global")
    for m in list(g.modules()) + list(d.modules()):   # train.py:127-130 init_weights
        if isinstance(m, torch.nn.Linear):
            torch.nn.init.kaiming_normal_(m.weight)
    return g, d


def host_cpus():
    """(logical CPUs of the machine, CPUs this process may use, CPU model):
    the affinity mask, further bounded by a cgroup CPU quota when one is set
    (a GPU box's share of a large host)."""
    total = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            usable = max(1, min(usable, int(-(-int(q) // int(per)))))
    except (OSError, ValueError):
        pass
    model = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return total, usable, model


def cpu_baseline(batch_scenes, n_peds, iters=2, threads=None):
    """Oracle (reference formulation) D-step + G-step on the host cores: every
    CPU this process may use (torch.set_num_threads)."""
    from oracle import sgan_oracle as O
    from sgan.data.synthetic import synthetic_batch
    total, usable, model = host_cpus()
    threads = threads or usable
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
    val = ""
    vpath = os.path.join(ROOT, "tests", "golden", "ref_cpu_timing.json")
    if os.path.exists(vpath):
        v = json.load(open(vpath))
        val = ("; validated in the build container (%s, %d threads, batch %d): reference %.2f vs oracle %.2f "
               "scenes/s, ratio %.2f (tests/golden/ref_cpu_timing.json)"
               % (v.get("cpu", "?"), v["threads"], v["batch"], v["reference_scenes_per_s"],
                  v["oracle_scenes_per_s"], v["oracle_over_reference"]))
    return {"value": round(batch_scenes * iters / dt, 3), "unit": "scenes/s", "cores": threads, "kind": "port",
            "host_cores": total, "usable_cpus": usable, "cpu_model": model,
            "sample": "%d train iterations (D-step + G-step, best_k=20) on %d x %d-ped synthetic scenes, oracle/"
                      "sgan_oracle.py reference formulation, torch CPU fp32, %d threads = every CPU this process may "
                      "use (host: %d logical CPUs, %s) (%.1f s)%s"
                      % (iters, batch_scenes, n_peds, threads, total, model, dt, val)}


def traffic_lookup(name, key):
    """HBM bytes per launch of (kernel, launch shape) from the committed PMC
    tables (tools/pmc_traffic.py: separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this bench with the gfx950 corrections of
    MI355X_MICROARCH.md), newest table first -> (bytes, source): the exact
    launch shape when a PMC run re-issued it (--pmc-target), else None."""
    for path in TRAFFIC_TABLES:
        if not os.path.exists(path):
            continue
        tab = json.load(open(path))
        ent = tab.get("%s|%s" % (name, list(key[1:])))
        if ent is not None:
            return ent["hbm_bytes"], "PMC bytes of this launch shape, %s (%s)" % (
                os.path.basename(path), ent.get("note", "re-issued %s x" % ent.get("dispatches", 0)))
    return None, None


def kernel_table(timed, n_it):
    """{name: per-iteration stats} from LaunchTimer.replay records."""
    agg = {}
    for key, r in timed.items():
        a = agg.setdefault(r["name"], dict(us_per_iter=0.0, launches_per_iter=0.0, flop=0.0, bytes=0.0, shapes=[]))
        per_it = r["launches"] / n_it
        a["us_per_iter"] += per_it * r["ms"] * 1e3
        a["launches_per_iter"] += per_it
        a["flop"] += per_it * r["flop"]
        a["bytes"] += per_it * r["bytes"]
        a["shapes"].append((key, r, per_it))
    return agg


def main_launch(a):
    """The kernel's main launch shape: the most algorithmic work per
    iteration (bytes, then FLOP) -- not a timing, so that separate processes
    (the two PMC passes, the bench) pick the same shape."""
    return max(a["shapes"], key=lambda s: (s[2] * s[1]["bytes"], s[2] * s[1]["flop"]))


def _steps_of(name, key):
    """Serial recurrence steps of one launch of a sequence kernel (the LSTM
    families: the launch key's first field is the step count T), else None."""
    if "lstm" in name and len(key) > 1 and isinstance(key[1], int):
        return key[1]
    return None


def roofline_of(name, a):
    """The kernel against its roof, per launch of its MAIN launch shape (the
    one the PMC passes re-issue, main_launch): achieved = that launch's
    algorithmic FLOP (or bytes) / its average device time, traffic = PMC
    bytes of that same launch -- so traffic / algorithmic_bytes is a re-read
    factor of one launch.

    bound: the roof the launch's arithmetic intensity points at ("mfma"
    above the ridge, "hbm" below) -- unless the launch runs far from both
    roofs because its time is a dependency chain: "latency" when the time
    per launch stays > 4x its roofline time and either (a) it is a serial
    recurrence (T dependent steps: the LSTM families; `latency.us_per_step`)
    or (b) another launch shape of the kernel with at most 2/3 of the work
    takes > 0.8x the time (the time does not follow the work).  frac is
    then roofline time / measured time: max(FLOP / FLOP peak, bytes / HBM
    peak) over the launch's duration, i.e. achieved / peak of the nearer
    roof."""
    key, r, per_it = main_launch(a)
    us = r["ms"] * 1e3
    fl, by = r["flop"], r["bytes"]
    ai = fl / max(by, 1.0)
    # a bf16-MFMA kernel (the opt-in precision) is priced at the dense bf16 peak
    bf16 = "bf16" in name or ("gcnmod" in name and "<true>" in name)
    fpeak = BF16_PEAK_TFLOPS if bf16 else FP32_PEAK_TFLOPS
    t_f, t_b = fl / (fpeak * 1e12), by / (HBM_PEAK_GBS * 1e9)
    t_roof = max(t_f, t_b)
    steps = _steps_of(name, key)
    evidence = None
    for k2, r2, _ in a["shapes"]:
        w1, w2 = max(fl / fpeak / 1e3, by / HBM_PEAK_GBS), max(r2["flop"] / fpeak / 1e3, r2["bytes"] / HBM_PEAK_GBS)
        if k2 != key and w2 <= w1 * 2.0 / 3.0 and r2["ms"] * 1e3 > 0.8 * us:
            evidence = "%s %s: %.2fx the work in %.2fx the time" % (name, list(k2[1:]), w2 / w1, r2["ms"] * 1e3 / us)
    latency = us * 1e-6 > 2.0 * t_roof and (steps is not None or evidence is not None)
    if t_f >= t_b:
        achieved, peak, unit = fl / (us * 1e-6) / 1e12, fpeak, "TFLOP/s"
    else:
        achieved, peak, unit = by / (us * 1e-6) / 1e9, HBM_PEAK_GBS, "GB/s"
    bound = "latency" if latency else ("mfma" if t_f >= t_b else "hbm")
    traffic = traffic_lookup(name, key)
    out = {"bound": bound, "achieved": round(achieved, 3), "peak": peak, "unit": unit,
           "frac": round(achieved / peak, 4), "traffic": traffic[0],
           "kernel": name, "launch": list(key[1:]), "avg_launch_us": round(us, 2),
           "launches_per_iteration": round(a["launches_per_iter"], 2), "us_per_iteration": round(a["us_per_iter"], 1),
           "flop_per_launch": fl, "algorithmic_bytes_per_launch": by,
           "traffic_over_algorithmic": round(traffic[0] / by, 3) if traffic[0] else None,
           "traffic_source": traffic[1], "arithmetic_intensity": round(ai, 2), "ridge": round(RIDGE, 2)}
    if latency:
        out["latency"] = {"roofline_us": round(t_roof * 1e6, 3), "us_per_step": round(us / steps, 3) if steps else None,
                          "steps": steps, "time_vs_work": evidence,
                          "note": "a dependency chain, not bandwidth or MFMA throughput: frac = roofline time / "
                                  "measured time (achieved / peak of the nearer roof)"}
    return out


# the reference's work per 20-ped scene and training
# iteration (D-step 0.42 + G-step 1.87 GFLOP; context x 20, the unfolded
# pooling MLP, every sample's backward)
REFERENCE_FLOP_PER_SCENE = 2.29e9


def iteration_roofline(agg, ms_step, scenes):
    """The whole iteration against the roofline, from the executed-work model:
    every instrumented launch's algorithmic FLOP and bytes (the work models
    the per-kernel table divides by).  A launch cannot
    finish faster than max(FLOP / fp32 peak, bytes / HBM peak); the sum of
    those bounds over the iteration's launches is its roofline time, and
    frac = roofline time / measured time per iteration."""
    fl = by = t_roof = t_meas = 0.0
    for a in agg.values():
        for _key, r, per_it in a["shapes"]:
            fl += per_it * r["flop"]
            by += per_it * r["bytes"]
            t_roof += per_it * max(r["flop"] / (FP32_PEAK_TFLOPS * 1e12), r["bytes"] / (HBM_PEAK_GBS * 1e9))
            t_meas += per_it * r["ms"] * 1e-3
    t = ms_step * 1e-3
    return {"flop": fl, "bytes": by, "flop_per_scene": fl / scenes,
            "achieved_tflops": round(fl / t / 1e12, 3), "achieved_gbs": round(by / t / 1e9, 1),
            "roofline_us": round(t_roof * 1e6, 2), "instrumented_device_us": round(t_meas * 1e6, 1),
            "measured_us": round(t * 1e6, 1), "frac": round(t_roof / t, 4),
            "reference_flop_per_scene": REFERENCE_FLOP_PER_SCENE,
            "reference_equivalent_tflops": round(REFERENCE_FLOP_PER_SCENE * scenes / t / 1e12, 2),
            "note": "executed-work model: the algorithmic FLOP / bytes of every instrumented launch of one iteration "
                    "(the per-kernel work models); roofline_us = sum over launches of max(FLOP / 157.3 TFLOP/s, "
                    "bytes / 8 TB/s); frac = roofline_us / measured_us.  The reference's own work (2.29 GFLOP per "
                    "scene, SURVEY.md 8d) is larger: the build computes the context once instead of best_k times, "
                    "folds the input embeddings, rolls out the best_k samples without autograd and skips discarded "
                    "gradients (DESIGN.md section 4, executed-work model); reference_equivalent_tflops is that work "
                    "over the measured time (above the fp32 peak because of those de-duplications)"}


def host_sched():
    """(run-queue wait of this thread in ns, the cgroup's throttled time in
    us, this thread's rusage: CPU s, minor / major page faults, voluntary /
    involuntary context switches) -- None where the kernel does not expose it."""
    import resource
    wait = thr = None
    try:
        ru = resource.getrusage(resource.RUSAGE_THREAD)
        ru = (ru.ru_utime + ru.ru_stime, ru.ru_minflt, ru.ru_majflt, ru.ru_nvcsw, ru.ru_nivcsw)
    except (AttributeError, OSError):
        ru = None
    try:
        wait = int(open("/proc/thread-self/schedstat").read().split()[1])
    except (OSError, ValueError, IndexError):
        pass
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            if line.startswith("throttled_usec"):
                thr = int(line.split()[1])
    except (OSError, ValueError):
        pass
    return wait, thr, ru


def real_data_leg(dev, iters=20, warmup=3, batch=64):
    """configs[1] on REAL data: training iterations over the zara1 train split
    (tests/golden/datasets_group/zara1/train, the reference's datasets_group
    files), batch 64, consecutive loader batches to the D-step and the G-step
    (scripts/train.py:279-297).  Three paths:
      graphed  HIP-graph replays through BucketedGraphTrainer: each batch
               pair padded into a capacity bucket whose iteration was captured
               once (the captures happen in an untimed first pass over the
               epoch; a capture leaves the training state unchanged);
      device   eager iterations, batches from the device-resident data path
               (the split in HBM, one gather launch per batch);
      host     eager iterations, the host DataLoader + .cuda() copies.
    The rate counts the D-step's scenes; the G-step consumes the next loader
    batch, so the loader delivers twice as many scenes per iteration."""
    from sgan.data.device import DeviceLoader, DeviceTrajectoryDataset
    from sgan.data.trajectories_GCN import TrajectoryDataset, seq_collate
    from sgan.scene import SceneIndex
    from sgan.train_step import BucketedGraphTrainer, DataParallel, GanTrainer
    from torch.utils.data import DataLoader
    path = os.path.join(ROOT, "tests", "golden", "datasets_group", "zara1", "train")
    if not os.path.isdir(path):
        return None
    dset = TrajectoryDataset(path)
    dd = DeviceTrajectoryDataset(dset, dev)
    out = {}
    for mode in ("graphed", "device", "host"):
        g, d = build_models(0)
        tr = GanTrainer(g.to(dev), d.to(dev), dp=DataParallel(), capturable=True)
        bt = BucketedGraphTrainer(tr, dd, batch_size=batch) if mode == "graphed" else None

        def batches():
            while True:
                if mode == "graphed":
                    yield from DeviceLoader(dd, batch_size=batch, shuffle=True).scene_batches()
                elif mode == "device":
                    yield from DeviceLoader(dd, batch_size=batch, shuffle=True)
                else:
                    for b in DataLoader(dset, batch_size=batch, shuffle=True, collate_fn=seq_collate):
                        yield ([t.to(dev, non_blocking=True) for t in b[:-1]] + [b[-1]],
                               SceneIndex.from_seq_start_end(b[-1], dev))
        it = batches()
        from sgan import kernels as K
        t_cap = time.perf_counter()
        n_warm = (len(dd) // batch + 1) if mode == "graphed" else warmup   # graphed: an epoch (every bucket)
        for w in range(n_warm):
            if mode == "graphed":
                bt.step(next(it), next(it))
                continue
            (bd, scd), (bg, scg) = next(it), next(it)
            # one warm-up iteration on the per-layer GAT path too: real batches
            # with a scene beyond the fused encoder's LDS plan take it, and the
            # first launch of each of its kernels loads a code object (tens of ms)
            K.GATENC_FUSED = w != 0
            try:
                tr.d_step(bd, scd)
                tr.g_step(bg, scg)
            finally:
                K.GATENC_FUSED = True
        torch.cuda.synchronize()
        t_cap = time.perf_counter() - t_cap
        # the captured graphs' state out of the collector's scans, scoped to the
        # timed loop (unfrozen on any exit, kernels.gc_frozen)
        with K.gc_frozen():
            # (the instrumentation's own set-up -- the allocator statistics, the
            # first scheduler sample -- comes before the clock starts: it was
            # ~1.2 ms of the first timed iteration)
            allocs0 = torch.cuda.memory_stats(dev).get("num_device_alloc")
            # host-side diagnostics per iteration: the thread's run-queue wait
            # (/proc/thread-self/schedstat: time runnable but not running) and the
            # cgroup's CPU-quota throttling (cpu.stat throttled_usec) -- a host
            # stall that is neither Python nor HIP shows up in one of them
            sched = [host_sched()]
            phases = []
            steps_info = []
            # HIP events between the iterations on the launch stream: each
            # iteration's device-side span (host timings alone cannot tell a host
            # stall from the host waiting on a device that is behind)
            evs = [torch.cuda.Event(enable_timing=True)]
            t0 = time.perf_counter()
            scenes = 0
            marks = [t0]
            evs[0].record()
            for _ in range(iters):
                if mode == "graphed":
                    tn = time.perf_counter()
                    sd, sg = next(it), next(it)
                    tn = (time.perf_counter() - tn) * 1e3
                    bt.step(sd, sg)
                    phases.append((tn,) + (bt.phase_ms or (None, None, None)))
                    steps_info.append(bt.last)
                    evs.append(torch.cuda.Event(enable_timing=True))
                    evs[-1].record()
                    sched.append(host_sched())
                    scenes += len(sd)
                else:
                    (bd, scd), (bg, scg) = next(it), next(it)
                    tr.d_step(bd, scd)
                    tr.g_step(bg, scg)
                    scenes += scd.S
                marks.append(time.perf_counter())
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        # host-side iteration times (eager issue is host-bound; a first-use
        # stall -- a kernel's code object loaded at its first launch -- is an outlier)
        per = sorted(b - a for a, b in zip(marks, marks[1:]))
        out[mode] = {"value": round(scenes / dt, 2), "ms_per_iteration": round(dt / iters * 1e3, 3),
                     "host_ms_median": round(per[len(per) // 2] * 1e3, 3), "host_ms_max": round(per[-1] * 1e3, 3)}
        if bt is not None:
            out[mode].update(buckets=sorted([list(k) for k in bt.buckets]), eager_fallback_steps=bt.eager_steps,
                             warm_epoch_s=round(t_cap, 2), warm_iterations=n_warm)
            # the slowest timed iteration: its bucket and that bucket's replays before it
            its = [b - a for a, b in zip(marks, marks[1:])]
            k = max(range(len(its)), key=lambda i: its[i])
            out[mode]["slowest_iteration"] = {"index": k, "host_ms": round(its[k] * 1e3, 3),
                                              "bucket": (list(steps_info[k][0]) if steps_info[k][0] is not None
                                                         else "eager"),
                                              "bucket_prior_replays": steps_info[k][1]}
            dev_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(iters)]
            kd = max(range(iters), key=lambda i: dev_ms[i])
            out[mode].update(device_ms_median=round(sorted(dev_ms)[iters // 2], 3), device_ms_max=round(dev_ms[kd], 3),
                             device_slowest_index=kd, host_ms_per_iteration=[round(x * 1e3, 2) for x in its],
                             device_ms_per_iteration=[round(x, 3) for x in dev_ms])
            dq = [(b[0] - a[0]) / 1e6 if a[0] is not None and b[0] is not None else None
                  for a, b in zip(sched, sched[1:])]
            dt_ = [(b[1] - a[1]) / 1e3 if a[1] is not None and b[1] is not None else None
                   for a, b in zip(sched, sched[1:])]
            out[mode]["slowest_iteration"].update(runqueue_wait_ms=dq[k], cgroup_throttled_ms=dt_[k])
            # where the slowest iteration's host time went: the loader's next
            # two batches, then BucketedGraphTrainer.step's phases (layout +
            # bucket, scene-structure uploads, draws + replay); the thread's
            # CPU time, page faults and context switches over the iteration
            # (a blocked thread -- a driver call, an allocation -- shows CPU
            # time far below the wall time and voluntary switches)
            ru0, ru1 = sched[k][2], sched[k + 1][2]
            out[mode]["slowest_iteration"].update(
                phase_ms=dict(zip(("next_batches", "layout_bucket", "scene_upload", "draw_replay"),
                                  [None if x is None else round(x, 3) for x in phases[k]])),
                thread_cpu_ms=None if ru0 is None else round((ru1[0] - ru0[0]) * 1e3, 3),
                minor_faults=None if ru0 is None else ru1[1] - ru0[1],
                major_faults=None if ru0 is None else ru1[2] - ru0[2],
                voluntary_switches=None if ru0 is None else ru1[3] - ru0[3],
                involuntary_switches=None if ru0 is None else ru1[4] - ru0[4])
            allocs1 = torch.cuda.memory_stats(dev).get("num_device_alloc")
            out[mode]["device_allocs_timed"] = (None if allocs0 is None or allocs1 is None
                                                else allocs1 - allocs0)
            out[mode].update(runqueue_wait_ms_total=round(sum(x for x in dq if x is not None), 3),
                             cgroup_throttled_ms_total=(round(sum(x for x in dt_ if x is not None), 3)
                                                        if any(x is not None for x in dt_) else None))
        del tr, g, d, bt
    return {"metric": "train-scenes/s on real data (D-step scenes per second; the G-step takes the next loader "
                      "batch)", "split": "zara1 train",
            "batch": batch, "iterations": iters, "num_seq": len(dset), "graphed_device_data_path": out["graphed"],
            "device_data_path": out["device"], "host_data_path": out["host"], "unit": "scenes/s"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(n):
    """Run this script under torch.distributed.run with one process per GPU.
    The parent never initialises HIP (no torch.cuda call before this), and
    starts the launcher as a child process (no exec from a GPU process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def make_step(trainer, batch, sc, batch_g, sc_g, kw, graph, world=1):
    """-> (run(k): k training iterations, graphed?, the one-iteration
    GraphedTrainer or None).  Graphed on one rank: a
    HIP graph of GRAPH_ITERS iterations replayed k // GRAPH_ITERS times (the
    per-replay graph launch paid once per GRAPH_ITERS iterations) and a
    one-iteration graph for the remainder, so run(k) does exactly k."""
    from sgan.train_step import GraphedTrainer
    if graph:
        g1 = gk = None
        err = None
        try:
            g1 = GraphedTrainer(trainer, batch, sc, warmup=2, batch_g=batch_g, sc_g=sc_g, overlap=OVERLAP, **kw)
            if GRAPH_ITERS > 1 and not trainer.dp.segmented:
                # (the timed trainer draws each replay's host RNG numbers
                # while the previous replay runs: GraphedTrainer draw_ahead;
                # both trainers take their draws from ONE DrawSource, so the
                # remainder iterations of g1 consume those draws in order and
                # every iteration sees the reference's host RNG sequence)
                gk = GraphedTrainer(trainer, batch, sc, warmup=0, batch_g=batch_g, sc_g=sc_g, iters=GRAPH_ITERS,
                                    draw_ahead=True, draws=g1.draws,
                                    overlap=OVERLAP, **kw)
        except Exception as e:  # capture unsupported (e.g. a collective): eager
            err = e
        # every rank takes the same form: a rank that ran eager while the
        # others replayed graphs would issue a different number of
        # collectives before the timed run (the graphs' first replays below)
        # and the job would hang in them.  Captures execute no collective, so
        # up to here every rank ran the same warm-up iterations.
        ok = err is None
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            f = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)   # (the host-control group: gloo)
            if ok and int(f.item()) == 0:
                err = RuntimeError("graph capture failed on another rank")
            ok = int(f.item()) == 1
        if ok:
            if gk is not None:   # both graphs replayed once before any timing (first-replay costs)
                gk.step()
                g1.step()

            def run(k):
                if gk is not None:
                    for _ in range(k // GRAPH_ITERS):
                        gk.step()
                    k %= GRAPH_ITERS
                for _ in range(k):
                    g1.step()
            return run, True, g1
        print("bench: graph capture failed (%s: %s); running eager" % (type(err).__name__, err), file=sys.stderr)
        g1 = gk = None
        torch.cuda.synchronize()
    def eager(k):
        for _ in range(k):
            trainer.step(batch, sc, batch_g, sc_g, **kw)
    return eager, False, None


def timed_run(run, steps, warmup, world, dev, on_start=None):
    run(warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if on_start is not None:
        on_start()
    t0 = time.perf_counter()
    run(steps)   # exactly `steps` iterations
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:   # (host control over gloo: a CPU tensor)
        t = torch.tensor([elapsed])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    return elapsed


def setup(per_gpu, peds, rank, world, dev, graph_kind):
    from sgan.data.synthetic import synthetic_batch
    from sgan.scene import SceneIndex
    from sgan.train_step import DataParallel, GanTrainer
    g, d = build_models(0, graph_kind)
    g, d = g.to(dev), d.to(dev)
    trainer = GanTrainer(g, d, dp=DataParallel(transport=TRANSPORT[0]), capturable=True)
    # the reference feeds consecutive loader batches to the D-step and the
    # G-step (scripts/train.py:279-297): two distinct synthetic batches
    batch = synthetic_batch([peds] * per_gpu, seed=1000 + rank, device=dev)
    batch_g = synthetic_batch([peds] * per_gpu, seed=5000 + rank, device=dev)
    sc = SceneIndex.from_seq_start_end(batch[-1], dev)
    sc_g = SceneIndex.from_seq_start_end(batch_g[-1], dev)
    kw = dict(S_global=sc.S * world, B_global=sc.B * world, shard=(rank * sc.S, (rank + 1) * sc.S))
    return trainer, batch, sc, batch_g, sc_g, kw


def measure(spec, steps, warmup, rank, world, dev, graph_on, n_it=3):
    """Time `steps` iterations of one configuration (HIP-graph replays), then
    every instrumented launch of n_it eager iterations on the same inputs,
    re-issued back to back between HIP events on its launch stream (graph
    replays carry no events); rocprofv3's kernel trace of the same command
    is the cross-check (profiles/)."""
    from sgan import kernels as K
    K.set_precision(spec["prec"])
    try:
        trainer, batch, sc, batch_g, sc_g, kw = setup(spec["per_gpu"], spec["peds"], rank, world, dev, spec["graph"])
        step, graphed, gt = make_step(trainer, batch, sc, batch_g, sc_g, kw, graph_on, world)
        # N > 1, segmented graphs (gloo): HIP events around each eager gradient
        # all-reduce between the graph segments; captured collectives (RCCL,
        # inside the graph): the same two flat buckets all-reduced eagerly
        # after the timed run -- on this rank, max over ranks
        comm = gt is not None and world > 1 and trainer.dp.segmented
        elapsed = timed_run(step, steps, warmup, world, dev, on_start=gt.time_allreduce if comm else None)
        ar_us = gt.allreduce_ms() * 1e3 / steps if comm else None
        if comm:
            gt.time_allreduce(False)
        elif world > 1:
            ar_us = bucket_allreduce_us(trainer, dev)
        if ar_us is not None:
            t = torch.tensor([ar_us])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ar_us = float(t)
        n_it = max(1, min(steps, n_it))
        K.timer.start()
        for _ in range(n_it):
            trainer.step(batch, sc, batch_g, sc_g, **kw)
        recs = K.timer.stop()
        timed = K.timer.replay(recs)
    finally:
        K.set_precision("fp32")
    return dict(elapsed=elapsed, graphed=graphed, agg=kernel_table(timed, n_it), recs=recs, n_it=n_it,
                allreduce_us=ar_us, captured=bool(graphed and world > 1 and not trainer.dp.segmented),
                transport=trainer.dp.transport)


def bucket_allreduce_us(trainer, dev, reps=20):
    """Device time of one iteration's two gradient all-reduces (the G and D
    flat buckets incl. the loss values), issued eagerly back to back between
    HIP events: the collectives' cost when they are captured inside the
    iteration's graph (no events there)."""
    nums = [sum(p.numel() for p in ps) + 3 for ps in (trainer.g_params, trainer.d_params)]
    bufs = [torch.zeros(n, device=dev) for n in nums]
    # the communicator the steps use (sgan.rccl), else the process group's
    rc = trainer.dp.rccl
    ar = rc.allreduce_sum_ if rc is not None else dist.all_reduce
    for b in bufs:
        ar(b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        for b in bufs:
            ar(b)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def top_kernels(agg, n=10):
    top = sorted(agg.items(), key=lambda kv: -kv[1]["us_per_iter"])
    return {k: {"us_per_iter": round(a["us_per_iter"], 1), "launches_per_iter": round(a["launches_per_iter"], 2),
                "GB/s": round(a["bytes"] / (a["us_per_iter"] * 1e-6) / 1e9, 1),
                "TFLOP/s": round(a["flop"] / (a["us_per_iter"] * 1e-6) / 1e12, 2)} for k, a in top[:n]}


def leg_line(name, spec, res, steps):
    """One extra BASELINE configuration on one GPU: its rate, its dominant
    kernel against its roof, its top kernels."""
    agg = res["agg"]
    dom_name, dom = max(agg.items(), key=lambda kv: kv[1]["us_per_iter"])
    ms = res["elapsed"] / steps * 1e3
    return {"config": name, "workload": spec["what"], "value": round(spec["per_gpu"] / (ms * 1e-3), 2),
            "unit": "scenes/s", "ms_per_step": round(ms, 3), "steps": steps, "scenes_per_gpu": spec["per_gpu"],
            "peds_per_scene": spec["peds"], "generator": spec["graph"], "dtype": spec["prec"],
            "hip_graph": res["graphed"],
            "instrumented_launches_per_iter": round(sum(a["launches_per_iter"] for a in agg.values()), 1),
            "roofline": dict(roofline_of(dom_name, dom),
                             # (fp32 legs: the bf16 node transforms would need their own peak)
                             iteration=iteration_roofline(agg, ms, spec["per_gpu"]) if spec["prec"] == "fp32"
                             else None),
            "kernels": top_kernels(agg, 5)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="scenes per GPU (default: 64 at N = 1, BASELINE configs[1]; 4096 / N at N > 1, configs[3])")
    ap.add_argument("--peds", type=int, default=20)
    ap.add_argument("--graph-kind", dest="graph_kind", default="gat", choices=["gat", "gcn", "sgangat"])
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--leg", default="", choices=[""] + list(LEGS),
                    help="measure this BASELINE configuration as the headline (e.g. for its PMC passes)")
    ap.add_argument("--no-legs", action="store_true", help="skip the other configurations (N = 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-scaling-reference", action="store_true")
    ap.add_argument("--no-real-data", action="store_true")
    ap.add_argument("--graph", type=int, default=1, help="capture the iteration in a HIP graph (1) or run eager (0)")
    ap.add_argument("--cpu-iters", type=int, default=2)
    ap.add_argument("--pmc-target", type=int, default=0,
                    help="after timing, re-issue the dominant kernel's main launch this many times (the LAST "
                         "dispatches of that kernel in a rocprofv3 --pmc run; tools/pmc_traffic.py)")
    ap.add_argument("--pmc-kernel", default="",
                    help="with --pmc-target: re-issue this kernel's main launch (default: the dominant one here)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    # one process per GPU.  The process group is gloo and carries host
    # control only (barriers, the max over ranks); the gradient all-reduces
    # go through RCCL on sgan.rccl's own communicator (DataParallel transport
    # "rccl", the unique id exchanged through the rendezvous store) -- no
    # ProcessGroupNCCL exists, so no watchdog thread polls events while the
    # step is captured.  SGG_BENCH_BACKEND=gloo (more
    # ranks than GPUs, ranks sharing a device) is only for rehearsing the
    # multi-rank path on a one-GPU box: the all-reduces then go through gloo.
    backend = os.environ.get("SGG_BENCH_BACKEND", "nccl")
    TRANSPORT[0] = "rccl" if backend == "nccl" else "pg"
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            raise SystemExit("bench: the process group reports world size %d, expected %d"
                             % (dist.get_world_size(), args.gpus))

    if args.leg:
        head = dict(LEGS[args.leg])
    else:
        per_gpu = args.batch or (64 if world == 1 else CONFIG4_GLOBAL // world)
        head = dict(per_gpu=per_gpu, peds=args.peds, graph=args.graph_kind, prec=args.precision)
    per_gpu = head["per_gpu"]
    res = measure(head, args.steps, args.warmup, rank, world, dev, args.graph)
    elapsed, agg, recs = res["elapsed"], res["agg"], res["recs"]
    pmc_target = None
    if args.pmc_target > 0 and rank == 0:
        from sgan import kernels as K
        if args.pmc_kernel and args.pmc_kernel in agg:   # the roofline kernel of the graphed run
            name, a = args.pmc_kernel, agg[args.pmc_kernel]
        else:
            name, a = max(agg.items(), key=lambda kv: kv[1]["us_per_iter"])
        key = main_launch(a)[0]
        fn = next(r[4] for r in recs if r[1] == key)
        K.set_precision(head["prec"])
        try:
            for _ in range(args.pmc_target):
                fn()
        finally:
            K.set_precision("fp32")
        torch.cuda.synchronize()
        pmc_target = {"kernel": name, "shape": list(key[1:]), "reps": args.pmc_target}
    del recs
    res["recs"] = None

    # the other BASELINE configurations, one GPU each (N = 1 only)
    legs = []
    if world == 1 and not args.no_legs and not args.leg:
        k_leg = max(3, args.steps // 2)
        for name, spec in LEGS.items():
            if name == "configs1" and (head["per_gpu"], head["peds"], head["graph"], head["prec"]) == (
                    64, 20, "gat", "fp32"):
                continue   # the headline itself
            r = measure(spec, k_leg, 2, 0, 1, dev, args.graph)
            legs.append(leg_line(name, spec, r, k_leg))
            del r

    scaling_ref = None
    if world == 1 and not args.no_scaling_reference and per_gpu != CONFIG4_GLOBAL and not args.leg:
        # configs[3]'s 4096-scene global batch on this one GPU: the N = 1 point
        # of the strong-scaling curve the N > 1 runs measure
        from sgan import kernels as K
        tr4, b4, sc4, bg4, scg4, kw4 = setup(CONFIG4_GLOBAL, args.peds, 0, 1, dev, "gat")
        st4, gr4, _ = make_step(tr4, b4, sc4, bg4, scg4, kw4, args.graph)
        k4 = max(3, args.steps // 4)
        e4 = timed_run(st4, k4, 2, 1, dev)
        scaling_ref = {"global_batch": CONFIG4_GLOBAL, "n_gpus": 1, "steps": k4, "ms_per_step": round(e4 / k4 * 1e3, 3),
                       "value": round(CONFIG4_GLOBAL / (e4 / k4), 2), "unit": "scenes/s", "hip_graph": gr4,
                       "note": "BASELINE configs[3] workload on one GPU: strong-scaling efficiency at N GPUs = "
                               "value(N) / (N * this value)"}
        del tr4, b4, bg4, st4

    real = None
    if world == 1 and not args.no_real_data and not args.leg:
        real = real_data_leg(dev)

    if rank == 0:
        n_it = res["n_it"]
        top = sorted(agg.items(), key=lambda kv: -kv[1]["us_per_iter"])
        dom_name, dom = top[0]
        roofline = roofline_of(dom_name, dom)
        it_roof = iteration_roofline(agg, elapsed / args.steps * 1e3, per_gpu)
        launches = sorted(((r["launches"] / n_it * r["ms"] * 1e3, n, r, k) for n, a in agg.items()
                           for k, r, _ in a["shapes"]), key=lambda x: -x[0])
        # every instrumented launch with its work model: the iteration's
        # executed-work table (tools/iteration_model.py)
        launch_table = [{"kernel": n, "shape": list(k[1:]), "per_iter": round(r["launches"] / n_it, 2),
                         "avg_us": round(r["ms"] * 1e3, 2), "us_per_iter": round(us, 1),
                         "flop": round(r["flop"]), "bytes": round(r["bytes"])}
                        for us, n, r, k in launches]
        total_launch_us = sum(x[0] for x in launches)
        if os.environ.get("SGG_BENCH_TABLE"):   # (the same table as text)
            with open(os.environ["SGG_BENCH_TABLE"], "w") as f:
                f.write("# kernel | launch shape | launches per iteration | avg us | us per iteration | algorithmic "
                        "FLOP per launch | algorithmic bytes per launch | roofline us per launch\n")
                for us, n, r, k in launches:
                    rl = max(r["flop"] / (FP32_PEAK_TFLOPS * 1e12), r["bytes"] / (HBM_PEAK_GBS * 1e9)) * 1e6
                    f.write("%-50s %-36s %5.2f %8.2f %8.1f %12.4g %12.4g %8.3f\n" % (
                        n[:50], str(list(k[1:]))[:36], r["launches"] / n_it, r["ms"] * 1e3, us, r["flop"],
                        r["bytes"], rl))
        ms_step = elapsed / args.steps * 1e3
        value = world * per_gpu / (elapsed / args.steps)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(per_gpu, head["peds"], iters=args.cpu_iters)
        is_c1 = world == 1 and (per_gpu, head["peds"], head["graph"], head["prec"]) == (64, 20, "gat", "fp32")
        # everything beyond the driver's fields goes to a side file named in
        # the line: the stdout line stays a few KB
        detail_path = os.environ.get("SGG_BENCH_DETAIL") or os.path.join(
            ROOT, "gpurun_out", "bench_detail_n%d_%d.json" % (world, os.getpid()))
        detail = {"roofline": roofline, "iteration_roofline": it_roof, "kernels": top_kernels(agg, 24),
                  "launch_table": launch_table, "cpu_baseline": cpu, "legs": legs, "scaling_reference": scaling_ref,
                  "real_data": real, "pmc_target": pmc_target}
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "scenes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak" if world == 1 else "strong",
            "vs_baseline": round(value / REFERENCE_CPU_SCENES_S, 1) if is_c1 else None,
            "vs_baseline_basis": "value / 13.9 scenes/s, the reference's CPU path on this workload in the survey "
                                 "container (BASELINE.md 2); no published throughput" if is_c1 else None,
            "vs_cpu_same_box": round(value / cpu["value"], 1) if cpu else None,
            "dtype": head["prec"],
            "data": "synthetic (random-init weights, SURVEY.md 8d recipe)",
            "config": {"workload": "train iteration = D-step + G-step (best_k=20, Adam), %s generator%s" % (
                                       head["graph"].upper(),
                                       "; BASELINE configs[1] shape (batch 64)" if is_c1 else
                                       "; BASELINE configs[3] (4096-scene global batch)"
                                       if world * per_gpu == CONFIG4_GLOBAL else
                                       "; %s" % head.get("what", "")),
                       "scenes_per_gpu": per_gpu, "global_batch": per_gpu * world, "peds_per_scene": head["peds"],
                       "obs_len": 8, "pred_len": 12, "generator": head["graph"], "hip_graph": res["graphed"],
                       "parallelism": "dp%d" % world},
            "roofline": {k: roofline[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel",
                                                  "launch", "avg_launch_us", "flop_per_launch",
                                                  "algorithmic_bytes_per_launch", "traffic_over_algorithmic")},
            "cpu_baseline": None if cpu is None else {k: cpu[k] for k in ("value", "unit", "cores", "kind", "cpu_model")}
            | {"sample": "%d train iterations on %d x %d-ped synthetic scenes, oracle reference formulation, torch CPU "
                         "fp32" % (args.cpu_iters, per_gpu, head["peds"])},
            "instrumented_us_per_iter": round(total_launch_us, 1),
            "detail": os.path.relpath(detail_path, ROOT),
        }
        if "latency" in roofline:
            line["roofline"]["latency"] = {k: roofline["latency"][k] for k in ("us_per_step", "steps", "roofline_us")}
        line["roofline"]["iteration_frac"] = it_roof["frac"]
        if legs:
            line["legs"] = [{"config": l["config"], "value": l["value"], "ms_per_step": l["ms_per_step"],
                             "dtype": l["dtype"], "roofline": {k: l["roofline"][k] for k in ("kernel", "bound", "frac")}}
                            for l in legs]
        if scaling_ref is not None:
            line["scaling_reference"] = {k: scaling_ref[k] for k in ("global_batch", "value", "ms_per_step")}
        if real is not None:
            gd = real["graphed_device_data_path"]
            line["real_data"] = {"split": real["split"], "batch": real["batch"],
                                 "graphed": {k: gd.get(k) for k in ("value", "ms_per_iteration", "host_ms_median",
                                                                    "host_ms_max", "device_ms_median")},
                                 "device_data_path": real["device_data_path"]["value"],
                                 "host_data_path": real["host_data_path"]["value"]}
        if pmc_target is not None:
            line["pmc_target"] = pmc_target
        if world > 1:
            ar = res["allreduce_us"]
            line["communication"] = {
                "transport": res["transport"], "control": dist.get_backend(), "world_size": dist.get_world_size(),
                "allreduce_us_per_iter": round(ar, 1) if ar is not None else None,
                "compute_us_per_iter": round(ms_step * 1e3 - ar, 1) if ar is not None else None,
                "allreduces_per_iter": 2,
                "collectives": "captured in the HIP graph" if res.get("captured") else "eager between graph segments"}
            detail["communication_note"] = (
                "one flat SUM bucket per optimizer step; transport rccl = ncclAllReduce on sgan.rccl's communicator "
                "(no ProcessGroupNCCL; gloo carries host control), pg = the gloo process group's all_reduce; "
                "captured: the two buckets all-reduced eagerly between HIP events after the timed run; segmented: "
                "HIP events around each eager all-reduce between the graph segments; per iteration, max over ranks; "
                "compute = ms_per_step - all-reduce time")
        try:
            os.makedirs(os.path.dirname(detail_path), exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(dict(line=line, **detail), f, indent=1, default=str)
        except OSError as e:
            line["detail"] = "unwritten (%s)" % e
        print(json.dumps(line), flush=True)
    if world > 1:
        import gc
        from sgan import rccl
        gc.collect()   # the captured graphs are gone before their communicator
        torch.cuda.synchronize()
        dist.barrier()
        rccl.release()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
