"""GPU tests that start other processes (torch.distributed.run ranks, the
bench's own spawn path, the RCCL world-1 worker).  They sit in a file that
sorts after every parity file: under `pytest -x` a failure of a child
process must not hide the parity results.

  test_rccl_world1_dp_path                 the DP path through RCCL on the
                                           lease's one GPU, set up as bench.py
                                           sets up N > 1 (gloo host control,
                                           sgan.rccl communicator), eager /
                                           captured / segmented, bitwise ==
                                           no DP, three rounds in one process;
  test_graphed_trainer_two_ranks           2 gloo ranks sharing the GPU,
                                           segmented graph replay == eager;
  test_two_rank_512_scene_shard_equals_single
                                           configs[3]'s DP on a 512-scene
                                           global batch == one rank;
  test_bench_gpus2_spawns_two_ranks        `bench.py --gpus 2` spawns its ranks.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _torchrun(n, script, env, timeout=110):
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                           "--master-addr", "127.0.0.1", "--master-port", str(_port()), script],
                          capture_output=True, text=True, timeout=timeout, env=env)


def test_rccl_world1_dp_path():
    """The data-parallel path through RCCL on this lease's one GPU (round-5
    abort): a gloo process group of world size 1 for
    host control, the flat SUM all-reduce on sgan.rccl's communicator every
    optimizer step, eager and graphed -- the collective CAPTURED inside the
    HIP graph (1- and 2-iteration graphs) and the segmented form -- each
    bitwise equal to the same execution without DP, three rounds in one
    process (tests/_nccl_world1_worker.py)."""
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "_nccl_world1_worker.py")], capture_output=True,
                       text=True, timeout=110, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "rank 0 OK" in out, out[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    for k in ("eager_dp", "graph1_captured", "graph1_segmented", "graph2_captured"):
        assert k in line, line
    assert line["rounds"] == 3
    assert line["allreduce_us_per_iter"] > 0
    print(line)


def test_graphed_trainer_two_ranks():
    """Scene-sharded DP with the segmented graph replay (GraphedTrainer cuts
    the capture at each gradient all-reduce): 2 ranks on this GPU over gloo
    (tests/_dp_graph_worker.py), graph replay == eager step on every rank."""
    r = _torchrun(2, os.path.join(HERE, "_dp_graph_worker.py"), dict(os.environ, OMP_NUM_THREADS="1"))
    out = r.stdout + r.stderr
    assert r.returncode == 0 and out.count(" OK") == 2, out[-3000:]


def test_two_rank_512_scene_shard_equals_single():
    """config 4's data parallelism: 2 ranks (gloo, sharing this GPU) on a
    512-scene global batch, segmented graph replay, == eager per rank, == the
    whole batch on one rank (tests/_dp_graph_worker.py, SGG_DP_VS_SINGLE)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", SGG_DP_SCENES="512", SGG_DP_VS_SINGLE="1")
    r = _torchrun(2, os.path.join(HERE, "_dp_graph_worker.py"), env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and out.count(" OK") == 2, out[-3000:]


def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` (not under torch.distributed.run) spawns one
    process per rank itself and reports the 2-rank job (rehearsal on this one
    GPU: both ranks share it, so the all-reduce is gloo's -- RCCL refuses two
    ranks on one device)."""
    env = dict(os.environ, SGG_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "16", "--no-cpu-baseline"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines[-1]) <= 6144, "the bench line must stay parseable: %d bytes" % len(lines[-1])
    line = json.loads(lines[-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 32 and line["config"]["parallelism"] == "dp2"
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    # the N > 1 line separates communication from compute
    comm = line["communication"]
    assert comm["world_size"] == 2 and comm["transport"] == "pg"
    assert comm["allreduce_us_per_iter"] > 0 and comm["compute_us_per_iter"] > 0
    assert comm["allreduce_us_per_iter"] < line["ms_per_step"] * 1e3
