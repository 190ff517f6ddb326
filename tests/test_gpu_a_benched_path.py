"""The benched path, pinned first: this file sorts
before every other GPU file, so its result is in every GPU run whatever
fails later.

bench.py times GanTrainer with paired contexts (the G-step's context formed
at the D-step, G.context_pair) replayed as HIP graphs (GraphedTrainer;
several iterations per graph, the host draws made ahead).  Here:

  * the reference's own two training iterations (train_step.npz:
    scripts/train.py:395-484 discriminator_step + generator_step, fresh Adam,
    seeded host RNGs) reproduced by a HIP-graph REPLAY of the paired step:
    losses 1e-4 rel, the gradients each optimizer step consumed 1e-3 of the
    tensor max (floor 1 % of the step's largest), weights within Adam's
    2 lr bound;
  * configs[1]'s shape (64 synthetic 20-ped scenes, distinct D / G batches):
    the bench's graphs -- a 4-iteration graph with draw-ahead and a
    1-iteration graph on one draw source -- bit-identical to the eager
    paired step over 5 iterations.
"""
import os
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN, check_step_grads, load_family

pytestmark = pytest.mark.gpu

DEV = "cuda"
KEYS = ["obs_traj", "pred_traj", "obs_traj_rel", "pred_traj_rel", "obs_vel", "pred_vel", "obs_traj_g",
        "pred_traj_g", "non_linear_ped", "loss_mask", "seq_start_end"]


def npz(name):
    return np.load(os.path.join(GOLDEN, name))


def T(a):
    return torch.from_numpy(np.asarray(a)).clone().to(DEV)


def models(fixture=True, seed=0):
    from sgan.models import TrajectoryDiscriminator, TrajectoryGenerator
    torch.manual_seed(seed)
    g = TrajectoryGenerator(8, 12, embedding_dim=16, encoder_h_dim=32, decoder_h_dim=32, mlp_dim=64, num_layers=1,
                            noise_dim=(8,), noise_type="gaussian", noise_mix_type="global",
                            pooling_type="pool_net", pool_every_timestep=False, dropout=0.0, bottleneck_dim=8,
                            batch_norm=False, n_units=[40, 16, 40], n_heads=1, dropout1=0.0, alpha=0.2, graph="gat")
    d = TrajectoryDiscriminator(8, 12, embedding_dim=16, h_dim=48, mlp_dim=64, num_layers=1, batch_norm=False,
                                dropout=0.0, d_type="global")
    if fixture:
        w = npz("weights.npz")
        load_family(g, {k[2:]: torch.from_numpy(w[k]) for k in w.files if k.startswith("g/")})
        d.load_state_dict({k[2:]: torch.from_numpy(w[k]) for k in w.files if k.startswith("d/")})
    else:
        for m in list(g.modules()) + list(d.modules()):   # train.py:127-130 init_weights
            if isinstance(m, torch.nn.Linear):
                torch.nn.init.kaiming_normal_(m.weight)
    return g.to(DEV), d.to(DEV)


def training_state(tr):
    """Every tensor a training iteration changes: parameters and the fused
    optimizers' state (step counters on the device, moments)."""
    ts = [p.data for p in tr.g_params + tr.d_params]
    for opt in (tr.opt_g, tr.opt_d):
        for p in opt.params:
            st = opt.opt.state.get(p)
            if st:
                ts += [st["step"], st["exp_avg"], st["exp_avg_sq"]]
    return ts


def test_benched_path_graph_replay_vs_reference_iterations():
    """Two reference iterations through the paired step replayed from HIP
    graphs.  Each iteration's graph is captured (its warm-up iteration
    runs), the training state and host RNG states are put back as they were
    before the capture, and the replay is the iteration that counts."""
    from sgan.scene import SceneIndex
    from sgan.train_step import GanTrainer, GraphedTrainer
    g, d = models()
    tr = GanTrainer(g, d, capturable=True)
    f = npz("train_step.npz")
    torch.manual_seed(1234)
    random.seed(1234)
    for it in range(2):
        b = [T(f["b%d/%s" % (it, k)]) for k in KEYS]
        sc = SceneIndex.from_seq_start_end(b[-1], DEV)
        assert tr._pairs(sc, sc), "the benched configuration pairs the contexts"
        saved = [t.detach().clone() for t in training_state(tr)]
        rng = (torch.get_rng_state(), random.getstate())
        gt = GraphedTrainer(tr, b, sc, warmup=1)
        assert gt.pair and not gt.segments
        with torch.no_grad():
            for t, s in zip(training_state(tr), saved):
                t.copy_(s)
        torch.set_rng_state(rng[0])
        random.setstate(rng[1])
        ld, lg = gt.step()
        torch.cuda.synchronize()
        for k, v in list(ld.items()) + list(lg.items()):
            tag = "D" if k.startswith("D") else "G"
            ref = float(f["it%d/%s/%s" % (it, tag, k)])
            assert abs(float(v) - ref) <= 1e-4 * max(1.0, abs(ref)), (it, k, float(v), ref)
        check_step_grads({k: p.grad for k, p in d.named_parameters() if p.grad is not None}, f, it, "D")
        check_step_grads({k: p.grad for k, p in g.named_parameters() if p.grad is not None}, f, it, "G")
        for mod, tag, lr in ((g, "g", 1e-4), (d, "d", 1e-3)):
            for k, v in mod.state_dict().items():
                ref = f["it%d/%s/%s" % (it, tag, k)]
                err = np.abs(v.detach().cpu().numpy().astype(np.float64) - ref).max()
                assert err <= 2 * lr * (it + 1) + 1e-5 * np.abs(ref).max(), (it, tag, k, err)
        del gt


def _run_configs1(graphed):
    from sgan.data.synthetic import synthetic_batch
    from sgan.scene import SceneIndex
    from sgan.train_step import GanTrainer, GraphedTrainer
    g, d = models(fixture=False)
    tr = GanTrainer(g, d, capturable=True)
    batch = synthetic_batch([20] * 64, seed=1000, device=DEV)
    batch_g = synthetic_batch([20] * 64, seed=5000, device=DEV)
    sc = SceneIndex.from_seq_start_end(batch[-1], DEV)
    scg = SceneIndex.from_seq_start_end(batch_g[-1], DEV)
    torch.manual_seed(7)
    random.seed(7)
    hist = []
    if graphed:
        g1 = GraphedTrainer(tr, batch, sc, warmup=2, batch_g=batch_g, sc_g=scg)
        gk = GraphedTrainer(tr, batch, sc, warmup=0, batch_g=batch_g, sc_g=scg, iters=4, draw_ahead=True,
                            draws=g1.draws)
        hist.append(gk.step())
        hist.append(g1.step())
    else:
        for _ in range(2 + 4 + 1):
            hist.append(tr.step(batch, sc, batch_g, scg))
    torch.cuda.synchronize()
    ld, lg = hist[-1]
    losses = {k: float(v) for k, v in list(ld.items()) + list(lg.items())}
    w = {"g." + k: v.detach().cpu().clone() for k, v in g.state_dict().items()}
    w.update({"d." + k: v.detach().cpu().clone() for k, v in d.state_dict().items()})
    return losses, w


def test_benched_graphs_bit_identical_to_eager_configs1():
    """configs[1]'s workload as bench.py runs it: 2 warm-up iterations, a
    4-iteration graph (draw-ahead) and a 1-iteration graph sharing one draw
    source == 7 eager paired iterations, bit for bit."""
    la, wa = _run_configs1(False)
    lb, wb = _run_configs1(True)
    assert la == lb, (la, lb)
    for k in wa:
        assert torch.equal(wa[k], wb[k]), (k, (wa[k] - wb[k]).abs().max().item())
