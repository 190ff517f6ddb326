"""Per-parameter gradient error of the sgangat 64-ped generator vs the
float64 oracle (diagnostic for test_sgangat_64ped_generator_vs_oracle).
usage: python tools/diag_gen_err.py [seed ...]  (one seed: per-parameter table;
several: the worst parameter per seed)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "group-gan-gcn-gat_amd")]
from test_gpu_configs import SIZES64, _oracle_pair, reference_gd  # noqa: E402
SEED64 = 73
from sgan.data.synthetic import synthetic_batch  # noqa: E402



def run(seed, table):
    torch.manual_seed(seed)
    g, d = reference_gd("sgangat")
    og, _ = _oracle_pair(g, d)
    og32, _ = _oracle_pair(g, d)
    og = og.double()
    b = synthetic_batch(SIZES64, seed=int(os.environ.get("DIAG_BATCH_SEED", SEED64)))
    obs, _, obs_rel, _, _, _, obs_g, _, _, _, sse = b
    z = torch.randn(len(SIZES64), 8)
    dy = torch.randn(12, sum(SIZES64), 2)
    margins = []

    def hook(mod, inp, out):   # leaky-ReLU kink margin of every (i, j) score, float64
        hp = torch.einsum("nf,hfo->hno", inp[0], mod.w)
        z = (hp @ mod.a_src) + (hp @ mod.a_dst).transpose(1, 2)
        margins.append((float(z.abs().min()), float(z.abs().max())))
    hooks = [m.register_forward_hook(hook) for m in og.gatencoder.gat_net.layer_stack]
    torch.set_default_dtype(torch.float64)
    y_ref = og(obs.double(), obs_rel.double(), sse, obs_g.double(), user_noise=z.double())
    (y_ref * dy.double()).sum().backward()
    torch.set_default_dtype(torch.float32)
    for h in hooks:
        h.remove()
    if table:
        for i in range(len(og.gatencoder.gat_net.layer_stack)):
            mins = [m[0] for m in margins[i::len(og.gatencoder.gat_net.layer_stack)]]
            maxs = [m[1] for m in margins[i::len(og.gatencoder.gat_net.layer_stack)]]
            print("layer %d: min |src_i + dst_j| %.3e over scenes (max %.3e)" % (i, min(mins), max(maxs)))
    y32 = og32(obs, obs_rel, sse, obs_g, user_noise=z)
    (y32 * dy).sum().backward()
    y = g(obs.cuda(), obs_rel.cuda(), sse.cuda(), obs_g.cuda(), user_noise=z.cuda())
    (y * dy.cuda()).sum().backward()
    ref = {k: p.grad.numpy() for k, p in og.named_parameters() if p.grad is not None}
    r32 = {k: p.grad.numpy() for k, p in og32.named_parameters() if p.grad is not None}
    fl = 1e-2 * max(np.abs(v).max() for v in ref.values())
    worst, worst32 = (0.0, "", 0.0), 0.0
    print("out err hip %.3e  cpu32 %.3e" % (np.abs(y.detach().cpu().double().numpy() - y_ref.detach().numpy()).max(),
                                             np.abs(y32.detach().double().numpy() - y_ref.detach().numpy()).max()))
    for k, p in g.named_parameters():
        if k not in ref:
            continue
        sc = max(np.abs(ref[k]).max(), fl)
        e = np.abs(p.grad.detach().cpu().double().numpy() - ref[k]).max() / sc
        e32 = np.abs(r32[k].astype(np.float64) - ref[k]).max() / sc
        worst32 = max(worst32, e32)
        worst = max(worst, (e, k, e32))
        if table:
            print("%-55s hip %.3e  cpu32 %.3e  scale %.3e%s" % (k, e, e32, sc, "  <<<" if e > 2e-4 else ""))
    print("seed %d worst: hip %.3e at %s (cpu32 %.3e there); cpu32 worst %.3e" % ((seed,) + worst + (worst32,)))


seeds = [int(a) for a in sys.argv[1:]] or [0]
for sd in seeds:
    run(sd, len(seeds) == 1)
