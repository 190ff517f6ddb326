"""Pin the CPU oracle (oracle/sgan_oracle.py) against fixtures produced by the
real reference (tests/golden/make_golden.py).  CPU only."""
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import sgan_oracle as O

from conftest import GOLDEN, RecordingAdam, check_step_grads, load_family

RTOL = 2e-5


def npz(name):
    return np.load(os.path.join(GOLDEN, name))


def T(a):
    return torch.from_numpy(np.asarray(a)).clone()


def close(a, b, rtol=RTOL, atol=None, floor=1e-6):
    """max |a-b| relative to max |b| (or to `floor` when the reference tensor is
    ~0, e.g. a gradient that cancels analytically)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), floor)
    err = np.abs(a - b).max() / scale
    assert err <= (rtol if atol is None else atol), "max rel err %.3e" % err


def grad_floor(f, prefix):
    """1e-2 of the largest reference parameter gradient of the module: a tensor
    whose gradient is analytically ~0 (the inter-group out_att.a, whose source
    half cancels under the row softmax) is compared on that scale."""
    return 1e-2 * max(np.abs(f[k]).max() for k in f.files if k.startswith(prefix))


def load_models(prefix_g="g/", prefix_d="d/", graph="gat", w=None):
    w = w if w is not None else npz("weights.npz")
    g, d = O.build_default(graph)
    load_family(g, {k[len(prefix_g):]: T(w[k]) for k in w.files if k.startswith(prefix_g)})
    d.load_state_dict({k[len(prefix_d):]: T(w[k]) for k in w.files if k.startswith(prefix_d)})
    return g, d


@pytest.mark.parametrize("tag", ["g", "d"])
def test_pool_fixture(tag):
    f = npz("pool.npz")
    hd = f[tag + "/h"].shape[1]
    bn = f[tag + "/out"].shape[1]
    net = O.PoolHiddenNet(16, hd, 64, bn, "relu", False)
    net.load_state_dict({k[len(tag) + 3:]: T(f[k]) for k in f.files if k.startswith(tag + "/w/")})
    h = T(f[tag + "/h"]).unsqueeze(0).requires_grad_(True)
    y = net(h, T(f[tag + "/sse"]), T(f[tag + "/pos"]))
    close(y.detach(), f[tag + "/out"])
    (y * T(f[tag + "/dout"])).sum().backward()
    close(h.grad[0], f[tag + "/dh"])
    for k, p in net.named_parameters():
        close(p.grad, f[tag + "/dw/" + k], floor=grad_floor(f, tag + "/dw/"))


@pytest.mark.parametrize("name,heads", [("gat_encoder.npz", 1), ("gat_encoder_h2.npz", 2), ("gcn_module.npz", 0)])
def test_graph_module_fixture(name, heads):
    f = npz(name)
    if heads:
        mod = O.GATEncoder([40, 16, 40], heads, 0.0, 0.2)
    else:
        mod = O.GCNModule(40, 72, 16, 2, 24)
    mod.load_state_dict({k[2:]: T(f[k]) for k in f.files if k.startswith("w/")})
    x = T(f["x"]).requires_grad_(True)
    y = mod(x, T(f["sse"]), None, T(f["labels"]).view(-1, 1))
    close(y.detach(), f["out"])
    (y * T(f["dout"])).sum().backward()
    close(x.grad, f["dx"])
    for k, p in mod.named_parameters():
        if "dw/" + k in f.files:
            close(p.grad, f["dw/" + k], rtol=1e-4, floor=grad_floor(f, "dw/"))


@pytest.mark.parametrize("graph", ["gat", "gcn"])
def test_generator_fixture(graph):
    f = npz("gen_fwd_%s.npz" % graph)
    g, _ = load_models(graph=graph)
    for b in ("synth", "zara1"):
        g.zero_grad()
        y = g(T(f[b + "/obs_traj"]), T(f[b + "/obs_traj_rel"]), T(f[b + "/seq_start_end"]),
              T(f[b + "/obs_traj_g"]), user_noise=T(f[b + "/noise"]))
        close(y.detach(), f[b + "/out"])
        (y * T(f[b + "/dout"])).sum().backward()
        for k, p in g.named_parameters():
            key = b + "/dw/" + k
            if key in f.files:
                close(p.grad, f[key], rtol=1e-4, floor=grad_floor(f, b + "/dw/"))


def test_sgangat_module_fixture():
    """Batched multi-head GAT (GAT.py:6-106 text) with instance norm."""
    f = npz("sgangat_gat.npz")
    mod = O.BatchGATEncoder([40, 16, 40], [4, 1], 0.0, 0.2)
    mod.load_state_dict({k[2:]: T(f[k]) for k in f.files if k.startswith("w/")})
    x = T(f["x"]).requires_grad_(True)
    y = mod(x, T(f["sse"]))
    close(y.detach(), f["out"])
    (y * T(f["dout"])).sum().backward()
    close(x.grad, f["dx"], rtol=1e-4)
    for k, p in mod.named_parameters():
        # layer 0's bias only reaches the loss through ELU + the next layer's
        # instance norm, which removes its per-feature mean: its gradient is a
        # sum of B large terms that nearly cancel (|dW| 0.3 vs 28 for w)
        close(p.grad, f["dw/" + k], rtol=1e-3 if k.endswith("0.bias") else 1e-4, floor=grad_floor(f, "dw/"))


def test_sgangat_generator_fixture():
    f = npz("gen_fwd_sgangat.npz")
    g, _ = O.build_default("sgangat")
    g.load_state_dict({k[2:]: T(f[k]) for k in f.files if k.startswith("w/")})
    for b in ("synth", "zara1"):
        g.zero_grad()
        y = g(T(f[b + "/obs_traj"]), T(f[b + "/obs_traj_rel"]), T(f[b + "/seq_start_end"]),
              T(f[b + "/obs_traj_g"]), user_noise=T(f[b + "/noise"]))
        close(y.detach(), f[b + "/out"])
        (y * T(f[b + "/dout"])).sum().backward()
        n = 0
        for k, p in g.named_parameters():
            key = b + "/dw/" + k
            if key in f.files:
                close(p.grad, f[key], rtol=1e-3 if k.endswith("stack.0.bias") else 1e-4,
                      floor=grad_floor(f, b + "/dw/"))
                n += 1
        assert n >= 20


def test_discriminator_fixture():
    f = npz("disc_fwd.npz")
    _, d = load_models()
    tr = T(f["traj_rel"]).requires_grad_(True)
    s = d(T(f["traj"]), tr, T(f["sse"]))
    close(s.detach(), f["scores"])
    feat = d.pool_net(d.encoder(tr).squeeze(), T(f["sse"]), T(f["traj"])[0])
    close(feat.detach(), f["feat"])
    (s * T(f["dscores"])).sum().backward()
    close(tr.grad, f["dtraj_rel"], atol=1e-5)
    for k, p in d.named_parameters():
        if "dw/" + k in f.files:
            close(p.grad, f["dw/" + k], rtol=1e-4, floor=grad_floor(f, "dw/"))


@pytest.mark.slow
def test_train_step_fixture():
    path = os.path.join(GOLDEN, "train_step.npz")
    if not os.path.exists(path):
        pytest.skip("train_step fixture not generated")
    f = np.load(path)
    g, d = load_models()
    og = RecordingAdam.make(g.named_parameters(), lr=O.Args.g_learning_rate)
    od = RecordingAdam.make(d.named_parameters(), lr=O.Args.d_learning_rate)
    torch.manual_seed(1234)
    random.seed(1234)
    keys = ["obs_traj", "pred_traj", "obs_traj_rel", "pred_traj_rel", "obs_vel", "pred_vel",
            "obs_traj_g", "pred_traj_g", "non_linear_ped", "loss_mask", "seq_start_end"]
    for it in range(2):
        b = [T(f["b%d/%s" % (it, k)]) for k in keys]
        ld = O.discriminator_step(O.Args, b, g, d, od)
        lg = O.generator_step(O.Args, b, g, d, og)
        for k, v in ld.items():
            assert abs(v - float(f["it%d/D/%s" % (it, k)])) <= 1e-4 * max(1.0, abs(v))
        for k, v in lg.items():
            assert abs(v - float(f["it%d/G/%s" % (it, k)])) <= 1e-4 * max(1.0, abs(v))
        # the gradients each Adam step consumed (D raw, G after clip 2.0)
        check_step_grads(od.rec[-1], f, it, "D", rtol=1e-4)
        check_step_grads(og.rec[-1], f, it, "G", rtol=1e-4)
        # Adam's first steps move each weight by ~lr * sign(grad); weights whose
        # gradient is rounding noise (the attention vectors `a`, whose source
        # half cancels in the row softmax) may flip sign: allow 2*lr per step.
        for mod, tag, lr in ((g, "g", O.Args.g_learning_rate), (d, "d", O.Args.d_learning_rate)):
            for k, v in mod.state_dict().items():
                ref = f["it%d/%s/%s" % (it, tag, k)]
                err = np.abs(v.numpy().astype(np.float64) - ref).max()
                assert err <= 2 * lr * (it + 1) + 1e-5 * np.abs(ref).max(), (tag, k, err)


@pytest.mark.parametrize("tag,pooling", [("none", None), ("pool", "pool_net")])
def test_vanilla_generator_fixture(tag, pooling):
    """Upstream Social-GAN generator (sgan-models / sgan-p-models families,
    mlp_decoder_context of models.py:796-804 / :898) vs the reference run."""
    f = npz("gen_fwd_vanilla.npz")
    g = O.TrajectoryGenerator(8, 12, embedding_dim=16, encoder_h_dim=32, decoder_h_dim=32, mlp_dim=64,
                              noise_dim=(8,), noise_mix_type="global", pooling_type=pooling,
                              pool_every_timestep=False, bottleneck_dim=8, batch_norm=False, graph="vanilla")
    pre = tag + "/w/"
    g.load_state_dict({k[len(pre):]: T(f[k]) for k in f.files if k.startswith(pre)})
    for b in ("synth", "zara1", "eth"):
        p = "%s/%s/" % (tag, b)
        g.zero_grad()
        y = g(T(f[p + "obs_traj"]), T(f[p + "obs_traj_rel"]), T(f[p + "seq_start_end"]), T(f[p + "obs_traj_g"]),
              user_noise=T(f[p + "noise"]))
        close(y.detach(), f[p + "out"])
        (y * T(f[p + "dout"])).sum().backward()
        n = 0
        for k, q in g.named_parameters():
            close(q.grad, f[p + "dw/" + k], rtol=1e-4, floor=grad_floor(f, p + "dw/"))
            n += 1
        assert n == (24 if pooling else 18)


def _oracle_from_trained(tag):
    """The oracle generator built from a trained upstream checkpoint's args
    (tests/golden/evaluate_trained.json) with its g_state (trained.npz)."""
    ev = json.load(open(os.path.join(GOLDEN, "evaluate_trained.json")))
    a = ev["args"][tag]
    g = O.TrajectoryGenerator(a["obs_len"], a["pred_len"], embedding_dim=a["embedding_dim"],
                              encoder_h_dim=a["encoder_h_dim_g"], decoder_h_dim=a["decoder_h_dim_g"],
                              mlp_dim=a["mlp_dim"], num_layers=a["num_layers"], noise_dim=tuple(a["noise_dim"]),
                              noise_type=a["noise_type"], noise_mix_type=a["noise_mix_type"],
                              pooling_type=a["pooling_type"], pool_every_timestep=a["pool_every_timestep"],
                              dropout=a["dropout"], bottleneck_dim=a["bottleneck_dim"], batch_norm=a["batch_norm"],
                              graph="vanilla")
    f = npz("trained.npz")
    g.load_state_dict({k[len(tag) + 3:]: T(f[k]) for k in f.files if k.startswith(tag + "/g/")})
    return g, a, ev


@pytest.mark.parametrize("tag,bs", [("sgan-models/eth_12", 64), ("sgan-models/eth_12", 1),
                                    ("sgan-p-models/hotel_12", 64), ("sgan-models/eth_8", 64)])
def test_oracle_evaluate_trained_checkpoints(tag, bs):
    """configs[0] on TRAINED weights: the oracle's evaluate_model restatement
    with the upstream checkpoints' g_state (loaded by the weights-only
    unpickler) reproduces the reference's best-of-20 ADE / FDE (seed 0)."""
    from sgan.data.trajectories_GCN import TrajectoryDataset, seq_collate
    from torch.utils.data import DataLoader
    g, a, ev = _oracle_from_trained(tag)
    split = tag.split("/")[1].split("_")[0]
    dset = TrajectoryDataset(os.path.join(GOLDEN, "datasets_group", split, "test"), obs_len=a["obs_len"],
                             pred_len=a["pred_len"], skip=a["skip"], delim=a["delim"])
    torch.manual_seed(0)
    loader = DataLoader(dset, batch_size=bs, shuffle=True, num_workers=0, collate_fn=seq_collate)
    ade, fde = O.evaluate(loader, g, num_samples=20, pred_len=a["pred_len"])
    ref = ev["%s/b%d" % (tag, bs)]
    assert abs(ade - ref["ade"]) <= 1e-4 * ref["ade"], (ade, ref)
    assert abs(fde - ref["fde"]) <= 1e-4 * ref["fde"], (fde, ref)
