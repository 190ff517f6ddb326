"""Generate the golden fixtures under tests/golden/ from the REAL reference.

Test infrastructure only.  Runs in the build container (CPU), where the
reference checkout lives read-only at /root/reference.  It never runs on the
GPU box and nothing in the product imports it; only the .npz / .json files it
writes travel.

The reference hard-codes `.cuda()` (sgan/models.py:26,28,58-59,267,278,283,
661,680,690,912), so we map `Tensor.cuda` / `Module.cuda` to identity before
importing it, and stub the `attrdict` package that scripts/evaluate_model.py:11
imports (absent here).  Nothing of the reference is copied: we call its
functions and record inputs/outputs.

Usage:  python tests/golden/make_golden.py [--only NAME ...] [--skip-eval]
"""
import argparse
import importlib.util
import json
import os
import random
import shutil
import sys
import time
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
SPLITS = ["eth", "hotel", "univ", "zara1", "zara2"]


# ----------------------------------------------------------------------------
# reference import shim
# ----------------------------------------------------------------------------
def _import_reference():
    sys.dont_write_bytecode = True
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.nn.Module.cuda = lambda self, *a, **k: self
    ad = types.ModuleType("attrdict")

    class AttrDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError:
                raise AttributeError(k)

    ad.AttrDict = AttrDict
    sys.modules["attrdict"] = ad
    sys.path.insert(0, REF)
    import sgan.models as m  # noqa
    import sgan.losses as l  # noqa
    import sgan.utils as u  # noqa
    import sgan.data.loader as dl  # noqa

    saved_argv = sys.argv
    sys.argv = ["train.py"]
    spec = importlib.util.spec_from_file_location("ref_train", os.path.join(REF, "scripts/train.py"))
    tr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tr)
    spec = importlib.util.spec_from_file_location("ref_eval", os.path.join(REF, "scripts/evaluate_model.py"))
    ev = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ev)
    sys.argv = saved_argv
    return m, l, u, dl, tr, ev


M, L, U, DL, TR, EV = _import_reference()
ARGS = TR.parser.parse_args([])  # train.py defaults (GAT config)
ARGS.loader_num_workers = 0


def build_models(seed=0):
    """Generator / discriminator exactly as scripts/train.py:173-220 builds them."""
    torch.manual_seed(seed)
    a = ARGS
    n_units = [40] + [int(x) for x in a.hidden_units.strip().split(",")] + [40]
    g = M.TrajectoryGenerator(
        obs_len=a.obs_len, pred_len=a.pred_len, embedding_dim=a.embedding_dim,
        encoder_h_dim=a.encoder_h_dim_g, decoder_h_dim=a.decoder_h_dim_g, mlp_dim=a.mlp_dim,
        num_layers=a.num_layers, noise_dim=a.noise_dim, noise_type=a.noise_type,
        noise_mix_type=a.noise_mix_type, pooling_type=a.pooling_type,
        pool_every_timestep=a.pool_every_timestep, dropout=a.dropout,
        bottleneck_dim=a.bottleneck_dim, neighborhood_size=a.neighborhood_size,
        grid_size=a.grid_size, batch_norm=a.batch_norm, n_units=n_units,
        n_heads=a.n_heads, dropout1=a.dropout1, alpha=a.alpha)
    g.apply(TR.init_weights)
    g.train()
    d = M.TrajectoryDiscriminator(
        obs_len=a.obs_len, pred_len=a.pred_len, embedding_dim=a.embedding_dim,
        h_dim=a.encoder_h_dim_d, mlp_dim=a.mlp_dim, num_layers=a.num_layers,
        dropout=a.dropout, batch_norm=a.batch_norm, d_type=a.d_type)
    d.apply(TR.init_weights)
    d.train()
    return g, d


def sd_arrays(module, prefix):
    return {prefix + k: v.detach().numpy().astype(np.float32).copy() for k, v in module.state_dict().items()}


def grad_arrays(module, prefix):
    out = {}
    for k, p in module.named_parameters():
        if p.grad is not None:
            out[prefix + k] = p.grad.detach().numpy().astype(np.float32).copy()
    return out


# ----------------------------------------------------------------------------
# synthetic scenes (SURVEY.md §8d recipe)
# ----------------------------------------------------------------------------
def synth_batch(sizes, seed, n_labels=5, obs_len=8, pred_len=12):
    rng = np.random.default_rng(seed)
    T = obs_len + pred_len
    B = int(sum(sizes))
    start = rng.uniform(0, 15, size=(B, 2))
    vel = rng.normal(0, 0.3, size=(B, 2))
    jit = rng.normal(0, 0.05, size=(T, B, 2))
    steps = vel[None] + jit
    steps[0] = 0.0
    abs_ = start[None] + np.cumsum(steps, axis=0)
    rel = np.zeros_like(abs_)
    rel[1:] = abs_[1:] - abs_[:-1]
    lab = rng.integers(0, n_labels, size=(B,)).astype(np.float64)
    g = np.broadcast_to(lab[None, :, None], (T, B, 1)).copy()
    off = np.concatenate([[0], np.cumsum(sizes)])
    sse = np.stack([off[:-1], off[1:]], axis=1).astype(np.int64)
    f = lambda x: torch.from_numpy(np.ascontiguousarray(x)).float()
    return dict(
        obs_traj=f(abs_[:obs_len]), pred_traj=f(abs_[obs_len:]),
        obs_traj_rel=f(rel[:obs_len]), pred_traj_rel=f(rel[obs_len:]),
        obs_traj_g=f(g[:obs_len]), pred_traj_g=f(g[obs_len:]),
        non_linear_ped=torch.zeros(B), loss_mask=torch.ones(B, T),
        seq_start_end=torch.from_numpy(sse))


def label_patterns(sizes, seed):
    """Group-label patterns covering all-singletons, one big group, mixed."""
    rng = np.random.default_rng(seed)
    labs = []
    for s, n in enumerate(sizes):
        kind = s % 4
        if kind == 0:
            l = np.zeros(n)                              # everybody ungrouped
        elif kind == 1:
            l = np.full(n, 3.0)                          # one big group
        elif kind == 2:
            l = rng.integers(0, 5, size=n).astype(float)  # mixed with label 0
        else:
            l = rng.integers(1, 1 + max(1, n // 2), size=n).astype(float)  # many small groups
        labs.append(l)
    return np.concatenate(labs)


def sse_of(sizes):
    off = np.concatenate([[0], np.cumsum(sizes)])
    return torch.from_numpy(np.stack([off[:-1], off[1:]], 1).astype(np.int64))


def save(name, arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print("wrote", path, "%.1f KB" % (os.path.getsize(path) / 1024))


# ----------------------------------------------------------------------------
# fixtures
# ----------------------------------------------------------------------------
POOL_SIZES = [1, 2, 5, 20, 57, 64, 3, 20]


def fx_weights():
    g, d = build_models(0)
    arr = {}
    arr.update(sd_arrays(g, "g/"))
    arr.update(sd_arrays(d, "d/"))
    save("weights.npz", arr)


def fx_pool():
    """PoolHiddenNet fwd + bwd, models.py:497-549, for G (h32->8) and D (h48->48)."""
    g, d = build_models(0)
    out = {}
    for tag, net, hd in (("g", g.pool_net, 32), ("d", d.pool_net, 48)):
        torch.manual_seed(11 if tag == "g" else 12)
        B = sum(POOL_SIZES)
        h = torch.randn(1, B, hd, requires_grad=True)
        pos = (torch.rand(B, 2) * 15.0)
        sse = sse_of(POOL_SIZES)
        y = net(h, sse, pos)
        dy = torch.randn_like(y)
        net.zero_grad()
        (y * dy).sum().backward()
        out[tag + "/h"] = h.detach().numpy()[0]
        out[tag + "/pos"] = pos.numpy()
        out[tag + "/sse"] = sse.numpy()
        out[tag + "/out"] = y.detach().numpy()
        out[tag + "/dout"] = dy.numpy()
        out[tag + "/dh"] = h.grad.numpy()[0]
        for k, p in net.named_parameters():
            out[tag + "/w/" + k] = p.detach().numpy()
            out[tag + "/dw/" + k] = p.grad.numpy()
    save("pool.npz", out)


GRAPH_SIZES = [1, 2, 5, 20, 20, 33, 57, 64, 7, 12, 20, 20]


def _graph_module_fixture(name, build_mod, seed):
    torch.manual_seed(seed)
    mod = build_mod()
    B = sum(GRAPH_SIZES)
    x = torch.randn(B, 40, requires_grad=True)
    lab = torch.from_numpy(label_patterns(GRAPH_SIZES, seed)).float().view(B, 1)
    sse = sse_of(GRAPH_SIZES)
    end_pos = torch.zeros(B, 2)
    y = mod(x, sse, end_pos, lab)
    dy = torch.randn_like(y)
    mod.zero_grad()
    (y * dy).sum().backward()
    out = dict(x=x.detach().numpy(), labels=lab.numpy()[:, 0], sse=sse.numpy(), out=y.detach().numpy(),
               dout=dy.numpy(), dx=x.grad.numpy())
    for k, p in mod.named_parameters():
        out["w/" + k] = p.detach().numpy()
        if p.grad is not None:
            out["dw/" + k] = p.grad.numpy()
    save(name, out)


def fx_gat():
    # GATEncoder, models.py:239-294 (dims hard-coded 40->72->16, 16->72->16, 32->24)
    _graph_module_fixture("gat_encoder.npz", lambda: M.GATEncoder(n_units=[40, 16, 40], n_heads=1, dropout=0, alpha=0.2), 21)
    # n_heads=2 variant exercises concat of heads (models.py:226-234)
    _graph_module_fixture("gat_encoder_h2.npz", lambda: M.GATEncoder(n_units=[40, 16, 40], n_heads=2, dropout=0, alpha=0.2), 22)


def fx_gcn():
    # GCNModule, models.py:583-712 (input 40, hidden 72, out 16, final 24)
    def mk():
        m = M.GCNModule(input_dim=40, hidden_dim=72, out_dim=16, gcn_layers=2, final_dim=24)
        # randn init (models.py:567-571) blows activations up by ~x50 per layer;
        # keep it, it is what the reference trains from.
        return m
    _graph_module_fixture("gcn_module.npz", mk, 31)


def _gen_forward(g, batch, noise, mode):
    """TrajectoryGenerator.forward, models.py:862-927; mode 'gcn' swaps in the
    commented call at models.py:902 (the sgan-g-p checkpoint family)."""
    if mode == "gat":
        return g(batch["obs_traj"], batch["obs_traj_rel"], batch["seq_start_end"], batch["obs_traj_g"], user_noise=noise)
    obs_traj, obs_rel, sse, obs_g = batch["obs_traj"], batch["obs_traj_rel"], batch["seq_start_end"], batch["obs_traj_g"]
    Bn = obs_rel.size(1)
    h = g.encoder(obs_rel)
    end_pos = obs_traj[-1]
    pool_h = g.pool_net(h, sse, end_pos)
    ctx = torch.cat([h.view(-1, g.encoder_h_dim), pool_h], dim=1)
    ni = g.gcn_module(ctx, sse, end_pos, obs_g[-1])
    dh = g.add_noise(ni, sse, user_noise=noise).unsqueeze(0)
    dc = torch.zeros(g.num_layers, Bn, g.decoder_h_dim)
    out, _ = g.decoder(obs_traj[-1], obs_rel[-1], (dh, dc), sse)
    return out


def real_batch(split="zara1", dset_type="test", n_scenes=16):
    path = os.path.join(REF, "datasets_group", split, dset_type)
    dset = DL.TrajectoryDataset(path, obs_len=8, pred_len=12, skip=1, delim="tab")
    from sgan.data.trajectories_GCN import seq_collate
    items = [dset[i] for i in range(min(n_scenes, len(dset)))]
    t = seq_collate(items)
    keys = ["obs_traj", "pred_traj", "obs_traj_rel", "pred_traj_rel", "obs_vel", "pred_vel",
            "obs_traj_g", "pred_traj_g", "non_linear_ped", "loss_mask", "seq_start_end"]
    return dict(zip(keys, t))


def fx_gen():
    g, d = build_models(0)
    batches = {"synth": synth_batch([20] * 6 + [2, 5, 33], seed=5), "zara1": real_batch("zara1", "test", 16)}
    for mode in ("gat", "gcn"):
        out = {}
        for bname, b in batches.items():
            S = b["seq_start_end"].size(0)
            torch.manual_seed(77)
            noise = torch.randn(S, 8)
            g.zero_grad()
            y = _gen_forward(g, b, noise, mode)
            dy = torch.randn_like(y)
            (y * dy).sum().backward()
            pre = bname + "/"
            for k in ("obs_traj", "obs_traj_rel", "obs_traj_g", "seq_start_end", "pred_traj", "pred_traj_rel"):
                out[pre + k] = b[k].numpy()
            out[pre + "noise"] = noise.numpy()
            out[pre + "out"] = y.detach().numpy()
            out[pre + "dout"] = dy.numpy()
            for k, v in grad_arrays(g, pre + "dw/").items():
                out[k] = v
        save("gen_fwd_%s.npz" % mode, out)


# ----------------------------------------------------------------------------
# sgangat family: the commented batched-GAT text of sgan/GAT.py:6-106
# ----------------------------------------------------------------------------
def _ref_sgat_classes():
    """Un-comment sgan/GAT.py lines 6-106 (BatchMultiHeadGraphAttention, GAT,
    GATEncoder) and execute that text in a private namespace.  Nothing is
    written to the repo; the module is imported this way only to produce the
    reference outputs for the sgangat checkpoint family."""
    lines = open(os.path.join(REF, "sgan/GAT.py")).read().split("\n")[5:106]
    src = "\n".join(l[2:] if l.startswith("# ") else "" for l in lines)
    ns = dict(torch=torch, nn=torch.nn, F=torch.nn.functional, np=np)
    exec(compile(src, "sgan/GAT.py:6-106 (commented text)", "exec"), ns)
    return ns


SGAT = None
SGAT_SIZES = [2, 5, 20, 20, 33, 57, 64, 7, 12, 20, 20, 3]   # the instance norm needs >= 2 peds


def build_sgangat(seed=0):
    """Generator of the sgangat-g-p family: build_models(seed)'s G (encoder,
    decoder, pool_net, gcn_module) + the batched GAT (heads 4,1; units
    40,16,40 from the checkpoint args) + mlp_decoder_context [40, 64, 24]."""
    global SGAT
    if SGAT is None:
        SGAT = _ref_sgat_classes()
    g, _ = build_models(seed)
    torch.manual_seed(seed + 500)
    sg = SGAT["GATEncoder"]([40, 16, 40], [4, 1], 0.0, 0.2)
    for layer in sg.gat_net.layer_stack:           # bias is zero-init (GAT.py:21); exercise it
        layer.bias.data.normal_(0.0, 0.1)
    mdc = M.make_mlp([40, 64, 24], activation="relu", batch_norm=False, dropout=0.0)
    return g, sg, mdc


def _sgat_call(sg, x, sse):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):      # GAT.py:101-102 print per scene
        return sg(x.unsqueeze(0), sse)[0]


def _sgangat_forward(g, sg, batch, noise):
    obs_traj, obs_rel, sse, obs_g = batch["obs_traj"], batch["obs_traj_rel"], batch["seq_start_end"], batch["obs_traj_g"]
    Bn = obs_rel.size(1)
    h = g.encoder(obs_rel)
    end_pos = obs_traj[-1]
    ctx = torch.cat([h.view(-1, g.encoder_h_dim), g.pool_net(h, sse, end_pos)], dim=1)
    ctx = _sgat_call(sg, ctx, sse)
    ni = g.gcn_module(ctx, sse, end_pos, obs_g[-1])
    dh = g.add_noise(ni, sse, user_noise=noise).unsqueeze(0)
    dc = torch.zeros(g.num_layers, Bn, g.decoder_h_dim)
    out, _ = g.decoder(obs_traj[-1], obs_rel[-1], (dh, dc), sse)
    return out


def _sgangat_state(g, sg, mdc, grads=False):
    """State dict (or grads) under the sgangat checkpoint's key names."""
    out = {}
    for prefix, mod in (("", g), ("gatencoder.", sg), ("mlp_decoder_context.", mdc)):
        for k, p in mod.named_parameters():
            if prefix == "" and k.startswith("gatencoder."):
                continue
            if grads:
                if p.grad is not None:
                    out[prefix + k] = p.grad.detach().numpy().copy()
            else:
                out[prefix + k] = p.detach().numpy().copy()
    return out


def fx_sgangat():
    # batched GAT module alone: fwd + bwd over scenes of 2..64 peds
    g, sg, mdc = build_sgangat(0)
    torch.manual_seed(61)
    B = sum(SGAT_SIZES)
    x = torch.randn(B, 40, requires_grad=True)
    sse = sse_of(SGAT_SIZES)
    y = _sgat_call(sg, x, sse)
    dy = torch.randn_like(y)
    sg.zero_grad()
    (y * dy).sum().backward()
    out = dict(x=x.detach().numpy(), sse=sse.numpy(), out=y.detach().numpy(), dout=dy.numpy(), dx=x.grad.numpy())
    for k, p in sg.named_parameters():
        out["w/" + k] = p.detach().numpy()
        out["dw/" + k] = p.grad.numpy()
    save("sgangat_gat.npz", out)
    # the whole generator
    batches = {"synth": synth_batch([20] * 6 + [2, 5, 33], seed=5), "zara1": real_batch("zara1", "test", 16)}
    out = {}
    for k, v in _sgangat_state(g, sg, mdc).items():
        out["w/" + k] = v
    for bname, b in batches.items():
        S = b["seq_start_end"].size(0)
        torch.manual_seed(77)
        noise = torch.randn(S, 8)
        g.zero_grad()
        sg.zero_grad()
        y = _sgangat_forward(g, sg, b, noise)
        dy = torch.randn_like(y)
        (y * dy).sum().backward()
        pre = bname + "/"
        for k in ("obs_traj", "obs_traj_rel", "obs_traj_g", "seq_start_end", "pred_traj", "pred_traj_rel"):
            out[pre + k] = b[k].numpy()
        out[pre + "noise"] = noise.numpy()
        out[pre + "out"] = y.detach().numpy()
        out[pre + "dout"] = dy.numpy()
        for k, v in _sgangat_state(g, sg, mdc, grads=True).items():
            out[pre + "dw/" + k] = v
    save("gen_fwd_sgangat.npz", out)


# ----------------------------------------------------------------------------
# vanilla family (upstream Social-GAN: sgan-models / sgan-p-models)
# ----------------------------------------------------------------------------
def build_vanilla(pooling, seed=0):
    """Generator of the sgan-models (pooling None, BASELINE configs[0]) /
    sgan-p-models (pool_net) families: the reference's own TrajectoryGenerator
    built with those checkpoints' args (read as text from
    models/sgan-models/eth_12_model.pt: embedding 16, encoder/decoder h 32,
    mlp 64, noise (8,) gaussian 'global', pooling 'none', bottleneck 8,
    batch_norm 0) plus the mlp_decoder_context the committed file comments
    out (models.py:796-804), built by the reference's make_mlp.  Its
    gatencoder / gcn_module are constructed by the reference but not part of
    the family (dropped from the saved state)."""
    torch.manual_seed(seed)
    g = M.TrajectoryGenerator(
        obs_len=8, pred_len=12, embedding_dim=16, encoder_h_dim=32, decoder_h_dim=32, mlp_dim=64,
        num_layers=1, noise_dim=(8,), noise_type="gaussian", noise_mix_type="global",
        pooling_type=pooling or "none", pool_every_timestep=False, dropout=0.0, bottleneck_dim=8,
        batch_norm=False, n_units=[40, 16, 40], n_heads=1, dropout1=0, alpha=0.2)
    in_dim = 32 + 8 if pooling else 32
    g.mlp_decoder_context = M.make_mlp([in_dim, 64, 32 - 8], activation="relu", batch_norm=False, dropout=0.0)
    g.apply(TR.init_weights)
    g.train()
    return g


def _vanilla_forward(g, batch, noise):
    """TrajectoryGenerator.forward (models.py:862-927) with the upstream
    context line models.py:898 (noise_input = mlp_decoder_context(ctx)) in
    place of the GAT call :903-905."""
    obs_traj, obs_rel, sse = batch["obs_traj"], batch["obs_traj_rel"], batch["seq_start_end"]
    Bn = obs_rel.size(1)
    h = g.encoder(obs_rel)
    ctx = h.view(-1, g.encoder_h_dim)
    if g.pooling_type:                                                      # :878-886
        ctx = torch.cat([ctx, g.pool_net(h, sse, obs_traj[-1])], dim=1)
    ni = g.mlp_decoder_context(ctx)                                         # :898
    dh = g.add_noise(ni, sse, user_noise=noise).unsqueeze(0)                # :909-910
    dc = torch.zeros(g.num_layers, Bn, g.decoder_h_dim)
    out, _ = g.decoder(obs_traj[-1], obs_rel[-1], (dh, dc), sse)
    return out


def _vanilla_state(g, grads=False):
    out = {}
    for k, p in g.named_parameters():
        if k.startswith("gatencoder.") or k.startswith("gcn_module."):
            continue
        if grads:
            if p.grad is not None:
                out[k] = p.grad.detach().numpy().copy()
        else:
            out[k] = p.detach().numpy().copy()
    return out


def fx_vanilla():
    out = {}
    batches = {"synth": synth_batch([20] * 6 + [2, 5, 33], seed=5), "zara1": real_batch("zara1", "test", 16),
               "eth": real_batch("eth", "test", 16)}
    for tag, pooling in (("none", None), ("pool", "pool_net")):
        g = build_vanilla(pooling, 0)
        for k, v in _vanilla_state(g).items():
            out[tag + "/w/" + k] = v
        for bname, b in batches.items():
            S = b["seq_start_end"].size(0)
            torch.manual_seed(77)
            noise = torch.randn(S, 8)
            g.zero_grad()
            y = _vanilla_forward(g, b, noise)
            dy = torch.randn_like(y)
            (y * dy).sum().backward()
            pre = "%s/%s/" % (tag, bname)
            for k in ("obs_traj", "obs_traj_rel", "obs_traj_g", "seq_start_end", "pred_traj", "pred_traj_rel"):
                out[pre + k] = b[k].numpy()
            out[pre + "noise"] = noise.numpy()
            out[pre + "out"] = y.detach().numpy()
            out[pre + "dout"] = dy.numpy()
            for k, v in _vanilla_state(g, grads=True).items():
                out[pre + "dw/" + k] = v
    save("gen_fwd_vanilla.npz", out)


def fx_disc():
    g, d = build_models(0)
    b = synth_batch([20] * 4 + [2, 9], seed=6)
    traj = torch.cat([b["obs_traj"], b["pred_traj"]], 0)
    traj_rel = torch.cat([b["obs_traj_rel"], b["pred_traj_rel"]], 0).requires_grad_(True)
    d.zero_grad()
    s = d(traj, traj_rel, b["seq_start_end"])
    ds = torch.randn_like(s)
    (s * ds).sum().backward()
    # also the pre-classifier features (trailing ReLU zeroes most scores)
    feat = d.pool_net(d.encoder(traj_rel).squeeze(), b["seq_start_end"], traj[0])
    out = dict(traj=traj.numpy(), traj_rel=traj_rel.detach().numpy(), sse=b["seq_start_end"].numpy(),
               scores=s.detach().numpy(), dscores=ds.numpy(), dtraj_rel=traj_rel.grad.numpy(),
               feat=feat.detach().numpy())
    out.update(grad_arrays(d, "dw/"))
    save("disc_fwd.npz", out)


class _RecordingAdam(torch.optim.Adam):
    """torch.optim.Adam that records every parameter's .grad when step() is
    called, i.e. after loss.backward() and after the reference's
    clip_grad_norm_ (train.py:423-427, 478-482), before the update."""

    def __init__(self, named, rec, **kw):
        named = list(named)
        super().__init__([p for _, p in named], **kw)
        self._named, self._rec = named, rec

    def step(self, closure=None):
        self._rec.append({k: p.grad.detach().numpy().copy() for k, p in self._named if p.grad is not None})
        return super().step(closure)


def fx_train_step():
    """discriminator_step + generator_step (scripts/train.py:395-484), 2 iterations,
    fresh Adam, seeded host RNGs (noise: torch CPU RNG, label smoothing: random).
    Also records the gradients each optimizer step consumes (D: raw; G: after
    clip_grad_norm_ 2.0) as it%d/gradD/<param>, it%d/gradG/<param>."""
    g, d = build_models(0)
    rec_g, rec_d = [], []
    opt_g = _RecordingAdam(g.named_parameters(), rec_g, lr=ARGS.g_learning_rate)
    opt_d = _RecordingAdam(d.named_parameters(), rec_d, lr=ARGS.d_learning_rate)
    out = {}
    batches = [synth_batch([20] * 5 + [7], seed=41), synth_batch([20] * 4 + [3, 12], seed=42)]
    torch.manual_seed(1234)
    random.seed(1234)
    keys = ["obs_traj", "pred_traj", "obs_traj_rel", "pred_traj_rel", "obs_vel", "pred_vel",
            "obs_traj_g", "pred_traj_g", "non_linear_ped", "loss_mask", "seq_start_end"]
    for it, b in enumerate(batches):
        b = dict(b)
        b["obs_vel"] = b["obs_traj_rel"] * 2.5
        b["pred_vel"] = b["pred_traj_rel"] * 2.5
        tup = [b[k] for k in keys]
        for k in keys:
            out["b%d/%s" % (it, k)] = b[k].numpy()
        ld = TR.discriminator_step(ARGS, tup, g, d, TR.gan_d_loss, opt_d)
        lg = TR.generator_step(ARGS, tup, g, d, TR.gan_g_loss, opt_g)
        for k, v in ld.items():
            out["it%d/D/%s" % (it, k)] = np.float64(v)
        for k, v in lg.items():
            out["it%d/G/%s" % (it, k)] = np.float64(v)
        out.update(sd_arrays(g, "it%d/g/" % it))
        out.update(sd_arrays(d, "it%d/d/" % it))
        for k, v in rec_d[-1].items():
            out["it%d/gradD/%s" % (it, k)] = v
        for k, v in rec_g[-1].items():
            out["it%d/gradG/%s" % (it, k)] = v
    save("train_step.npz", out)


EVAL_MODES = ("gat", "gcn", "sgangat", "vanilla", "vanilla_p")


def fx_eval(splits, modes=EVAL_MODES):
    """scripts/evaluate_model.py:72-99 on the test split, 20 samples, seeded host RNG,
    seeded random-init weights (trained checkpoints are not loadable with the
    safe loader: they hold collections.defaultdict).  Also the vanilla family
    on ETH with batch_size 1 (BASELINE configs[0]) as 'vanilla_b1/eth'.
    Entries are merged into the existing evaluate.json."""
    path_json = os.path.join(HERE, "evaluate.json")
    res = json.load(open(path_json)) if os.path.exists(path_json) else {}
    runs = [(m, sp, 64) for m in modes for sp in splits]
    if "vanilla" in modes and "eth" in splits:
        runs.append(("vanilla_b1", "eth", 1))
    for mode, split, bs in runs:
        g, _ = build_models(0)
        if mode.startswith("vanilla"):
            g = build_vanilla("pool_net" if mode == "vanilla_p" else None, 0)
            g.forward = types.MethodType(
                lambda self, ot, orl, sse, og, user_noise=None: _vanilla_forward(
                    self, dict(obs_traj=ot, obs_traj_rel=orl, seq_start_end=sse), user_noise), g)
        if mode == "sgangat":
            g, sg, _ = build_sgangat(0)
            g.forward = types.MethodType(
                lambda self, ot, orl, sse, og, user_noise=None, sg=sg: _sgangat_forward(
                    self, sg, dict(obs_traj=ot, obs_traj_rel=orl, seq_start_end=sse, obs_traj_g=og), user_noise),
                g)
        if mode == "gcn":
            g.forward = types.MethodType(
                lambda self, ot, orl, sse, og, user_noise=None: _gen_forward(
                    self, dict(obs_traj=ot, obs_traj_rel=orl, seq_start_end=sse, obs_traj_g=og), user_noise, "gcn"), g)
        path = os.path.join(REF, "datasets_group", split, "test")
        a = EV.AttrDict(dict(vars(ARGS)))
        a["batch_size"] = bs
        _, loader = DL.data_loader(a, path)
        torch.manual_seed(0)
        t0 = time.time()
        ade, fde = EV.evaluate(a, loader, g, 20)
        res["%s/%s" % (mode, split)] = dict(ade=float(ade), fde=float(fde), seconds=time.time() - t0,
                                             num_seq=len(loader.dataset))
        print(mode, split, res["%s/%s" % (mode, split)], flush=True)
    with open(path_json, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


# ----------------------------------------------------------------------------
# trained checkpoints of the configs[0] families (sgan-models / sgan-p-models)
# ----------------------------------------------------------------------------
TRAINED = [("sgan-models", s, 12) for s in SPLITS] + [("sgan-p-models", s, 12) for s in SPLITS] + \
          [("sgan-models", "eth", 8), ("sgan-p-models", "zara1", 8)]
TRAINED_ARGS = ("obs_len", "pred_len", "embedding_dim", "encoder_h_dim_g", "decoder_h_dim_g", "mlp_dim", "num_layers",
                "noise_dim", "noise_type", "noise_mix_type", "pooling_type", "pool_every_timestep", "dropout",
                "bottleneck_dim", "neighborhood_size", "grid_size", "batch_norm", "skip", "delim", "dataset_name")


def safe_load(path):
    """torch.load with the weights-only unpickler (no code from the file is
    executed); collections.defaultdict is allow-listed because the upstream
    checkpoints store their metric histories in one.  The group-family
    checkpoints (sgan-gat, sgan-g(-p), sgangat) are refused by this loader
    (SETITEMS on a defaultdict) and are not used."""
    import collections
    with torch.serialization.safe_globals([collections.defaultdict]):
        return torch.load(path, weights_only=True, map_location="cpu")


def fx_trained():
    """Trained upstream Social-GAN checkpoints (BASELINE configs[0]: the
    sgan-models family; and sgan-p-models): their g_state and args, and the
    reference's best-of-20 ADE / FDE on the test split (evaluate_model.py:
    72-99 with the upstream context line models.py:898, seed 0), batch 64 on
    every split, plus ETH at batch_size 1 for sgan-models/eth_12 (configs[0]
    literally).  -> trained.npz, evaluate_trained.json"""
    arrs, res = {}, {}
    for fam, split, pl in TRAINED:
        tag = "%s/%s_%d" % (fam, split, pl)
        ck = safe_load(os.path.join(REF, "models", fam, "%s_%d_model.pt" % (split, pl)))
        a = dict(ck["args"])
        for k, v in ck["g_state"].items():
            arrs[tag + "/g/" + k] = v.numpy().copy()
        res.setdefault("args", {})[tag] = {k: a[k] for k in TRAINED_ARGS}
        pooling = a["pooling_type"] if a["pooling_type"] not in (None, "none") else None
        g = M.TrajectoryGenerator(
            obs_len=a["obs_len"], pred_len=a["pred_len"], embedding_dim=a["embedding_dim"],
            encoder_h_dim=a["encoder_h_dim_g"], decoder_h_dim=a["decoder_h_dim_g"], mlp_dim=a["mlp_dim"],
            num_layers=a["num_layers"], noise_dim=a["noise_dim"], noise_type=a["noise_type"],
            noise_mix_type=a["noise_mix_type"], pooling_type=a["pooling_type"],
            pool_every_timestep=a["pool_every_timestep"], dropout=a["dropout"], bottleneck_dim=a["bottleneck_dim"],
            neighborhood_size=a["neighborhood_size"], grid_size=a["grid_size"], batch_norm=a["batch_norm"],
            n_units=[40, 16, 40], n_heads=1, dropout1=0, alpha=0.2)
        in_dim = a["encoder_h_dim_g"] + (a["bottleneck_dim"] if pooling else 0)
        g.mlp_decoder_context = M.make_mlp([in_dim, a["mlp_dim"], a["decoder_h_dim_g"] - a["noise_dim"][0]],
                                           activation="relu", batch_norm=a["batch_norm"], dropout=a["dropout"])
        r = g.load_state_dict(ck["g_state"], strict=False)
        assert not r.unexpected_keys, r.unexpected_keys
        assert all(k.startswith(("gatencoder.", "gcn_module.")) for k in r.missing_keys), r.missing_keys
        g.train()
        g.forward = types.MethodType(
            lambda self, ot, orl, sse, og, user_noise=None: _vanilla_forward(
                self, dict(obs_traj=ot, obs_traj_rel=orl, seq_start_end=sse), user_noise), g)
        batches = [64] + ([1] if (fam, split, pl) == ("sgan-models", "eth", 12) else [])
        for bs in batches:
            ea = EV.AttrDict(dict(a))
            ea["batch_size"], ea["loader_num_workers"] = bs, 0
            _, loader = DL.data_loader(ea, os.path.join(REF, "datasets_group", split, "test"))
            torch.manual_seed(0)
            t0 = time.time()
            ade, fde = EV.evaluate(ea, loader, g, 20)
            res["%s/b%d" % (tag, bs)] = dict(ade=float(ade), fde=float(fde), seconds=time.time() - t0,
                                             num_seq=len(loader.dataset))
            print(tag, bs, res["%s/b%d" % (tag, bs)], flush=True)
    save("trained.npz", arrs)
    with open(os.path.join(HERE, "evaluate_trained.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


def copy_test_data():
    for split in SPLITS:
        src = os.path.join(REF, "datasets_group", split, "test")
        dst = os.path.join(HERE, "datasets_group", split, "test")
        os.makedirs(dst, exist_ok=True)
        for f in os.listdir(src):
            shutil.copyfile(os.path.join(src, f), os.path.join(dst, f))


def _time_iters(disc_step, gen_step, b, n):
    disc_step(b)                                        # warm-up (not timed)
    t0 = time.perf_counter()
    for _ in range(n):
        disc_step(b)
        gen_step(b)
    return (time.perf_counter() - t0) / n


def fx_cpu_timing(batch=64, threads=8, iters=2):
    """CPU train-iteration timing on this host of the REAL
    reference (scripts/train.py discriminator_step + generator_step) and of
    the oracle's reference formulation (oracle/sgan_oracle.py, what bench.py's
    cpu_baseline leg times on the GPU box) on the same synthetic batch, same
    thread count; the two must agree within +-20 % for the oracle to stand in
    for the reference (SURVEY.md:450-453)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import sgan_oracle as O
    torch.set_num_threads(threads)
    keys = ["obs_traj", "pred_traj", "obs_traj_rel", "pred_traj_rel", "obs_vel", "pred_vel",
            "obs_traj_g", "pred_traj_g", "non_linear_ped", "loss_mask", "seq_start_end"]
    b = synth_batch([20] * batch, seed=0)
    b["obs_vel"] = b["obs_traj_rel"] * 2.5
    b["pred_vel"] = b["pred_traj_rel"] * 2.5
    tup = [b[k] for k in keys]
    g, d = build_models(0)
    opt_g = torch.optim.Adam(g.parameters(), lr=ARGS.g_learning_rate)
    opt_d = torch.optim.Adam(d.parameters(), lr=ARGS.d_learning_rate)
    dt_ref = _time_iters(lambda x: TR.discriminator_step(ARGS, x, g, d, TR.gan_d_loss, opt_d),
                         lambda x: TR.generator_step(ARGS, x, g, d, TR.gan_g_loss, opt_g), tup, iters)
    torch.manual_seed(0)
    og, od = O.build_default("gat")
    oopt_g = torch.optim.Adam(og.parameters(), lr=1e-4)
    oopt_d = torch.optim.Adam(od.parameters(), lr=1e-3)
    dt_orc = _time_iters(lambda x: O.discriminator_step(O.Args, x, og, od, oopt_d),
                         lambda x: O.generator_step(O.Args, x, og, od, oopt_g), tup, iters)
    ratio = dt_ref / dt_orc
    res = dict(reference_scenes_per_s=batch / dt_ref, oracle_scenes_per_s=batch / dt_orc,
               oracle_over_reference=ratio, threads=threads, batch=batch, n_peds=20, iters=iters,
               cpu=_cpu_model(), note="D-step + G-step (best_k=20) per iteration, 1 warm-up D-step")
    print("cpu timing", res)
    with open(os.path.join(HERE, "ref_cpu_timing.json"), "w") as f:
        json.dump(res, f, indent=1)
    assert 0.8 <= ratio <= 1.2, "oracle reference formulation is not within 20%% of the reference: %.3f" % ratio


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


ALL = dict(weights=fx_weights, pool=fx_pool, gat=fx_gat, gcn=fx_gcn, gen=fx_gen, sgangat=fx_sgangat,
           vanilla=fx_vanilla, disc=fx_disc, trained=fx_trained,
           train=fx_train_step, data=copy_test_data, timing=fx_cpu_timing)

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--skip-eval", action="store_true")
    ap.add_argument("--splits", nargs="*", default=SPLITS)
    ap.add_argument("--modes", nargs="*", default=list(EVAL_MODES))
    a = ap.parse_args()
    names = a.only if a.only else list(ALL)
    for n in names:
        if n == "eval":
            continue
        t0 = time.time()
        ALL[n]()
        print("[%s] %.1fs" % (n, time.time() - t0), flush=True)
    if (a.only is None and not a.skip_eval) or (a.only and "eval" in a.only):
        fx_eval(a.splits, tuple(a.modes))
