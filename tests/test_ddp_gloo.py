"""Scene-sharded data parallelism (sgan/train_step.py) on CPU with gloo,
world_size 2: one D-step + G-step on a global batch split across ranks must
equal the single-process step on the whole batch (losses and weights).  The
models are the CPU oracle's behind a thin adapter: this checks the host-side
DP logic (sharding, global noise draw and slicing, loss scaling, the one
flat all-reduce, clipping after the reduce), not the kernels."""
import os
import random
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN

SIZES = [20, 7, 13, 2, 20, 9]


class _Adapt(torch.nn.Module):
    """Oracle module with the product's keyword-only `scenes=` argument."""

    def __init__(self, m):
        super().__init__()
        self.m = m

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.m, name)

    def forward(self, *a, scenes=None, **k):
        return self.m(*a, **k)

    # the product generator's context() / decode() split of forward(),
    # restated over the oracle's submodules (models.py:877-925)
    def context(self, obs_traj, obs_traj_rel, seq_start_end, obs_traj_g, scenes=None):
        g = self.m
        h = g.encoder(obs_traj_rel)
        ctx = h.view(-1, g.encoder_h_dim)
        if g.pooling_type:
            ctx = torch.cat([ctx, g.pool_net(h, seq_start_end, obs_traj[-1])], 1)
        return g.gatencoder(ctx, seq_start_end, obs_traj[-1], obs_traj_g[-1])

    def decode(self, ni, obs_traj, obs_traj_rel, seq_start_end, user_noise=None, scenes=None, copies=1,
               noise_index=None):
        g = self.m
        if noise_index is not None and user_noise is not None:   # (K, S, nz) draws, picked per copy
            best, first_k = noise_index
            parts = [user_noise[best, torch.arange(scenes.S)]] if best is not None else []
            parts += [user_noise[first_k + r] for r in range(copies - len(parts))]
            user_noise = torch.cat(parts, 0)
        sc = scenes.repeat(copies)
        sse = torch.from_numpy(np.stack([sc.host_off[:-1], sc.host_off[1:]], 1))
        dh = g.add_noise(ni.repeat(copies, 1), sse, user_noise).unsqueeze(0)
        dc = torch.zeros(1, sc.B, g.decoder_h_dim)
        out, _ = g.decoder(obs_traj[-1].repeat(copies, 1), obs_traj_rel[-1].repeat(copies, 1), (dh, dc), sse)
        return out


def _models():
    from oracle import sgan_oracle as O
    w = np.load(os.path.join(GOLDEN, "weights.npz"))
    g, d = O.build_default("gat")
    g.load_state_dict({k[2:]: torch.from_numpy(w[k]) for k in w.files if k.startswith("g/")})
    d.load_state_dict({k[2:]: torch.from_numpy(w[k]) for k in w.files if k.startswith("d/")})
    return _Adapt(g), _Adapt(d)


def _bce_pair(scores, split, y_a, y_b, w=1.0):
    """Torch restatement of kernels.bce_pair over the oracle's bce_loss."""
    from oracle import sgan_oracle as O
    x = scores.reshape(-1)
    a, b = x[:split], x[split:]
    terms = [O.bce_loss(t, torch.ones_like(t) * y) for t, y in ((a, y_a), (b, y_b)) if t.numel()]
    return w * sum(terms)


class _TorchClipAdam:
    """Torch restatement of kernels.ClipAdam (adam.hip)."""

    def __init__(self, params, lr):
        self.params = list(params)
        self.opt = torch.optim.Adam(self.params, lr=lr)

    def zero_grad(self, set_to_none=True):
        self.opt.zero_grad(set_to_none=set_to_none)

    def step(self, max_norm=0.0):
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_(self.params, max_norm)
        self.opt.step()


class _TorchOps:
    """Torch restatement of train_step.KernelOps (glue.hip / loss.hip / adam.hip)."""
    optimizer = staticmethod(_TorchClipAdam)

    @staticmethod
    def traj_cat(head, a, b=None, pos0=None):
        if b is None:
            out = torch.cat([head, a], 0)
        else:
            out = torch.cat([torch.cat([head, a], 0), torch.cat([head, b], 0)], 1)
        if pos0 is None:
            return out
        return out, pos0.reshape(1, -1, 2).repeat(1, out.shape[1] // pos0.reshape(-1, 2).shape[0], 1)

    @staticmethod
    def l2_select(pred, gt, mask, scenes, k):
        T, B = gt.shape[0], gt.shape[1]
        l2 = ((gt.unsqueeze(1) - pred.view(T, k, B, 2)) ** 2).sum(3) * mask.t().unsqueeze(1)
        seg = scenes.ped_scene_long()
        return torch.zeros(k, scenes.S).index_add_(1, seg, l2.sum(0)).argmin(0)

    @staticmethod
    def l2_loss(pred, gt, mask, scenes, w=1.0):
        seg = scenes.ped_scene_long()
        l2 = (mask.t().unsqueeze(2) * (gt - pred) ** 2).sum((0, 2))
        num = torch.zeros(scenes.S).index_add_(0, seg, w * l2)
        den = torch.zeros(scenes.S).index_add_(0, seg, mask.sum(1))
        return (num / den).sum()

    bce_pair = staticmethod(_bce_pair)
    split2 = staticmethod(lambda x, B: (x[:, :B], x[:, B:]))
    one = staticmethod(lambda device: torch.ones((), device=device))


def _run(rank, world, port, out):
    from sgan.data.synthetic import synthetic_batch
    from sgan.scene import SceneIndex
    from sgan.train_step import DataParallel, GanTrainer, shard_batch
    torch.set_num_threads(1)
    if world > 1:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    g, d = _models()
    tr = GanTrainer(g, d, dp=DataParallel(), ops=_TorchOps())
    batch = synthetic_batch(SIZES, seed=11)
    sc = SceneIndex(np.concatenate([[0], np.cumsum(SIZES)]), "cpu")
    s0, s1 = tr.dp.shard(sc.S)
    local, lsc = shard_batch(batch, sc, s0, s1)
    torch.manual_seed(5)
    random.seed(5)
    losses = []
    for _ in range(2):
        ld, lg = tr.step(local, lsc, S_global=sc.S, B_global=sc.B, shard=(s0, s1))
        losses.append([float(v) for v in list(ld.values()) + list(lg.values())])
    if rank == 0:
        torch.save({"g": g.m.state_dict(), "d": d.m.state_dict(), "losses": losses}, out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_two_rank_step_equals_single_process():
    with tempfile.TemporaryDirectory() as td:
        single, multi = os.path.join(td, "single.pt"), os.path.join(td, "multi.pt")
        _run(0, 1, 0, single)
        mp.spawn(_run, args=(2, _free_port(), multi), nprocs=2, join=True)
        a = torch.load(single, weights_only=True)
        b = torch.load(multi, weights_only=True)
    for la, lb in zip(a["losses"], b["losses"]):
        np.testing.assert_allclose(la, lb, rtol=1e-5, atol=1e-6)
    for key, lr in (("g", 1e-4), ("d", 1e-3)):
        for k, v in a[key].items():
            err = (v - b[key][k]).abs().max().item()
            # Adam sign flips on noise-level gradients bound the difference (2 lr / step)
            assert err <= 4 * lr + 1e-5 * v.abs().max().item(), (key, k, err)


def test_shard_covers_scenes():
    from sgan.train_step import DataParallel
    dp = DataParallel()
    dp.world, dp.rank = 3, 0
    spans = []
    for r in range(3):
        dp.rank = r
        spans.append(dp.shard(8))
    assert spans == [(0, 3), (3, 6), (6, 8)]


def test_rccl_uid_round_trip_keeps_nul_bytes():
    """the RCCL unique id is 128 raw bytes whose sockaddr
    part holds zeros; packing must not cut it at the first NUL."""
    from sgan import rccl
    raw = bytes([0x11, 0x22, 0, 0, 2, 0, 0x1f, 0x90] + [i % 7 for i in range(120)])
    assert len(raw) == rccl.UID_BYTES and raw.count(0) > 10
    uid = rccl.unpack_uid(raw)
    assert rccl.pack_uid(uid) == raw
    assert bytes(uid.internal) != raw    # (what the round-5 code sent: cut at byte 2)
    with pytest.raises(ValueError):
        rccl.unpack_uid(raw[:9])


def _uid_rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sgan import rccl
    from sgan.train_step import DataParallel
    got = []
    for n in range(3):   # repeated exchanges of one group use distinct keys
        made = bytes([n, 0, 0, 2] + [rank] * 124)
        got.append(rccl.exchange_uid(lambda: made, None))
    dp = DataParallel()
    torch.save({"got": got, "transport": dp.transport, "capture": dp.capture, "collective": dp.collective},
               "%s.%d" % (out, rank))
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_uid_exchange_through_store_world2():
    """The id travels through the rendezvous store (no collective of any
    process group): every rank receives rank 0's 128 bytes exactly, for each
    of several exchanges in order; a gloo group's DataParallel picks the pg
    transport (never captured)."""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "uid")
        mp.spawn(_uid_rank, args=(2, _free_port(), out), nprocs=2, join=True)
        r0 = torch.load(out + ".0", weights_only=True)
        r1 = torch.load(out + ".1", weights_only=True)
    assert r0["got"] == r1["got"]
    for n, g in enumerate(r0["got"]):
        assert g == bytes([n, 0, 0, 2] + [0] * 124)
    for r in (r0, r1):
        assert r["transport"] == "pg" and not r["capture"] and r["collective"]


def test_dataparallel_transport_choice(monkeypatch):
    from sgan.train_step import DataParallel
    dp = DataParallel()   # no process group: one rank, nothing to reduce
    assert not dp.on and not dp.collective and dp.rccl is None and dp.transport == "pg"
    with pytest.raises(ValueError):
        DataParallel(transport="mpi")
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda g=None: 2)
    monkeypatch.setattr(dist, "get_rank", lambda g=None: 0)
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "nccl")
    dp = DataParallel()
    assert dp.transport == "rccl" and dp.capture and not dp.segmented
    monkeypatch.setenv("SGG_CAPTURE_COLLECTIVE", "0")
    assert DataParallel().segmented
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "gloo")
    dp = DataParallel()
    assert dp.transport == "pg" and dp.segmented
    with pytest.raises(ValueError):
        DataParallel(capture=True)          # a host collective cannot be captured
    monkeypatch.setenv("SGG_DP_TRANSPORT", "rccl")
    assert DataParallel().transport == "rccl"
