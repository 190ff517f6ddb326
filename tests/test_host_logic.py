"""Host-side logic of the product that needs no GPU: optimizer-state format,
scene sharding, trainer guards, device-scalar cache, the vanilla family's
module set.  (No kernel is launched here.)"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN  # noqa: F401  (sys.path setup)


def _gen(graph="gat", pooling="pool_net"):
    from sgan.models import TrajectoryGenerator
    return TrajectoryGenerator(8, 12, embedding_dim=16, encoder_h_dim=32, decoder_h_dim=32, mlp_dim=64,
                               noise_dim=(8,), noise_mix_type="global", pooling_type=pooling,
                               pool_every_timestep=False, bottleneck_dim=8, batch_norm=False, n_units=[40, 16, 40],
                               n_heads=[4, 1] if graph == "sgangat" else 1, dropout1=0.0, alpha=0.2, graph=graph)


def test_clip_adam_state_dict_roundtrips_reference_format():
    """A reference checkpoint's g_optim_state is torch.optim.Adam over ALL of
    G.parameters() (train.py:238, :363) with state only for the parameters
    that had gradients: ClipAdam loads it, and torch's Adam loads ClipAdam's."""
    from sgan.kernels import ClipAdam
    torch.manual_seed(0)
    g = _gen()
    ref = torch.optim.Adam(g.parameters(), lr=1e-4)
    for n, p in g.named_parameters():
        p.grad = None if n.startswith("gcn_module.") else torch.randn_like(p)
    ref.step()
    sd = ref.state_dict()
    ours = ClipAdam(g.parameters(), lr=1e-4)
    ours.load_state_dict(sd)
    out = ours.state_dict()
    assert len(out["param_groups"][0]["params"]) == len(list(g.parameters()))
    assert sorted(out["state"]) == sorted(sd["state"])
    for k, st in sd["state"].items():
        assert float(out["state"][k]["step"]) == float(st["step"]) == 1.0
        assert torch.equal(out["state"][k]["exp_avg"].cpu(), st["exp_avg"])
    back = torch.optim.Adam(g.parameters(), lr=1e-4)
    back.load_state_dict(out)
    # a fresh ClipAdam keeps no state for a parameter that never had a gradient
    assert not ClipAdam(g.parameters(), lr=1e-4).state_dict()["state"]


def test_shard_balanced_and_guarded():
    from sgan.train_step import DataParallel
    dp = DataParallel()
    dp.world = 8
    spans = []
    for r in range(8):
        dp.rank = r
        spans.append(dp.shard(9))
    assert spans[0] == (0, 2) and all(b - a == 1 for a, b in spans[1:])
    assert spans[-1][1] == 9 and all(spans[i][1] == spans[i + 1][0] for i in range(7))
    with pytest.raises(ValueError):
        dp.shard(7)


def test_trainer_rejects_batchnorm():
    from sgan.models import TrajectoryDiscriminator
    from sgan.train_step import GanTrainer
    d = TrajectoryDiscriminator(8, 12, embedding_dim=16, h_dim=48, mlp_dim=64, batch_norm=True, d_type="global")
    with pytest.raises(NotImplementedError):
        GanTrainer(_gen(), d)


def test_const_caches_only_fixed_values():
    from sgan import kernels as K
    n0 = len(K._CONST)
    for _ in range(5):
        K.const(0.913, "cpu")
    assert len(K._CONST) == n0
    assert K.const(1.0, "cpu") is K.const(1.0, "cpu")


@pytest.mark.parametrize("pooling,n", [(None, 18), ("pool_net", 24)])
def test_vanilla_family_state_dict_keys(pooling, n):
    """The vanilla family carries exactly the upstream Social-GAN module set
    (sgan-models checkpoints: encoder, decoder, [pool_net], mlp_decoder_context)."""
    g = _gen("vanilla", pooling)
    keys = [k for k, _ in g.named_parameters()]
    assert len(keys) == n
    assert not any(k.startswith(("gatencoder.", "gcn_module.")) for k in keys)
    assert "mlp_decoder_context.0.weight" in keys and "mlp_decoder_context.2.bias" in keys
    assert ("pool_net.mlp_pre_pool.0.weight" in keys) == bool(pooling)


def test_bench_traffic_table_lookups():
    """Every launch-shape entry of the committed PMC traffic tables is readable
    by bench.py's roofline (the driver's bench line must not fail on it); a
    shape no PMC run re-issued reports no traffic (null), never a mean over
    other shapes."""
    import importlib.util
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    n = 0
    for path in b.TRAFFIC_TABLES:
        if not os.path.exists(path):
            continue
        tab = json.load(open(path))
        for k in tab:
            if "|" in k:
                name, shape = k.split("|")
                shape = json.loads(shape.replace("False", "false").replace("True", "true"))
                nb, src = b.traffic_lookup(name, (name,) + tuple(shape))
                assert nb >= 0 and isinstance(src, str)
                n += 1
    assert n > 0
    assert b.traffic_lookup("sgg::no_such_kernel", ("sgg::no_such_kernel", -1)) == (None, None)


def _family_state(graph, pooling="pool_net"):
    """A state dict of `graph`'s checkpoint family, built by an explicit-family
    model (the layout a reference checkpoint of that family holds)."""
    torch.manual_seed(3)
    return {k: v.clone() for k, v in _gen(graph, pooling).state_dict().items()}


def _reference_style_gen(pooling="pool_net", n_heads=1):
    """TrajectoryGenerator(**checkpoint args) exactly as the reference's
    scripts/evaluate_model.py:30-51 builds it: no family hint."""
    from sgan.models import TrajectoryGenerator
    return TrajectoryGenerator(obs_len=8, pred_len=12, embedding_dim=16, encoder_h_dim=32, decoder_h_dim=32,
                               mlp_dim=64, num_layers=1, noise_dim=(8,), noise_type="gaussian",
                               noise_mix_type="global", pooling_type=pooling, pool_every_timestep=False,
                               dropout=0.0, bottleneck_dim=8, neighborhood_size=2.0, grid_size=8, batch_norm=False,
                               n_units=[40, 16, 40], n_heads=n_heads, dropout1=0.0, alpha=0.2)


@pytest.mark.parametrize("graph,pooling", [("gat", "pool_net"), ("gcn", "pool_net"), ("sgangat", "pool_net"),
                                           ("vanilla", None), ("vanilla", "pool_net")])
def test_family_inferred_from_state_dict_on_strict_load(graph, pooling):
    """scripts/evaluate_model.py:30-52 (construct from the checkpoint args,
    then a strict load_state_dict of g_state) works for every checkpoint
    family without the `graph=` keyword: the family is read off the key set,
    the module set and its registration order are the family's (so the
    optimizer-state order matches), and every tensor is loaded."""
    from sgan.models import TrajectoryGenerator
    sd = _family_state(graph, pooling)
    assert TrajectoryGenerator.family_of(sd) == graph
    g = _reference_style_gen(pooling)
    g.load_state_dict(sd)                                      # strict
    assert g.graph == graph
    ref = _gen(graph, pooling)
    assert [k for k, _ in g.named_parameters()] == [k for k, _ in ref.named_parameters()]
    for k, v in g.state_dict().items():
        assert torch.equal(v, sd[k]), k


def test_family_switch_keeps_shared_modules_and_sgangat_shapes():
    """A gat -> gcn switch keeps gcn_module's parameter objects; the sgangat
    batched-GAT head / unit lists come from the state's tensor shapes (the
    checkpoint's `n_heads` argument is a plain int); a partial non-strict
    load without family keys keeps the family."""
    from sgan.models import TrajectoryGenerator
    g = _reference_style_gen()
    keep = g.gcn_module.gcn_intra.W[0]
    g.load_state_dict(_family_state("gcn"))
    assert g.graph == "gcn" and g.gcn_module.gcn_intra.W[0] is keep and hasattr(g, "mlp_decoder_context")
    assert not hasattr(g, "gatencoder")
    g = _reference_style_gen(n_heads=4)
    g.load_state_dict(_family_state("sgangat"))
    heads = [l.n_head for l in g.gatencoder.gat_net.layer_stack]
    assert g.graph == "sgangat" and heads == [4, 1]
    g.load_state_dict({"encoder.spatial_embedding.bias": torch.zeros(16)}, strict=False)
    assert g.graph == "sgangat"
    with pytest.raises(RuntimeError):                          # a genuine key mismatch still fails strictly
        bad = _family_state("gat")
        bad.pop("gatencoder.out_embedding.bias")
        _reference_style_gen().load_state_dict(bad)


def test_padded_sizes_fit_rules():
    """padded_sizes: exactly S_cap scenes / B_cap peds, real scenes first,
    padding scenes non-empty and within np_cap; None when it cannot fit."""
    from sgan.scene import padded_sizes
    rng = np.random.default_rng(0)
    for _ in range(200):
        S = int(rng.integers(1, 65))
        sizes = rng.integers(1, 58, size=S)
        S_cap, np_cap = 96, 64
        B_cap = int(-(-(sizes.sum() + S_cap - S) // 256) * 256)
        out = padded_sizes(sizes, S_cap, B_cap, np_cap)
        assert out is not None and len(out) == S_cap and out.sum() == B_cap
        assert np.array_equal(out[:S], sizes) and out[S:].min() >= 1 and out.max() <= np_cap
    assert padded_sizes([70], 8, 128, 64) is None           # a scene over np_cap
    assert padded_sizes([5] * 9, 8, 128, 64) is None        # too many scenes
    assert padded_sizes([5, 5], 8, 12, 64) is None          # fewer padding peds than padding scenes
    assert padded_sizes([5, 5], 2, 11, 64) is None          # padding peds but no padding scene
    assert list(padded_sizes([5, 5], 2, 10, 64)) == [5, 5]


def test_padded_scenes_pack_layout():
    """PaddedScenes.pack (host side, the layout one H2D copy moves): scene
    offsets, ped -> scene map, gather rows (-1 = padding), the repeat's
    offsets, and per pooling plan a chunk count + table of the fixed gpw that
    covers every (scene, row) of the padded batch exactly once."""
    from sgan import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libsgg.so not built")
    from sgan.scene import PaddedScenes
    rng = np.random.default_rng(1)
    ps = PaddedScenes(96, 1024, "cpu", np_cap=64, reps=(2,))
    sizes = np.minimum(rng.geometric(0.1, size=64), 57)
    sizes[:3] = (57, 40, 1)
    off_r = np.concatenate([[0], np.cumsum(sizes)])
    rows_r = rng.integers(0, 10000, size=int(off_r[-1])).astype(np.int32)
    ps.load(off_r, rows_r)
    for rep, bn in ((1, 8), (1, 48), (2, 48)):
        sub = ps if rep == 1 else ps.repeat(2)
        tab, grid, mr, gpw, cnt = sub.pool_plan(bn)
        assert tab.shape == (ps.pool_cap, 4) and int(cnt) == grid and mr == 64 and gpw in (1, 2, 4)
    for trial in range(3):
        sizes = np.minimum(rng.geometric(0.1, size=64 - trial * 10), 57)
        off_r = np.concatenate([[0], np.cumsum(sizes)])
        B_r = int(off_r[-1])
        assert B_r + 96 - len(sizes) <= 1024
        rows_r = rng.integers(0, 10000, size=B_r).astype(np.int32)
        ps.load(off_r, rows_r)
        buf = ps._dev.numpy()
        L = ps._lay
        off = buf[L["scene_off"]:L["scene_off"] + 97]
        assert buf[0] == B_r and off[-1] == 1024 and np.array_equal(off[:len(off_r)], off_r)
        assert np.array_equal(buf[L["rows"]:L["rows"] + B_r], rows_r) and (buf[L["rows"] + B_r:L["rows"] + 1024] == -1).all()
        ped = buf[L["ped_scene"]:L["ped_scene"] + 1024]
        assert np.array_equal(ped, np.repeat(np.arange(96), np.diff(off)))
        r2 = buf[L["rep2"]:L["rep2"] + 2 * 96 + 1]
        assert np.array_equal(r2, np.concatenate([off, off[1:] + 1024]))
        for k, (rep, bn, gpw, _) in enumerate(ps._plans):
            o = ps._plan_region(k)
            tab = buf[o + 4:o + 4 + 4 * ps.pool_cap].reshape(-1, 4)[:buf[o]]
            so = off if rep == 1 else r2
            seen = set()
            for s, i0, i1, g in tab:
                assert g == gpw
                for i in range(i0, i1):
                    assert (s, i) not in seen
                    seen.add((int(s), int(i)))
            assert len(seen) == int(so[-1])


def test_check_ownership_walks_closures_and_descriptors():
    """kernels.check_ownership (the launch timer's record-time check): every
    pointer inside a re-issuable launch's ctypes descriptors must lie in a
    tensor / storage the closure itself keeps alive -- found through closure
    cells, bound defaults, functools.partial, nested closures, arrays of
    descriptors and pointer arrays of nested structs."""
    import functools
    from sgan import _native as N
    from sgan import kernels as K
    a, b = torch.zeros(32), torch.zeros(16)
    job = N.L2Job(N.ptr(a), 3, N.ptr(b[4:]))          # a view: its storage counts
    K.check_ownership(lambda k=(a, b): job)
    K.check_ownership(functools.partial(lambda j, s: j, job, [a.untyped_storage(), b.untyped_storage()]))
    inner = lambda: (a, b)   # noqa: E731
    K.check_ownership(lambda: (inner(), job))          # nested closure holds them
    with pytest.raises(K.OwnershipError):
        K.check_ownership(lambda k=(a,): job, "l2")      # b only named by the descriptor
    arr = (N.L2Job * 2)(job, N.L2Job(N.ptr(a), 1, None))
    K.check_ownership(lambda: (arr, a, b))
    with pytest.raises(K.OwnershipError):
        K.check_ownership(lambda: (arr, a))
    ge = N.GatEncArgs()
    ge.w.Wi[1] = N.ptr(b).value
    with pytest.raises(K.OwnershipError):
        K.check_ownership(lambda: (ge, a))
    K.check_ownership(lambda: (ge, b))
    # an owned descriptor: its kept buffers ride on the instance
    job2 = N.L2Job(N.ptr(a), 1, N.ptr(b))
    job2._keep = (a, b)
    K.check_ownership(lambda: job2)


def test_loss_deferral_limit_is_per_kind():
    """The finish launch takes SGG_LOSSJOB_MAX jobs of EACH kind: a third BCE
    value is not queued even while the L2 list is empty (it would fail the
    launch's job check), and eager_losses() turns queueing off."""
    from sgan import _native as N
    from sgan import kernels as K
    K._DEFER[0] += 1
    saved = dict(K._LOSS)
    try:
        K._LOSS.update(l2=[], bce=[object()] * N.LOSSJOB_MAX, keep=[], out=set())
        assert not K._loss_deferrable("bce")
        assert K._loss_deferrable("l2")
        with K.eager_losses():
            assert not K._loss_deferrable("l2")
        assert K._loss_deferrable("l2")
    finally:
        K._DEFER[0] -= 1
        K._LOSS.clear()
        K._LOSS.update(saved)


def test_trainer_skips_deferred_finish_when_grads_are_observed():
    """A parameter hook (or retain_grad) reads gradients during the backward:
    the trainer's step scope then leaves the deferred finishes out."""
    from sgan.models import TrajectoryDiscriminator
    from sgan.train_step import GanTrainer, KernelOps

    class Ops(KernelOps):
        optimizer = staticmethod(lambda params, lr: torch.optim.Adam(params, lr=lr))
    g = _gen()
    d = TrajectoryDiscriminator(8, 12, embedding_dim=16, h_dim=48, mlp_dim=64, batch_norm=False, d_type="global")
    tr = GanTrainer(g, d, ops=Ops())
    assert not tr._grad_observed()
    h = next(iter(d.parameters())).register_hook(lambda gr: gr)
    assert tr._grad_observed()
    h.remove()
    assert not tr._grad_observed()


def test_bucketed_trainer_requires_a_padding_scene():
    from sgan.train_step import BucketedGraphTrainer

    class _T:
        class dp:
            on = False
            world = 1
    with pytest.raises(ValueError):
        BucketedGraphTrainer(_T(), None, batch_size=64, pad_scenes=0)
    assert BucketedGraphTrainer(_T(), None, batch_size=64, pad_scenes=1).S_cap == 65


def test_draw_source_orders_draws_across_trainers():
    """DrawSource (sgan/train_step.py): a look-ahead does not consume, the
    sequence number names the first pending draw, and take() after a
    look-ahead returns the draw made ahead (no second RNG draw)."""
    import itertools
    from sgan.train_step import DrawSource
    c = itertools.count()
    src = DrawSource(lambda: next(c))
    seq, items = src.ahead(3)
    assert (seq, items) == (0, [0, 1, 2])
    assert src.take() == 0            # the other trainer consumes the head
    seq, items = src.ahead(3)
    assert (seq, items) == (1, [1, 2, 3])
    src.pop(3)
    assert src.take() == 4 and src.seq == 5 and not src.pending


def test_pool_plan_targets_by_bottleneck(monkeypatch):
    """SceneIndex.pool_plan's chunk target (round 5): the generator's bn-8
    pooling of a configs[1] batch (64 scenes of 20) runs two pair groups per
    wave (256 chunks: one round of the fragment kernel), the discriminator's
    bn-48 pooling keeps the 512 target (its 128-scene D-step batch at two
    groups, its 64-scene G-step batch at one)."""
    from sgan import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libsgg.so not built")
    from sgan import scene
    from sgan.scene import SceneIndex
    # (the plan is host code of the C ABI: no device needed)
    real_load = _native.load
    monkeypatch.setattr(scene.N, "load", lambda require_gpu=True: real_load(require_gpu=False))
    for S, bn, want_gpw, want_nc in ((64, 8, 2, 256), (128, 48, 2, 512), (64, 48, 1, 448)):
        sc = SceneIndex(np.arange(0, 20 * S + 1, 20, dtype=np.int64), "cpu")
        _, nc, mr, gpw = sc.pool_plan(bn)[:4]
        assert (gpw, nc) == (want_gpw, want_nc), (S, bn, gpw, nc)
