"""Buffer lifetimes of the re-issuable launches and of captured HIP graphs
(the round-3 hipErrorIllegalAddress in LaunchTimer
replay and the ~CUDAGraph abort inside a capture), and loss values read
before the backward (GanTrainer with a custom bce_pair)."""
import gc
import random

import pytest
import torch

from test_gpu_parity import DEV, build_models

pytestmark = pytest.mark.gpu


def _batches():
    from sgan.data.synthetic import synthetic_batch
    from sgan.scene import SceneIndex
    b = synthetic_batch([20, 7, 13, 20, 2, 20], seed=21, device=DEV)
    bg = synthetic_batch([20, 7, 13, 20, 2, 20], seed=22, device=DEV)
    return b, SceneIndex.from_seq_start_end(b[-1], DEV), bg, SceneIndex.from_seq_start_end(bg[-1], DEV)


def test_timer_records_own_their_buffers_after_outputs_dropped():
    """Record a training step under the launch timer (every record passes
    check_ownership), drop every output of the step and the step's own
    tensors, collect garbage, then re-issue every recorded launch: no fault,
    and the same per-launch table as a replay before the drop."""
    from sgan import kernels as K
    from sgan.train_step import GanTrainer
    g, d = build_models()
    tr = GanTrainer(g, d, capturable=True)
    b, sc, bg, scg = _batches()
    torch.manual_seed(5)
    random.seed(5)
    tr.step(b, sc, bg, scg)   # warm (folds, optimizer state)
    K.timer.start()
    out = tr.step(b, sc, bg, scg)
    recs = K.timer.stop()
    assert len(recs) >= 20, len(recs)
    before = K.timer.replay(recs, reps=2)
    del out, b, bg, sc, scg
    for p in tr.g_params + tr.d_params:
        p.grad = None
    gc.collect()
    # allocate and fill fresh memory: a freed buffer a record still pointed to
    # would now hold these values (or be unmapped)
    junk = [torch.full((1 << 20,), float("nan"), device=DEV) for _ in range(16)]
    after = K.timer.replay(recs, reps=2)
    torch.cuda.synchronize()
    del junk
    assert sorted(before) == sorted(after)
    for k in before:
        assert before[k]["launches"] == after[k]["launches"], k


def test_check_ownership_rejects_an_unowned_descriptor_pointer():
    """A closure whose descriptor names a buffer it does not hold is refused
    at record time (the timer raises before storing it)."""
    from sgan import _native as N
    from sgan import kernels as K
    held = torch.empty(64, device=DEV)
    loose = torch.empty(64, device=DEV)
    desc = N.L2Job(N.ptr(held), 1, N.ptr(loose))
    with pytest.raises(K.OwnershipError):
        K.check_ownership(lambda h=held: desc, "l2")
    K.check_ownership(lambda h=(held, loose): desc, "l2")


def test_gc_inside_capture_after_a_dropped_trainer():
    """A GraphedTrainer that is dropped leaves no CUDAGraph in a reference
    cycle: a garbage collection INSIDE the next trainer's capture (its
    prologue runs there) destroys nothing, and the new graph replays."""
    from sgan.train_step import GanTrainer, GraphedTrainer
    g, d = build_models()
    tr = GanTrainer(g, d, capturable=True)
    b, sc, bg, scg = _batches()
    torch.manual_seed(6)
    random.seed(6)
    gt = GraphedTrainer(tr, b, sc, warmup=1, batch_g=bg, sc_g=scg)
    gt.step()
    torch.cuda.synchronize()
    del gt
    calls = []

    def prologue():
        if torch.cuda.is_current_stream_capturing():
            gc.collect()   # would run ~CUDAGraph of a cyclic-garbage graph here
            calls.append(1)
    gt2 = GraphedTrainer(tr, b, sc, warmup=1, batch_g=bg, sc_g=scg, prologue=prologue)
    for _ in range(3):
        ld, lg = gt2.step()
    torch.cuda.synchronize()
    assert calls, "the prologue never ran inside a capture"
    assert all(torch.isfinite(v).all() for v in list(ld.values()) + list(lg.values()))


def test_custom_bce_pair_total_loss_equals_default():
    """GanTrainer(bce_pair=...) takes the eager add of the loss values; the L2
    value it reads must be written before the add (not queued for the
    finish launch): G_total_loss equals the default one-launch path."""
    from sgan import kernels as K
    from sgan.train_step import GanTrainer
    res = []
    for custom in (False, True):
        g, d = build_models()
        tr = GanTrainer(g, d, capturable=True, bce_pair=K.bce_pair if custom else None)
        b, sc, bg, scg = _batches()
        torch.manual_seed(7)
        random.seed(7)
        for _ in range(2):
            ld, lg = tr.step(b, sc, bg, scg)
        torch.cuda.synchronize()
        res.append({k: float(v) for k, v in list(ld.items()) + list(lg.items())})
    a, c = res
    assert sorted(a) == sorted(c)
    for k in a:
        assert abs(a[k] - c[k]) <= 1e-5 * max(1.0, abs(a[k])), (k, a[k], c[k])
    assert abs(c["G_total_loss"] - (c["G_l2_loss_rel"] + c["G_discriminator_loss"])) <= 1e-5 * abs(c["G_total_loss"])


def test_decoder_init_rejects_mismatched_shapes_before_launch(monkeypatch):
    """The round-4 fault: the eager real-data pairing
    handed the G batch (more scenes) the D batch's noise, and the decoder's
    prologue read z[k][s] past its scene count.  decoder_init checks noise,
    context rows and last_rel against the scenes on the host: ValueError,
    and no launch is attempted (the library is unreachable in this test)."""
    from sgan import kernels as K
    from sgan.scene import SceneIndex
    sc = SceneIndex([0, 3, 7], DEV)                      # S = 2 scenes, B = 7 peds
    ctx = torch.randn(7, 24, device=DEV)
    last = torch.randn(7, 2, device=DEV)
    z_ok = torch.randn(1, 2, 8, device=DEV)

    def no_launch():
        raise AssertionError("decoder_init reached the library with bad shapes")
    monkeypatch.setattr(K, "_lib", no_launch)
    bad = [
        (ctx, torch.randn(1, 3, 8, device=DEV), None, last),      # noise of a batch with more scenes
        (ctx, torch.randn(1, 1, 8, device=DEV), None, last),      # ... and with fewer
        (ctx, torch.randn(2, 8, device=DEV), None, last),         # noise not (K, S, nz)
        (torch.randn(9, 24, device=DEV), z_ok, None, last),       # context rows of another batch
        (ctx, z_ok, None, torch.randn(9, 2, device=DEV)),         # last_rel rows of another batch
        (ctx, z_ok, torch.zeros(3, dtype=torch.int64, device=DEV), last),   # best of another batch
    ]
    for i, (c, z, best, lr) in enumerate(bad):
        with pytest.raises(ValueError, match="decoder_init"):
            K.decoder_init(c, z, best, 0, 1, sc, lr)
    with pytest.raises(ValueError, match="decoder_init"):     # fewer draws than the copies need
        K.decoder_init(ctx, z_ok, None, 0, 3, sc, last)


def test_dropped_graphed_trainer_in_a_cycle_is_reclaimed():
    """capture_guard leaves no process-wide trace (it used to
    gc.freeze() every live object after each capture, so cyclic garbage
    among them was never collected): a GraphedTrainer captured, then dropped
    while sitting in a reference cycle, is reclaimed by gc.collect(); and
    gc_frozen() unfreezes what it froze."""
    import weakref
    from sgan import kernels as K
    from sgan.train_step import GanTrainer, GraphedTrainer
    g, d = build_models()
    tr = GanTrainer(g, d, capturable=True)
    b, sc, bg, scg = _batches()
    torch.manual_seed(3)
    random.seed(3)
    gt = GraphedTrainer(tr, b, sc, warmup=1, batch_g=bg, sc_g=scg)
    gt.step()
    torch.cuda.synchronize()
    assert gc.get_freeze_count() == 0

    class Holder:
        pass
    h = Holder()
    h.me, h.gt = h, gt                      # a cycle holding the trainer
    ref = weakref.ref(gt)
    del gt, h
    gc.collect()
    assert ref() is None, "GraphedTrainer in a dropped cycle was not collected"
    with K.gc_frozen():
        assert gc.get_freeze_count() > 0
    assert gc.get_freeze_count() == 0
