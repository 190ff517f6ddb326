"""Fast GAN training iteration (reference scripts/train.py:395-484), with
scene-sharded data parallelism over RCCL.

Same maths and the same host RNG streams as the reference's
discriminator_step / generator_step:
  D-step: fake = G(batch) (1 noise draw), D on fake and real, gan_d_loss
          (2 random.uniform draws), backward, [clip], Adam.
  G-step: best_k G samples (best_k noise draws, in order), per-scene
          min_k sum_peds l2 / sum(mask) summed over scenes, + gan_g_loss on
          D(last sample) (1 random.uniform draw), backward, clip 2.0, Adam.

What differs is the execution plan, all results-neutral:
  * D on fake and real runs as ONE call over the two batches stacked.
  * The D-step's G forward runs without autograd: its gradients are
    discarded by the reference (optimizer_g.zero_grad() precedes the G
    backward, train.py:478).
  * The best_k G samples differ only in the noise appended after the graph
    module (models.py:909), so the encoder / pooling / GAT context runs ONCE
    per G-step, with autograd (G.context), and only the decoder rolls out
    the k samples (G.decode): one no-grad rollout over the k-times
    replicated context; the per-scene argmin picks each scene's best sample,
    and only that sample and the last one (the D input) are rolled out again
    with autograd.  The gradient of min_k and of the D term flows only
    through those two, so the gradients equal the reference's (every other
    sample's contribution is exactly zero).  `selective_backward=False`
    keeps all k rollouts in the graph.
  * The G-step's D forward backpropagates to G only (its D parameter
    gradients are discarded by the reference, train.py:397-427).
  * Loss values come back as device tensors (no per-step host sync).

Data parallelism (one process per GPU, torch.distributed, backend nccl=RCCL):
every rank holds S_local whole scenes of the global batch; all ranks draw the
GLOBAL noise tensors from identically seeded host generators and slice their
own rows, and draw the same label-smoothing numbers; local losses are scaled
so that the SUM over ranks is the global loss (the l2 term is a sum over
scenes, the BCE terms are means over the B_global peds); one flat bucket
all-reduce per optimizer step (grads + loss values), then clip and Adam.
The result equals single-GPU training on the global batch up to summation
order.
"""
import contextlib
import collections
import functools
import os
import random
import time

import numpy as np
import torch
import torch.distributed as dist

from . import kernels as K
from .models import get_noise
from .scene import SceneIndex


# step(): the G-step's generator context formed at the D-step beside the
# D-step's own (G.context_pair: one GATEncoder launch for both batches)
PAIR = os.environ.get("SGG_PAIR", "1") != "0"
# with PAIR: the D-step's generator decoder launched together with the
# G-step's best-of-k rollout (kernels.decoder_pair: one batch-MFMA launch)
DEC_PAIR = os.environ.get("SGG_DEC_PAIR", "1") != "0"


class TrainArgs:
    """scripts/train.py:29-124 defaults of the fields the steps read."""

    def __init__(self, **kw):
        self.obs_len = 8
        self.pred_len = 12
        self.best_k = 20
        self.l2_loss_weight = 1.0
        self.clipping_threshold_g = 2.0
        self.clipping_threshold_d = 0.0
        self.g_learning_rate = 1e-4
        self.d_learning_rate = 1e-3
        self.__dict__.update(kw)


def _sse_of(sc):
    return torch.from_numpy(np.stack([sc.host_off[:-1], sc.host_off[1:]], 1))


def _valid(sc):
    """The BCE's real-score count of a padded batch (PaddedScenes.nvalid)."""
    nv = getattr(sc, "nvalid", None)
    return {"nvalid": nv} if nv is not None else {}


class DataParallel:
    """Scene-sharded DP context (world 1 = plain single-GPU).

    transport: how the gradient all-reduce travels --
      "rccl"  ncclAllReduce on a communicator of sgan.rccl (one per process
              group, its id exchanged through the rendezvous store): eager,
              or captured inside GraphedTrainer's HIP graph (capture=True,
              the default for this transport: one graph per replay);
      "pg"    the process group's own all_reduce (gloo: host collectives,
              CPU tensors or ranks sharing one GPU) -- never captured: the
              graph is cut into segments with the all-reduces run eagerly
              between them.
    Default: "rccl" for a process group whose backend includes nccl, else
    "pg"; SGG_DP_TRANSPORT overrides it, SGG_CAPTURE_COLLECTIVE=0 forces the
    segment form.  No transport issues a collective of torch's
    ProcessGroupNCCL: its watchdog thread polls the events of the
    collectives it issued, and a poll that meets a capturing stream aborts
    the process (sgan/rccl.py).

    exercise: run the gradient all-reduce even at world size 1 (the DP code
    path on one GPU: an RCCL SUM over one rank is the identity, so the step
    must stay bitwise equal to the non-DP one)."""

    def __init__(self, group=None, exercise=False, capture=None, transport=None):
        self.on = dist.is_available() and dist.is_initialized()
        self.group = group
        self.world = dist.get_world_size(group) if self.on else 1
        self.rank = dist.get_rank(group) if self.on else 0
        self.exercise = bool(exercise) and self.on
        if transport is None:
            transport = os.environ.get("SGG_DP_TRANSPORT") or (
                "rccl" if self.on and "nccl" in str(dist.get_backend(group)) else "pg")
        if transport not in ("rccl", "pg"):
            raise ValueError("DataParallel: transport %r (rccl | pg)" % (transport,))
        self.transport = transport
        if capture is None:
            capture = transport == "rccl" and os.environ.get("SGG_CAPTURE_COLLECTIVE", "1") != "0"
        if capture and transport != "rccl":
            raise ValueError("DataParallel: only the rccl transport's all-reduce can be captured in a graph")
        self.capture = bool(capture) and self.on
        self.cut = None   # set by GraphedTrainer while capturing: graph segment boundary

    @property
    def rccl(self):
        """The RCCL communicator of the rccl transport (sgan.rccl.comm_for:
        made at the first use, one per process group), else None."""
        if self.transport != "rccl" or not self.collective:
            return None
        from .rccl import comm_for
        return comm_for(self.group)

    def prepare(self):
        """Make the communicator now (a collective point of every rank):
        before any graph capture, which must not create it."""
        self.rccl

    @property
    def collective(self):
        """Whether the steps issue gradient all-reduces at all."""
        return self.on and (self.world > 1 or self.exercise)

    @property
    def segmented(self):
        """Whether a captured iteration must be cut at each all-reduce."""
        return self.collective and not self.capture

    def shard(self, S_global):
        """Contiguous scene range [s0, s1) of this rank: a balanced split
        (floor + remainder: shard sizes differ by at most one scene).  Every
        rank must hold >= 1 scene (the kernels take no empty batch); the check
        depends only on (S_global, world), so every rank raises together,
        before any collective is entered."""
        if S_global < self.world:
            raise ValueError("scene-sharded DP needs >= %d scenes (one per rank), got %d: the reference loader "
                             "keeps a short last batch (loader.py:22-27); drop it or run it on fewer ranks"
                             % (self.world, S_global))
        per, rem = divmod(S_global, self.world)
        s0 = self.rank * per + min(self.rank, rem)
        return s0, s0 + per + (1 if self.rank < rem else 0)

    def allreduce_(self, tensors):
        """SUM-all-reduce a list of tensors through one flat bucket."""
        if not self.collective or not tensors:
            return
        if self.cut is not None:       # capturing: end the graph segment here
            self.cut(tensors)
            return
        flat = torch.cat([t.reshape(-1) for t in tensors])
        if self.transport == "rccl":
            self.rccl.allreduce_sum_(flat)
        else:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        # unpack with one multi-tensor copy (a copy per tensor would add ~45
        # launches per optimizer step)
        views = flat.split([t.numel() for t in tensors])
        torch._foreach_copy_(tensors, [v.view_as(t) for v, t in zip(views, tensors)])


class StepInputs:
    """Host-RNG draws of one iteration, in the reference's order, staged in
    device tensors: noise of the D-step's G call, the best_k noises of the
    G-step, and the three label-smoothing numbers (D real, D fake, G)."""

    def __init__(self, z_d, z_g, y):
        self.z_d, self.z_g, self.y = z_d, z_g, y


class KernelOps:
    """The step's glue and loss ops on the HIP kernels (kernels.py); the CPU
    data-parallel tests plug in a torch restatement of the same interface
    together with the oracle's models."""
    traj_cat = staticmethod(K.traj_cat)
    l2_select = staticmethod(K.l2_select)
    l2_loss = staticmethod(K.l2_loss)
    bce_pair = staticmethod(K.bce_pair)
    bce_pair_total = staticmethod(K.bce_pair_total)
    split2 = staticmethod(K.split2)
    prefold = staticmethod(K.prefold)
    one = staticmethod(lambda device: K.const(1.0, device))
    # clip_grad_norm_ + Adam in two launches (sgg_adam_step; torch's state
    # layout, capturable): optimizer(params, lr).step(max_norm)
    optimizer = staticmethod(lambda params, lr: K.ClipAdam(params, lr=lr))
    # the discriminator head forms the BCE gradient in its own backward
    # (kernels.BceLink) inside the steps only
    handoff = staticmethod(K.bce_handoff)
    # the backward ops' weight-gradient finishes queued and issued together
    # (two launches per backward pass instead of two per op)
    defer_finish = staticmethod(K.defer_grad_finish)
    # the discriminator encoder's observed steps run once, in the generator
    # encoder's launch (kernels.SharedPrefix)
    shared_prefix = staticmethod(K.shared_prefix)
    traj_ahead = staticmethod(K.traj_ahead)
    decoder_pair = staticmethod(K.decoder_pair)
    # loss ops inside this scope write their values at once (not queued for
    # the finish launch): for values read before the backward
    eager_losses = staticmethod(K.eager_losses)


class GanTrainer:
    def __init__(self, G, D, args=None, dp=None, selective_backward=True, capturable=False, bce_pair=None, ops=None):
        """ops: KernelOps-like (traj_cat, l2_select, l2_loss, bce_pair,
        optimizer); bce_pair(scores, split, y_a, y_b, w) overrides
        ops.bce_pair.  `capturable` is kept for API compatibility: the
        optimizer step is always graph-capturable."""
        self.G, self.D = G, D
        self.ops = ops or KernelOps()
        self._bce_override = bce_pair
        self.bce_pair = bce_pair or self.ops.bce_pair
        self.args = args or TrainArgs()
        self.dp = dp or DataParallel()
        self.selective_backward = selective_backward
        bn = [n for n, m in list(G.named_modules()) + list(D.named_modules()) if isinstance(m, torch.nn.BatchNorm1d)]
        if bn:
            # the execution plan (one stacked [fake | real] D call, the shared G
            # context, scene sharding) changes the batch a BatchNorm averages over
            raise NotImplementedError("GanTrainer: BatchNorm layers (%s) are not supported (train.py's batch_norm=0 "
                                      "default); drive the modules with the reference's own step functions" % bn[:3])
        # Adam over ALL of G's parameters, as train.py:238 builds it, so the
        # optimizer state (and its index order) matches reference checkpoints;
        # the unused graph module gets no gradient and Adam skips it
        self.g_params = list(G.parameters())
        self.d_params = list(D.parameters())
        self.opt_g = self.ops.optimizer(self.g_params, self.args.g_learning_rate)
        self.opt_d = self.ops.optimizer(self.d_params, self.args.d_learning_rate)

    # -- helpers -----------------------------------------------------------
    def _noise(self, S_global, s0, s1):
        G = self.G
        if not G.noise_dim:
            return None
        if G.noise_mix_type != "global":
            raise NotImplementedError("GanTrainer shards scenes; per-ped noise ('ped' mix) is not sharded yet")
        z = get_noise((S_global,) + tuple(G.noise_dim), G.noise_type)   # host RNG, global draw
        return z[s0:s1]

    def _finish(self, params, opt, loss_terms, clip):
        """all-reduce grads (+ loss values), clip, step."""
        K.side_join()   # the weight gradients of the side stream (normally joined at the end of backward)
        K.grad_flush()  # the backward ops' queued weight-gradient finishes (KernelOps.defer_finish)
        grads = [p.grad for p in params if p.grad is not None]
        if self.dp.collective:   # the loss values ride along with the gradients
            vals = torch.stack([t.detach().reshape(()) for t in loss_terms])
            self.dp.allreduce_(grads + [vals])
        else:                                  # one rank: no copy (callers index the values)
            vals = [t.detach().reshape(()) for t in loss_terms]
        opt.step(max_norm=clip)    # clip_grad_norm_(params, clip) when clip > 0, then Adam
        return vals

    # -- steps ---------------------------------------------------------------
    def _prefix(self, obs_rel, copies):
        """The discriminator encoder's observed steps run once, beside the
        generator's encoder (ops.shared_prefix; a no-op without it)."""
        sp = getattr(self.ops, "shared_prefix", None)
        if sp is None or getattr(self.D, "encoder", None) is None or os.environ.get("SGG_NO_SHARED_PREFIX"):
            return contextlib.nullcontext()
        return sp(self.D, obs_rel, self.args.obs_len + self.args.pred_len, copies)

    def _traj_ahead(self, head, T1, ncol, col0=0, b=None, pos0=None):
        """The discriminator input written by the next decoder launch
        (ops.traj_ahead; a no-op without it)."""
        ta = getattr(self.ops, "traj_ahead", None)
        if ta is None:
            return contextlib.nullcontext()
        return ta(head, T1, ncol, col0, b, pos0)

    def _scope(self):
        st = contextlib.ExitStack()
        st.enter_context(getattr(self.ops, "handoff", contextlib.nullcontext)())
        if not self._grad_observed():
            st.enter_context(getattr(self.ops, "defer_finish", contextlib.nullcontext)())
        return st

    def _grad_observed(self):
        """Does anything read a parameter gradient DURING the backward (a
        tensor hook, a post-accumulate hook, retain_grad)?  Deferred finishes
        (kernels.defer_grad_finish) write the weight gradients only at
        grad_flush(), before the optimizer: such a reader would see unwritten
        memory, so the step then lets every op finish its own gradients."""
        for p in self.g_params + self.d_params:
            if getattr(p, "_backward_hooks", None) or getattr(p, "_post_accumulate_grad_hooks", None) \
                    or p.retains_grad:
                return True
        return False

    def d_step(self, batch, sc, S_global=None, B_global=None, shard=(0, None), inputs=None, pair=None):
        """discriminator_step (train.py:395-429). `batch` holds this rank's
        scenes (device tensors), `sc` their SceneIndex.  `inputs` (StepInputs)
        replaces the host RNG draws by pre-drawn device tensors (graph mode).
        pair = (batch_g, sc_g): the next G-step's batch -- its generator
        context is formed here beside this step's (G.context_pair: G's weights
        do not change in between) together with its best-of-k rollout and
        argmin; returns (losses, prefix) for g_rest(prefix)."""
        with self._scope():
            return self._d_step(batch, sc, S_global, B_global, shard, inputs, pair)

    def _pairs(self, sc, sc_g):
        """step() forms the G-step's context at the D-step (d_step pair=)."""
        G = self.G
        return (PAIR and self.selective_backward and self.args.best_k > 1 and self.args.l2_loss_weight > 0
                and hasattr(G, "context_pair") and G.pair_ok(sc, sc_g))

    def _d_step(self, batch, sc, S_global, B_global, shard, inputs, pair=None):
        a = self.args
        G = self.G
        (obs, pred_gt, obs_rel, pred_gt_rel, _ov, _pv, obs_g, _pg, _nl, _lm, sse) = batch
        g_kw = (S_global, B_global)   # the G-step's own (None: its batch's sizes)
        S_global = S_global or sc.S
        B_global = B_global or sc.B
        s0 = shard[0]
        z = inputs.z_d if inputs is not None else self._noise(S_global, s0, s0 + sc.S)
        prefold = getattr(self.ops, "prefold", None)
        if prefold is not None and hasattr(G, "fold_specs") and hasattr(self.D, "fold_specs") \
                and G.num_layers == 1 and self.D.encoder.num_layers == 1:
            # G's folds (stale since the last G-step) and D's (since the last
            # D-step) in ONE launch; the forwards below find them cached
            prefold(G.fold_specs() + self.D.fold_specs())
        pre = None
        dpair = getattr(self.ops, "decoder_pair", None)
        dpair = dpair() if (pair is not None and DEC_PAIR and dpair is not None) else contextlib.nullcontext()
        with self._prefix(obs_rel, 2):
            with dpair:
                with self._traj_ahead(obs_rel, pred_gt_rel.shape[0], sc.B, 0, pred_gt_rel, obs[0]):
                    if pair is not None:
                        # this step's generator context (no autograd) and the G-step's
                        # (autograd) with one GATEncoder launch for both
                        bg, scg = pair
                        ctx_d, ctx_g = G.context_pair((obs, obs_rel, sse, obs_g, sc),
                                                      (bg[0], bg[2], bg[10], bg[6], scg))
                        with torch.no_grad():
                            fake_rel = G.decode(ctx_d, obs, obs_rel, sse, user_noise=z, scenes=sc)
                    else:
                        with torch.no_grad():
                            fake_rel = G(obs, obs_rel, sse, obs_g, user_noise=z, scenes=sc)
                    # D reads traj[0] (the start positions, models.py:989) and traj_rel
                    # only: [fake | real] side by side, no relative_to_abs needed (the
                    # decoder launch writes it: ops.traj_ahead)
                    traj_rel, start = self.ops.traj_cat(obs_rel, fake_rel, pred_gt_rel, obs[0])
                if pair is not None:
                    # the G-step's best-of-k rollout (its launch also runs this
                    # step's decoder, held since above: decoder_pair) and argmin
                    self._no_shared = True
                    try:
                        pre = self._g_prefix(bg, scg, g_kw[0], g_kw[1], shard, inputs, ctx=ctx_g)
                    finally:
                        self._no_shared = False
            sc2 = sc.repeat(2)
            scores = self.D(start, traj_rel, _sse_of(sc2), scenes=sc2)
        if inputs is not None:
            y_real = inputs.y[0]
        else:
            y_real = random.uniform(0.7, 1.2)
            random.uniform(0, 0.3)   # the fake-label draw (losses.py:47): consumed, but zeros_like * y == 0
        # gan_d_loss = bce(real, y_real) + bce(fake, 0); scores = [fake | real]
        loss = self.bce_pair(scores, sc.B, 0.0, y_real, sc.B / B_global, **_valid(sc))
        self.opt_d.zero_grad(set_to_none=True)
        torch.autograd.backward(loss, grad_tensors=self.ops.one(loss.device))
        vals = self._finish(self.d_params, self.opt_d, [loss], a.clipping_threshold_d)
        out = {"D_data_loss": vals[0], "D_total_loss": vals[0]}
        return out if pair is None else (out, pre)

    def g_step(self, batch, sc, S_global=None, B_global=None, shard=(0, None), inputs=None):
        """generator_step (train.py:432-484)."""
        with self._scope():
            return self._g_step(batch, sc, S_global, B_global, shard, inputs)

    def _g_step(self, batch, sc, S_global, B_global, shard, inputs):
        return self._g_rest(self._g_prefix(batch, sc, S_global, B_global, shard, inputs))

    def g_prefix(self, batch, sc, S_global=None, B_global=None, shard=(0, None), inputs=None, shared=False):
        """The part of generator_step that reads G's weights and the G batch
        only (train.py:441-455): the context (encoder, pooling, GAT, with
        autograd), the no-grad best-of-k rollout and the per-scene argmin.
        Nothing of the D-step before it changes its inputs, so it may run
        beside the D-step (GraphedTrainer(overlap=True)); g_rest(prefix)
        finishes the G-step after it.  shared=False: the discriminator's
        observed steps are NOT run in the generator encoder's launch (D's
        weights change in the D-step's Adam); the G-step's D forward then runs
        its whole encoder."""
        if shared:
            return self._g_prefix(batch, sc, S_global, B_global, shard, inputs)
        self._no_shared = True
        try:
            return self._g_prefix(batch, sc, S_global, B_global, shard, inputs)
        finally:
            self._no_shared = False

    def g_rest(self, pre):
        """The rest of generator_step after g_prefix: the two samples with
        autograd, the losses, D's frozen forward, backward, clip, Adam."""
        with self._scope():
            return self._g_rest(pre)

    def _g_prefix(self, batch, sc, S_global, B_global, shard, inputs, ctx=None):
        a = self.args
        G, ops = self.G, self.ops
        (obs, pred_gt, obs_rel, pred_gt_rel, _ov, _pv, obs_g, _pg, _nl, loss_mask, sse) = batch
        S_global = S_global or sc.S
        B_global = B_global or sc.B
        s0 = shard[0]
        S, B, k = sc.S, sc.B, a.best_k
        mask = loss_mask[:, a.obs_len:]                                   # (B, pred_len) view
        if inputs is not None:
            z_all = inputs.z_g                                            # (k, S, nz) on the device
        else:
            zs = [self._noise(S_global, s0, s0 + S) for _ in range(k)]    # k draws, reference order
            z_all = torch.stack(zs, 0) if zs[0] is not None else None
        use_l2 = a.l2_loss_weight > 0
        # the k samples differ only in the noise appended after the graph
        # module: the encoder / pooling / GAT context runs once (with autograd)
        # and only the decoder rolls out k times
        # (no shared prefix here: g_rest arms it for its decoder launch)
        pfx = None if getattr(self, "_no_shared", False) else self._prefix(obs_rel, 1)
        if pfx is not None:
            pfx.__enter__()
        try:
            if ctx is None:   # (else formed by the D-step: G.context_pair)
                ctx = G.context(obs, obs_rel, sse, obs_g, scenes=sc)
            best = None
            if self.selective_backward and k > 1 and use_l2:
                with torch.no_grad():
                    pred_all = G.decode(ctx.detach(), obs, obs_rel, sse, user_noise=z_all, scenes=sc, copies=k,
                                        noise_index=(None, 0))
                    best = ops.l2_select(pred_all, pred_gt_rel, mask, sc, k)   # (S,) int64
        except BaseException:
            if pfx is not None:
                pfx.__exit__(None, None, None)
            raise
        return dict(batch=batch, sc=sc, S_global=S_global, B_global=B_global, z_all=z_all, ctx=ctx, best=best,
                    pfx=pfx, mask=mask, inputs=inputs)

    def _g_rest(self, pre):
        a = self.args
        G, D, ops = self.G, self.D, self.ops
        batch, sc, B_global, z_all, ctx, pfx, mask, inputs = (pre[n] for n in (
            "batch", "sc", "B_global", "z_all", "ctx", "pfx", "mask", "inputs"))
        (obs, pred_gt, obs_rel, pred_gt_rel, _ov, _pv, obs_g, _pg, _nl, loss_mask, sse) = batch
        # the shared prefix stays armed until D's forward, and is disarmed on
        # any exception before it
        with contextlib.ExitStack() as stack:
            S, B, k = sc.S, sc.B, a.best_k
            use_l2 = a.l2_loss_weight > 0
            if pfx is None:
                # the context was formed without the discriminator's observed-steps
                # prefix (G.context_pair / g_prefix): it rides with the decoder
                # launch below (D's weights are final by now)
                stack.enter_context(self._prefix(obs_rel, 1))
            else:
                stack.push(pfx)   # (entered by _g_prefix)
            if self.selective_backward and k > 1:
                best = pre["best"]
                copies = 2 if use_l2 else 1
                # the last sample's columns become the discriminator input below
                tah = self._traj_ahead(obs_rel, a.pred_len, B, (copies - 1) * B)
                tah.__enter__()
                try:
                    out = G.decode(ctx, obs, obs_rel, sse, user_noise=z_all, scenes=sc, copies=copies,
                                   noise_index=(best, k - 1))
                except BaseException:
                    tah.__exit__(None, None, None)
                    raise
                if use_l2:
                    fake_rel_best, fake_rel_last = ops.split2(out, B)
                else:
                    fake_rel_best, fake_rel_last = None, out
            else:
                tah = contextlib.nullcontext()
                out = G.decode(ctx, obs, obs_rel, sse, user_noise=z_all, scenes=sc, copies=k, noise_index=(None, 0))
                fake_rel_last = out[:, (k - 1) * B:]
                fake_rel_best = None
                if use_l2:   # every sample in the graph: min over k of the per-scene terms
                    seg = sc.ped_scene_long()
                    m = mask.t().unsqueeze(2)
                    l2s = torch.stack([(m * (pred_gt_rel - out[:, i * B:(i + 1) * B]) ** 2).sum((0, 2))
                                       for i in range(k)], 0)                       # (k, B)
                    scene_l2 = torch.zeros(k, S, device=obs.device).index_add_(1, seg, l2s)
                    mask_sum = torch.zeros(S, device=obs.device).index_add_(0, seg, mask.sum(1))
            terms = []
            total = getattr(self.ops, "bce_pair_total", None)
            fused_total = use_l2 and total is not None and self._bce_override is None
            # without the one-launch total below, the loss values are read by an
            # eager add before the backward: they must not be queued (a queued L2
            # value is formed from terms its backward writes)
            eager = contextlib.nullcontext if fused_total else getattr(self.ops, "eager_losses", contextlib.nullcontext)
            if use_l2:
                if fake_rel_best is not None:
                    with eager():
                        g_l2 = ops.l2_loss(fake_rel_best, pred_gt_rel, mask, sc, a.l2_loss_weight)
                else:
                    g_l2 = (a.l2_loss_weight * scene_l2.min(0)[0] / mask_sum).sum()
                terms.append(g_l2)
            # the reference back-propagates into D's weights here and discards the
            # result (optimizer_d never sees it, train.py:478-482): freeze them for
            # this forward so D's backward produces input gradients only
            for p in self.d_params:
                p.requires_grad_(False)
            try:
                scores = D(obs[:1], ops.traj_cat(obs_rel, fake_rel_last), sse, scenes=sc)
            finally:
                tah.__exit__(None, None, None)
                stack.close()   # the prefix is spent once D has run
                for p in self.d_params:
                    p.requires_grad_(True)
            y = inputs.y[2] if inputs is not None else random.uniform(0.7, 1.2)
            if terms and fused_total:
                # gan_g_loss and the total loss with the L2 term from one launch
                adv, loss = total(scores, scores.shape[0], y, y, sc.B / B_global, terms[0], **_valid(sc))
            else:
                with eager():
                    adv = self.bce_pair(scores, scores.shape[0], y, y, sc.B / B_global, **_valid(sc))    # gan_g_loss
                loss = adv + (terms[0] if terms else 0.0)
            self.opt_g.zero_grad(set_to_none=True)
            torch.autograd.backward(loss, grad_tensors=self.ops.one(loss.device), inputs=self._g_inputs())
            vals = self._finish(self.g_params, self.opt_g, [terms[0] if terms else adv * 0, adv, loss],
                                a.clipping_threshold_g)
            out = {"G_discriminator_loss": vals[1], "G_total_loss": vals[2]}
            if use_l2:
                out["G_l2_loss_rel"] = vals[0]
            return out

    def _g_inputs(self):
        """G parameters on the forward's path (the family's unused graph
        module -- gcn_module under 'gat', mlp_decoder_context under 'gcn' /
        'sgangat' -- has no gradient and is left out of backward's inputs)."""
        if not hasattr(self, "_g_in"):
            graph = getattr(self.G, "graph", "gat")
            skip = {"gat": ("gcn_module.",), "gcn": ("gatencoder.", "mlp_decoder_context."),
                    "sgangat": ("mlp_decoder_context.",), "vanilla": ()}.get(graph, ())
            self._g_in = [p for n, p in self.G.named_parameters() if not n.startswith(skip)]
        return self._g_in

    def step(self, batch, sc, batch_g=None, sc_g=None, **kw):
        """One reference iteration (d_steps = g_steps = 1): the D-step on
        `batch`, the G-step on `batch_g` (default: the same batch).  The
        reference's loop feeds consecutive loader batches to the two steps
        (scripts/train.py:279-297); batch_g must have the same scene / ped
        counts when S_global / B_global are given."""
        bg, scg = (batch, sc) if batch_g is None else (batch_g, sc_g)
        if self._pairs(sc, scg):
            ld, pre = self.d_step(batch, sc, pair=(bg, scg), **kw)
            return ld, self.g_rest(pre)
        ld = self.d_step(batch, sc, **kw)
        lg = self.g_step(bg, scg, **kw)
        return ld, lg

    def step_split(self, batch, sc, batch_g=None, sc_g=None, **kw):
        """The same iteration in the order GraphedTrainer(overlap=True) issues
        it: g_prefix (the G-step's context, rollout and argmin -- G's weights
        and the G batch only), the D-step, then g_rest.  Needs pre-drawn host
        RNG numbers (kw['inputs'], StepInputs): the noise of the G-step is
        consumed before the D-step's, so the draws must already be in the
        reference's order."""
        if kw.get("inputs") is None and self.G.noise_dim:
            raise ValueError("step_split: pass inputs=StepInputs (draw_inputs) -- the G-step's noise is used first")
        pre = self.g_prefix(batch if batch_g is None else batch_g, sc if sc_g is None else sc_g, **kw)
        ld = self.d_step(batch, sc, **kw)
        lg = self.g_rest(pre)
        return ld, lg

    def draw_inputs(self, S_global, s0, s1):
        """The host draws one iteration makes, in the reference's order (torch
        RNG: D-step noise, then best_k G-step noises; Python random: D real,
        D fake, G label smoothing)."""
        z_d = self._noise(S_global, s0, s1)
        yr, yf = random.uniform(0.7, 1.2), random.uniform(0, 0.3)
        z_g = [self._noise(S_global, s0, s1) for _ in range(self.args.best_k)]
        yg = random.uniform(0.7, 1.2)
        zg = torch.stack(z_g, 0) if z_g[0] is not None else None
        return z_d, zg, torch.tensor([yr, yf, yg], dtype=torch.float32)


class DrawSource:
    """The host RNG draws of consecutive iterations, in order, with look-ahead.
    `ahead(n)` makes sure the next n iterations' draws exist (drawing them now
    if needed) and returns them with the sequence number of the first;
    `pop(n)` consumes them.  Trainers replaying the same training run share
    one source, so a draw made ahead by one (GraphedTrainer draw_ahead) is
    the draw the next iteration uses whichever trainer runs it: the host RNG
    streams are advanced exactly in the reference's iteration order."""

    def __init__(self, draw):
        self.draw = draw
        self.pending = collections.deque()
        self.seq = 0          # sequence number of pending[0]

    def ahead(self, n):
        while len(self.pending) < n:
            self.pending.append(self.draw())
        return self.seq, [self.pending[j] for j in range(n)]

    def pop(self, n):
        for _ in range(n):
            self.pending.popleft()
        self.seq += n

    def take(self):
        self.ahead(1)
        item = self.pending[0]
        self.pop(1)
        return item


class GraphedTrainer:
    """One full iteration (D-step + G-step, both Adam updates) captured once
    into a HIP graph and replayed; with several ranks, three graph segments
    with the two gradient all-reduces run eagerly between them.

    The batch lives in static device tensors (copy new data into
    `self.batch` between replays for real training); each replay first draws
    the host RNG numbers exactly as the eager step would (StepInputs) into
    pinned buffers and copies them to the device inputs of the graph.  The
    trainer must be built with capturable=True (Adam keeps its step on the
    device)."""

    def __init__(self, trainer, batch, sc, S_global=None, B_global=None, shard=(0, None), warmup=2, batch_g=None,
                 sc_g=None, draw=None, prologue=None, iters=1, overlap=False, draw_ahead=False, draws=None,
                 head=None):
        """draw: () -> (z_d, z_g, y) host tensors of the staging shapes (default:
        trainer.draw_inputs over this rank's span); draws: a DrawSource shared
        with other trainers of the same run (default: one over `draw`);
        prologue: launches captured
        ahead of the step (the padded real-data path's batch gathers);
        head: head(i) captured at the start of graph i of the pair, before the
        prologue -- copies from host staging buffers that the caller fills for
        graph i after stage_ready() (the padded path's scene structure).
        iters (one rank): iterations per graph -- a replay runs `iters`
        consecutive iterations on the same batches (their host draws made in
        order before it), so the per-replay graph launch is paid once per
        `iters` iterations; step() then advances `iters` iterations.
        overlap (one rank): each iteration as three graphs -- the G-step's
        prefix (GanTrainer.g_prefix: context, best-of-k rollout, argmin),
        the D-step, the rest of the G-step -- the first two replayed on two
        streams at once (the prefix depends on G's weights and the G batch
        only), the third after both.  Forked branches INSIDE one captured
        graph do not overlap on this runtime (profiles/r04_graph_fork_probe);
        separate graphs on separate streams do."""
        self.t = trainer
        self.ar_events = None   # time_allreduce()
        self.iters = iters = max(1, int(iters))
        self.overlap = overlap = bool(overlap) and not trainer.dp.collective
        self.prologue = prologue or (lambda: None)
        self.head = head
        self.batch, self.sc = batch, sc
        self.batch_g, self.sc_g = batch_g, sc_g
        if batch_g is not None:
            assert sc_g is not None and (sc_g.S, sc_g.B) == (sc.S, sc.B), "G-step batch must match the D-step's sizes"
        self.kw = dict(S_global=S_global or sc.S, B_global=B_global or sc.B, shard=shard)
        dev = batch[0].device
        s0 = shard[0]
        self.span = (self.kw["S_global"], s0, s0 + sc.S)
        # (no closure over self anywhere in this object: a GraphedTrainer must
        # never sit in a reference cycle, see kernels.capture_guard)
        self.draws = draws if draws is not None else DrawSource(
            draw or functools.partial(trainer.draw_inputs, *self.span))
        self.draw = self.draws.take
        G = trainer.G
        nd = tuple(G.noise_dim) if G.noise_dim else None
        k = trainer.args.best_k
        # the step's host RNG numbers [z_d | z_g | y] in ONE flat buffer (one
        # H2D copy per replay); two pinned staging copies, alternated, each
        # guarded by an event so the host never overwrites a buffer whose
        # copy is still pending
        shp = [(sc.S,) + (nd or ()), (k, sc.S) + (nd or ()), (3,)] if nd else [(3,)]
        sizes = [int(np.prod(x)) for x in shp]
        per = sum(sizes)   # floats per iteration; iteration j's block at j * per
        views = lambda flat: [flat[o:o + n].view(x) for o, n, x in zip(np.cumsum([0] + sizes[:-1]), sizes, shp)]
        blocks = lambda flat: [views(flat[j * per:(j + 1) * per]) for j in range(iters)]
        self.stage_flat = [torch.empty(iters * per).pin_memory() for _ in range(2)]
        self.stage = [[tuple(v) if nd else (None, None, v[0]) for v in blocks(f)] for f in self.stage_flat]
        self.stage_ev = [None, None]
        self.cur = 0
        # draw_ahead (one rank): the host draws of the next replay are made
        # right after this replay is queued (taken ahead from the DrawSource,
        # so the sequence is unchanged), and a replay never waits for the
        # host RNG.  A trainer sharing the source that runs an iteration in
        # between consumes the first of those draws; the staged buffer is then
        # refilled at the next replay.  Off by default: code that draws from
        # the host RNG OUTSIDE the source between steps would see the state
        # one replay ahead
        self.draw_ahead = draw_ahead
        self.staged = [None, None]   # DrawSource sequence number each staging buffer holds
        self.inp_flat = torch.zeros(iters * per, device=dev)
        self.inps = [StepInputs(v[0], v[1], v[2]) if nd else StepInputs(None, None, v[0]) for v in blocks(self.inp_flat)]
        self.inp = self.inps[0]
        if iters > 1 and trainer.dp.segmented:
            raise ValueError("GraphedTrainer: iters > 1 needs the collectives inside the graph (DataParallel "
                             "capture=True: nccl) or one rank -- segmented collectives cut the graph")
        # warm-up and capture on the same side stream: the parameters'
        # AccumulateGrad nodes (created by the first backward, kept alive by
        # the captured graph) are bound to the stream that created them.  A
        # stream of our own, outside torch's pool (kernels.private_stream):
        # never a process group's stream
        cap = K.private_stream("capture")
        trainer.dp.prepare()   # the RCCL communicator (if any) exists before the capture
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            for _ in range(warmup):
                self._load(*self.draw())
                self.prologue()
                (trainer.step_split if overlap else trainer.step)(batch, sc, batch_g, sc_g, inputs=self.inp,
                                                                   **self.kw)
        torch.cuda.current_stream().wait_stream(cap)
        torch.cuda.synchronize()
        trainer.opt_g.zero_grad(set_to_none=True)
        trainer.opt_d.zero_grad(set_to_none=True)
        # One graph per replay when the collectives (if any) are captured with
        # it (one rank, or RCCL: DataParallel.capture).  Otherwise (gloo) the
        # capture is cut at each gradient all-reduce (DataParallel.cut): the
        # collectives run eagerly between graph segments on the segments'
        # static buffers (gloo cannot be captured; a failed capture would
        # poison the stream).
        self.segments = []
        self.pair = []
        dp = trainer.dp
        params = trainer.g_params + trainer.d_params
        cap.wait_stream(torch.cuda.current_stream())
        if not dp.segmented:
            # TWO graphs, each starting with the H2D copy of its own
            # pinned staging buffer, replayed alternately -- the next replay is
            # queued behind the running one with no host copy between them,
            # and the host fills buffer i while graph i's previous replay
            # (two steps back) is known to be done.  Each graph has its own
            # memory pool: its outputs (the losses, every p.grad) can then
            # never share memory with the other graph's temporaries, so they
            # stay intact while the other graph replays.
            if overlap:
                self._capture_overlap(cap, params)
                return
            for i in range(2):
                K.clear_fold_cache()   # every fold the replays need must be a node of this graph
                with torch.cuda.stream(cap), K.capture_guard():
                    g = torch.cuda.CUDAGraph()
                    g.capture_begin(pool=torch.cuda.graph_pool_handle(), capture_error_mode=K.capture_error_mode())
                    self.inp_flat.copy_(self.stage_flat[i], non_blocking=True)
                    if head is not None:
                        head(i)
                    for j in range(iters):
                        self.prologue()
                        losses = trainer.step(batch, sc, batch_g, sc_g, inputs=self.inps[j], **self.kw)
                    g.capture_end()
                self.pair.append((g, losses, [(p, p.grad) for p in params]))
            torch.cuda.current_stream().wait_stream(cap)
            torch.cuda.synchronize()
            K.clear_fold_cache()
            self.done_ev = [None, None]
            self.losses = self.pair[1][1]
            return
        if head is not None:
            raise ValueError("GraphedTrainer: head copies need the one-graph pair (no segmented collectives)")
        K.clear_fold_cache()   # every fold the replays need must be a node of the graph
        pool = torch.cuda.graph_pool_handle()   # the segments replay in capture order: one shared pool
        with torch.cuda.stream(cap), K.capture_guard():
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=pool, capture_error_mode=K.capture_error_mode())

            def cut(tensors):
                nonlocal g
                g.capture_end()
                self.segments.append((g, list(tensors)))
                g = torch.cuda.CUDAGraph()
                g.capture_begin(pool=pool, capture_error_mode=K.capture_error_mode())
            dp.cut = cut if dp.segmented else None
            try:
                self.prologue()
                self.losses = trainer.step(batch, sc, batch_g, sc_g, inputs=self.inp, **self.kw)
            finally:
                dp.cut = None
            g.capture_end()
            self.segments.append((g, None))
        torch.cuda.current_stream().wait_stream(cap)
        torch.cuda.synchronize()
        K.clear_fold_cache()

    def _capture_overlap(self, cap, params):
        """The two alternating graph sets of the overlapped plan: per set a
        head graph (the H2D copy of its staging buffer, the prologue) and per
        iteration the prefix / D-step / rest graphs.  Pools: the prefix graphs
        get their own (they replay beside the D-step, so nothing of theirs
        may share memory with it), the head, D-step and rest graphs share one
        (they replay in capture order on one stream).  The fold cache is
        emptied before each prefix and D-step capture: each computes the
        folds it reads itself, so no graph reads a fold another graph wrote
        on the other stream."""
        t = self.t
        bg, scg = (self.batch, self.sc) if self.batch_g is None else (self.batch_g, self.sc_g)
        self.side = K.private_stream("overlap")
        for i in range(2):
            pool_b, pool_a = torch.cuda.graph_pool_handle(), torch.cuda.graph_pool_handle()
            parts = []
            with torch.cuda.stream(cap), K.capture_guard():
                head = torch.cuda.CUDAGraph()
                head.capture_begin(pool=pool_a, capture_error_mode=K.capture_error_mode())
                self.inp_flat.copy_(self.stage_flat[i], non_blocking=True)
                if self.head is not None:
                    self.head(i)
                self.prologue()
                head.capture_end()
                for j in range(self.iters):
                    K.clear_fold_cache()
                    gb = torch.cuda.CUDAGraph()
                    gb.capture_begin(pool=pool_b, capture_error_mode=K.capture_error_mode())
                    pre = t.g_prefix(bg, scg, inputs=self.inps[j], **self.kw)
                    gb.capture_end()
                    K.clear_fold_cache()
                    ga = torch.cuda.CUDAGraph()
                    ga.capture_begin(pool=pool_a, capture_error_mode=K.capture_error_mode())
                    ld = t.d_step(self.batch, self.sc, inputs=self.inps[j], **self.kw)
                    ga.capture_end()
                    gc = torch.cuda.CUDAGraph()
                    gc.capture_begin(pool=pool_a, capture_error_mode=K.capture_error_mode())
                    lg = t.g_rest(pre)
                    gc.capture_end()
                    del pre
                    parts.append((gb, ga, gc))
            self.pair.append(((head, parts), (ld, lg), [(p, p.grad) for p in params]))
        torch.cuda.current_stream().wait_stream(cap)
        torch.cuda.synchronize()
        K.clear_fold_cache()
        self.done_ev = [None, None]
        self.losses = self.pair[1][1]

    def _replay_overlap(self, head, parts):
        main = torch.cuda.current_stream()
        head.replay()
        for gb, ga, gc in parts:
            self.side.wait_stream(main)      # G's weights of the previous G-step, the inputs
            with torch.cuda.stream(self.side):
                gb.replay()
            ga.replay()
            main.wait_stream(self.side)
            gc.replay()

    def stage_ready(self):
        """Index i of the graph the next step() replays, once graph i's previous
        replay (which read the staging buffers of its head copies) is done:
        the caller may then fill those buffers (head)."""
        i = self.cur
        if self.done_ev[i] is not None:
            self.done_ev[i].synchronize()
        return i

    def _load(self, z_d, z_g, y):
        i = self.cur
        self.cur ^= 1
        if self.stage_ev[i] is not None:
            self.stage_ev[i].synchronize()        # that set's previous copies are done
        h_zd, h_zg, h_y = self.stage[i][0]
        if z_d is not None:
            h_zd.copy_(z_d)
        if z_g is not None:
            h_zg.copy_(z_g)
        h_y.copy_(y)
        self.inp_flat.copy_(self.stage_flat[i], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.stage_ev[i] = ev

    def _fill(self, i):
        """The host draws of graph i's next replay (the next `iters` draws of
        the source, in order) into its staging buffer, once graph i's previous
        replay (which read that buffer) is done; nothing if it holds them."""
        seq, items = self.draws.ahead(self.iters)
        if self.staged[i] == seq:
            return
        if self.done_ev[i] is not None:
            self.done_ev[i].synchronize()
        for j, (z_d, z_g, y) in enumerate(items):
            h_zd, h_zg, h_y = self.stage[i][j]
            if z_d is not None:
                h_zd.copy_(z_d)
            if z_g is not None:
                h_zg.copy_(z_g)
            h_y.copy_(y)
        self.staged[i] = seq

    def step(self):
        """Draw this iteration's host RNG numbers, replay the graph; returns the
        (device) loss dicts of the captured step."""
        if self.pair:
            i = self.cur
            self.cur ^= 1
            self._fill(i)
            self.draws.pop(self.iters)
            g, self.losses, grads = self.pair[i]
            if self.overlap:
                self._replay_overlap(*g)
            else:
                g.replay()
            ev = torch.cuda.Event()
            ev.record()
            self.done_ev[i] = ev
            self.staged[i] = None
            if self.draw_ahead:   # the next replay's draws while this one runs
                self._fill(i ^ 1)
            self._after_replay(grads)
            return self.losses
        self._load(*self.draw())
        for g, tensors in self.segments:
            g.replay()
            if tensors is not None:
                if self.ar_events is not None:   # HIP events around the collective (bench.py)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    self.t.dp.allreduce_(tensors)
                    e1.record()
                    self.ar_events.append((e0, e1))
                else:
                    self.t.dp.allreduce_(tensors)
        self._after_replay(None)
        return self.losses

    def time_allreduce(self, on=True):
        """Record HIP events around every gradient all-reduce of the following
        replays (several ranks); allreduce_ms() sums them."""
        self.ar_events = [] if on else None

    def allreduce_ms(self):
        """Device time of the recorded all-reduces (ms, summed); synchronises."""
        if not self.ar_events:
            return 0.0
        self.ar_events[-1][1].synchronize()
        return sum(a.elapsed_time(b) for a, b in self.ar_events)

    @staticmethod
    def _after_replay(grads):
        """Leave eager code a consistent view: every p.grad is the gradient
        the replayed graph consumed (with two graphs, the other graph's
        tensors would be one step old), and the fold cache is dropped -- the
        replay updated the weights in place without moving their version
        counters, so a cached fold would be stale for an eager forward."""
        if grads is not None:
            for p, gr in grads:
                p.grad = gr
        K.clear_fold_cache()


def shard_batch(batch, sc, s0, s1):
    """Rows of scenes [s0, s1) of a global batch + their re-based SceneIndex."""
    p0, p1 = int(sc.host_off[s0]), int(sc.host_off[s1])
    (obs, pred, obs_rel, pred_rel, ov, pv, obs_g, pg, nl, lm, sse) = batch
    t = lambda x: x[:, p0:p1]
    off = sc.host_off[s0:s1 + 1] - p0
    local = SceneIndex(off, sc.device)
    sse_l = _sse_of(local)
    return (t(obs), t(pred), t(obs_rel), t(pred_rel), t(ov), t(pv), t(obs_g), t(pg), nl[p0:p1], lm[p0:p1],
            sse_l), local


class BucketedGraphTrainer:
    """HIP-graph replayed training on REAL batches.  The reference's loader
    yields batches of varying scene and ped counts (scripts/train.py:279-297:
    the D-step takes one loader batch, the G-step the next), which one
    captured graph cannot take.  Here each iteration's two batches are padded
    into a capacity bucket -- S_cap = batch_size + pad_scenes scenes and B_cap
    peds, a multiple of `gran` (sgan.scene.PaddedScenes: padding scenes of
    zero-mask peds that the losses leave out) -- whose iteration was captured
    once (GraphedTrainer over fixed-address buffers, the batch gathers from
    the device-resident split included).  A replay then needs two packed
    host-to-device copies (the batches' scene structure) and the host RNG
    draws, exactly the eager step's (noise of the real scenes only).

    A bucket is (B_cap, np_cap): np_cap, the largest scene it holds, is the
    smallest of `np_caps` that fits both batches (the kernels size their LDS
    plans by it; the one-launch GAT encoder takes scenes of up to 64 peds --
    its backward past 49 on the compact LDS plan).

    Capturing a new bucket runs GraphedTrainer's warm-up iterations; the
    parameters, the optimizer state and the host RNG states are saved before
    and restored after, so training is unchanged by a capture.  A batch that
    fits no bucket (a scene over max(np_caps) peds) runs eagerly."""

    def __init__(self, trainer, ddset, batch_size=64, pad_scenes=32, gran=256, np_caps=(48, 64), pool_cap=None):
        if trainer.dp.on and trainer.dp.world > 1:
            raise NotImplementedError("BucketedGraphTrainer: one rank (the padded batches are not sharded)")
        self.t, self.dd = trainer, ddset
        if pad_scenes < 1:
            # a full batch (S == batch_size) still needs one padding scene to
            # absorb the bucket's spare peds (padded_sizes): without it every
            # such iteration would silently run eagerly
            raise ValueError("BucketedGraphTrainer: pad_scenes must be >= 1 (got %d)" % pad_scenes)
        self.S_cap = batch_size + pad_scenes
        self.gran, self.np_caps, self.pool_cap = gran, tuple(sorted(np_caps)), pool_cap
        self.buckets = {}
        self.eager_steps = 0
        # (diagnostics: the last step's bucket and its replays before it, or
        # (None, "eager") for a batch pair no bucket holds; the last step's
        # host time in ms per phase: batch layout + bucket choice, the two
        # scene-structure uploads, the draws + graph replay)
        self.last = None
        self.phase_ms = None
        # replays in flight across buckets: before staging a batch the host
        # waits for the replay `depth` steps back, so it runs at most that far
        # ahead of the device.  (Each bucket's graph pair alone would let it
        # run ahead by two replays PER BUCKET and then wait for all of them
        # at once: multi-millisecond host iterations that are the queue
        # draining, not work.)
        self.depth = 2
        self._inflight = collections.deque()

    def bucket_of(self, off_d, off_g):
        """(B_cap, np_cap) of the bucket holding both batches, or None."""
        need, big = 0, 0
        for off in (off_d, off_g):
            S, B = len(off) - 1, int(off[-1])
            if S > self.S_cap or S == 0:
                return None
            big = max(big, int(np.diff(off).max()))
            need = max(need, B + max(self.S_cap - S, 1))
        caps = [c for c in self.np_caps if c >= big]
        if not caps:
            return None
        B_cap = -(-need // self.gran) * self.gran
        from .scene import padded_sizes
        for off in (off_d, off_g):
            if padded_sizes(np.diff(off), self.S_cap, B_cap, caps[0]) is None:
                return None
        return B_cap, caps[0]

    def step(self, scenes_d, scenes_g):
        """One reference iteration: the D-step on the split's scenes scenes_d,
        the G-step on scenes_g (the two consecutive loader batches)."""
        t0 = time.perf_counter()
        off_d, rows_d = self.dd.layout(scenes_d)
        off_g, rows_g = self.dd.layout(scenes_g)
        key = self.bucket_of(off_d, off_g)
        self.phase_ms = None
        if key is None:
            self.eager_steps += 1
            self.last = (None, "eager")
            bd, scd = self.dd.batch(scenes_d)
            bg, scg = self.dd.batch(scenes_g)
            return self.t.step(bd, scd, bg, scg)
        ent = self.buckets.get(key)
        if ent is None:
            ent = self.buckets[key] = self._capture(key, off_d, rows_d, off_g, rows_g)
            ent["replays"] = 0
        self.last = (key, ent["replays"])
        ent["replays"] += 1
        t1 = time.perf_counter()
        # the scene structure into the staging buffers of the graph replayed
        # next: its head copies them (no host-issued copy per batch)
        while len(self._inflight) >= self.depth:
            self._inflight.popleft().synchronize()
        i = ent["gt"].stage_ready()
        ent["sc_d"].load(off_d, rows_d, graph_stage=i)
        ent["sc_g"].load(off_g, rows_g, graph_stage=i)
        ent["state"]["S_real"] = (len(off_d) - 1, len(off_g) - 1)
        t2 = time.perf_counter()
        out = ent["gt"].step()
        self._inflight.append(ent["gt"].done_ev[i])
        t3 = time.perf_counter()
        self.phase_ms = ((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3)
        return out

    @staticmethod
    def _draw(t, S_cap, state):
        """The host RNG draws of one iteration in the reference's order
        (StepInputs; TrainArgs.draw_inputs with the two batches' own scene
        counts), zero-padded to S_cap rows.  (A static function over the
        trainer and the bucket's state, not a closure over the bucket: the
        bucket holds the GraphedTrainer holding this draw.)"""
        S_d, S_g = state["S_real"]

        def pad(z):
            if z is None:
                return None
            out = torch.zeros((S_cap,) + tuple(z.shape[1:]), dtype=z.dtype)
            out[:z.shape[0]] = z
            return out
        z_d = pad(t._noise(S_d, 0, S_d))
        yr, yf = random.uniform(0.7, 1.2), random.uniform(0, 0.3)
        z_g = [pad(t._noise(S_g, 0, S_g)) for _ in range(t.args.best_k)]
        yg = random.uniform(0.7, 1.2)
        return z_d, (torch.stack(z_g, 0) if z_g[0] is not None else None), torch.tensor([yr, yf, yg])

    def _state(self):
        ts = [p.data for p in self.t.g_params + self.t.d_params]
        for opt in (self.t.opt_g, self.t.opt_d):
            for p in opt.params:
                st = opt.opt.state.get(p)
                if st:
                    ts += [st["step"], st["exp_avg"], st["exp_avg_sq"]]
        return ts

    def _capture(self, key, off_d, rows_d, off_g, rows_g):
        from .scene import PaddedScenes
        B_cap, np_cap = key
        lib = N_lib()
        dev = self.dd.device
        dd = self.dd
        To, Tp = dd.obs_len, dd.pred_len
        ent = {"state": {"S_real": (len(off_d) - 1, len(off_g) - 1)}}
        ent["sc_d"] = PaddedScenes(self.S_cap, B_cap, dev, np_cap, reps=(2,), pool_cap=self.pool_cap)
        ent["sc_g"] = PaddedScenes(self.S_cap, B_cap, dev, np_cap, reps=(), pool_cap=self.pool_cap)
        ent["sc_d"].load(off_d, rows_d)
        ent["sc_g"].load(off_g, rows_g)
        nf = int(lib.sgg_gather_batch_floats(B_cap, To, Tp))
        bufs = [torch.empty(nf, device=dev, dtype=torch.float32) for _ in range(2)]
        batches = [dd.views(b, B_cap, sc.host_off) for b, sc in zip(bufs, (ent["sc_d"], ent["sc_g"]))]

        def prologue(bufs=bufs, scs=(ent["sc_d"], ent["sc_g"])):   # (no reference to ent: no cycle)
            for b, sc in zip(bufs, scs):
                dd.gather_into(sc.rows, B_cap, b)

        def head(i, scs=(ent["sc_d"], ent["sc_g"])):
            for sc in scs:
                sc.head_copy(i)
        # the warm-up iterations must leave no trace: parameters, optimizer
        # state (created here where missing: zeros == torch Adam's fresh
        # state) and the host RNG streams are restored afterwards
        before = {t.data_ptr(): t.clone() for t in self._state()}
        rng = (torch.get_rng_state(), random.getstate())
        try:
            gt = GraphedTrainer(self.t, batches[0], ent["sc_d"], warmup=2, batch_g=batches[1], sc_g=ent["sc_g"],
                                draw=functools.partial(self._draw, self.t, self.S_cap, ent["state"]),
                                prologue=prologue, head=head)
        finally:
            with torch.no_grad():
                for t in self._state():
                    t.copy_(before[t.data_ptr()]) if t.data_ptr() in before else t.zero_()
            torch.set_rng_state(rng[0])
            random.setstate(rng[1])
            K.clear_fold_cache()
        torch.cuda.synchronize()
        ent.update(gt=gt, bufs=bufs, batches=batches)
        return ent


def N_lib():
    from . import _native
    return _native.load()
