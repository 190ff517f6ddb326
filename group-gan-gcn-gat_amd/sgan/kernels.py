"""Autograd wrappers around the libsgg.so C ABI (include/sgg.h).

Every op launches on torch's current stream through ctypes; forward and
backward are hand-written HIP kernels, the parameter-gradient reductions over
all nodes (X^T dY, column sums) included (sgg_xtw, xtw.hip).  No op has a CPU
path.
"""
import contextlib
import functools
import os
import weakref

import torch

from . import _native as N

# the one-launch GATEncoder (sgg_gatenc_*); "0" forces the per-layer kernels
GATENC_FUSED = os.environ.get("SGG_GATENC_FUSED", "1") != "0"
# the fused GATEncoder forward keeps its layer state for the backward (0: the backward recomputes it)
GATENC_SAVE = os.environ.get("SGG_GATENC_SAVE", "1") != "0"
# the pooling backward's dh = dU W1h and h^T dU partials in one launch
# (sgg_pool_dh_dw); "0": two launches (sgg_xw + sgg_xtw_partial)
DUAL_POOL_BWD = os.environ.get("SGG_DUAL_POOL_BWD", "1") != "0"
# weight-gradient reductions of the backward on a side stream (needed only by
# the optimizer step, which joins it).  Off by default: measured slower at
# configs[1] (61.1k vs 68.9k scenes/s graph-replayed, 12.4k vs 14.8k eager
# real data) -- the cross-stream edges cost more than the overlap wins
SIDE_STREAM = os.environ.get("SGG_SIDE_STREAM", "0") == "1"


# SGG_DEBUG=1: host-side consistency checks that cost a device read
DEBUG = os.environ.get("SGG_DEBUG", "0") == "1"


def _lib():
    return N.load()


def _req(t, name, dtype=torch.float32):
    if not t.is_cuda:
        raise N.NativeError("%s must be a device tensor (no CPU path)" % name)
    if t.dtype != dtype:
        raise N.NativeError("%s must be %s, got %s" % (name, dtype, t.dtype))
    return t


def _rows(t, name):
    """2-D with unit column stride (row stride is passed as leading dim)."""
    _req(t, name)
    if t.dim() != 2 or t.stride(1) != 1:
        t = t.contiguous()
    return t


# ---------------------------------------------------------------------------
# precision of the node transforms
# ---------------------------------------------------------------------------
_PRECISION = os.environ.get("SGG_PRECISION", "fp32")


def set_precision(p):
    """'fp32' (default; exact f32 MFMA, the parity path) or 'bf16': every
    forward dense node transform X W (sgg_xw: the GAT / GCN XW, Linear
    layers, the pooling's h W1h) runs on bf16 MFMA with fp32 accumulation
    (BASELINE configs 3 and 5: "bf16 + MFMA XW"); the backward's input
    gradients, LSTMs, attention, pooling pairs and weight-gradient
    reductions stay fp32 (bf16 input gradients through the sgangat instance
    norms lose the encoder's gradient: tests/test_gpu_configs.py)."""
    global _PRECISION
    if p not in ("fp32", "bf16"):
        raise ValueError("precision must be 'fp32' or 'bf16'")
    _PRECISION = p


def precision():
    return _PRECISION


# ---------------------------------------------------------------------------
# dense node transform
# ---------------------------------------------------------------------------
_private = {}   # (tag, device index) -> torch.cuda.ExternalStream
_hiprt = None


def private_stream(tag, device=None):
    """A HIP stream of this package's own as a torch.cuda.ExternalStream --
    hipStreamCreateWithFlags(hipStreamNonBlocking) through the HIP runtime
    torch loaded, one per (tag, device), kept for the process.  It lies
    outside torch's stream pool (32 pooled streams handed out round-robin),
    so it can never be the stream of a torch.distributed process group or of
    other torch code: the graph captures (GraphedTrainer, tag "capture"), the
    weight-gradient side stream ("side"), the overlap plan's second stream
    ("overlap") and the launch timer ("timer") run on such streams."""
    global _hiprt
    import ctypes
    dev = torch.cuda.current_device() if device is None else torch.device(device).index
    if dev is None:
        dev = torch.cuda.current_device()
    key = (tag, dev)
    st = _private.get(key)
    if st is None:
        if _hiprt is None:
            lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
            lib.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            lib.hipStreamCreateWithFlags.restype = ctypes.c_int
            _hiprt = lib
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            rc = _hiprt.hipStreamCreateWithFlags(ctypes.byref(h), 1)   # hipStreamNonBlocking
        if rc != 0 or not h.value:
            raise N.NativeError("hipStreamCreateWithFlags failed (%d)" % rc)
        st = _private[key] = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", dev))
    return st


class _Side:
    stream = None
    origin = None   # the stream that must wait for the side work
    keep = []
    active = False


@contextlib.contextmanager
def side(*keep):
    """Run the block's launches on the weight-gradient side stream: it first
    waits for everything issued so far on the current stream; the tensors in
    `keep` (read by the block, allocated on the current stream) stay alive
    until side_join().  Off (SGG_SIDE_STREAM=0): the block runs in line."""
    if not SIDE_STREAM:
        yield
        return
    cur = torch.cuda.current_stream()
    if _Side.stream is None or _Side.stream.device != cur.device:
        _Side.stream = private_stream("side", cur.device)
    st = _Side.stream
    st.wait_stream(cur)
    _Side.keep.extend(t for t in keep if t is not None)
    if not _Side.active:
        _Side.active = True
        _Side.origin = cur
        try:   # inside a backward pass: join when it ends (any optimizer, e.g. torch.optim.Adam, then sees .grad)
            torch.autograd.Variable._execution_engine.queue_callback(side_join)
        except RuntimeError:
            pass    # outside backward: the caller joins
    with torch.cuda.stream(st):
        yield


def side_join():
    """The stream the side work was forked from waits for it (end of the
    backward pass, or explicitly before reading .grad); no-op when idle."""
    if _Side.active:
        _Side.origin.wait_stream(_Side.stream)
        _Side.keep.clear()
        _Side.active = False
        _Side.origin = None


def xw_raw(x, w, bias=None, trans_w=False, act=0, out=None, mask=None, prec=None):
    """act(x @ W + bias); W = w (K x N) or w^T (w stored N x K, trans_w).  w
    may be a row-strided column block (e.g. W1[:, E:]), passed in place.
    mask (same shape as x): x counts only where mask > 0 (fused ReLU backward).
    prec: None = the global precision (set_precision) -- the forward
    transforms; 'fp32' forces exact f32 (the backward's input gradients)."""
    x = _rows(x, "x")
    if mask is not None:
        mask = _rows(mask, "mask")
        assert mask.shape == x.shape
    w = _rows(w, "w")
    M, K = x.shape
    Nn = w.shape[0] if trans_w else w.shape[1]
    assert (w.shape[1] if trans_w else w.shape[0]) == K, (x.shape, w.shape, trans_w)
    if bias is not None:
        bias = _req(bias, "bias").contiguous()
        assert bias.numel() == Nn
    y = out if out is not None else torch.empty(M, Nn, device=x.device, dtype=torch.float32)

    bf16 = (prec or _PRECISION) == "bf16"
    fn = _lib().sgg_xw_bf16 if bf16 else _lib().sgg_xw

    def launch():
        N.check(fn(N.ptr(x), x.stride(0), N.ptr(mask), mask.stride(0) if mask is not None else 0,
                   N.ptr(w), w.stride(0), int(bool(trans_w)), N.ptr(bias), N.ptr(y), y.stride(0), M, K, Nn,
                   int(act), N.stream_ptr()), "sgg_xw")
    launch()
    if timer.active and M > 0:
        tw = "true" if trans_w else "false"
        name = ("sgg::xw_bf16_kernel<%s>" % tw if bf16 else
                "sgg::xw_splitk_kernel<%s>" % tw if K >= 256 else
                "sgg::xw_kernel<true, true>" if trans_w and K <= 256 else
                "sgg::xw_kernel<%s, false>" % tw)
        timer.add(name, (M, K, Nn, mask is not None), 2.0 * M * K * Nn,
                  4.0 * (M * K * (2 if mask is not None else 1) + K * Nn + M * Nn), launch)
    return y


def xtw(X, Y, colsum=False, trans_c=False, out=None, mask=None):
    """C = X^T Y (M x N), or C^T (N x M) with trans_c, plus the column sums of
    Y, with the split-K MFMA reduction (sgg_xtw).  X: R x M, Y: R x N,
    row-strided 2-D views allowed; `out` (row-strided, unit column stride)
    receives C in place."""
    lib = _lib()
    X = _rows(X, "X")
    Y = _rows(Y, "Y")
    if mask is not None:
        mask = _rows(mask, "mask")
        assert mask.shape == Y.shape
    R, M = X.shape
    Nn = Y.shape[1]
    assert Y.shape[0] == R
    shape = (Nn, M) if trans_c else (M, Nn)
    if out is None:
        C = torch.empty(shape, device=X.device, dtype=torch.float32)
    else:
        assert tuple(out.shape) == shape and out.stride(1) == 1, (out.shape, shape)
        C = out
    if R == 0:
        C.zero_()
        return (C, torch.zeros(Nn, device=X.device)) if colsum else C
    splits = lib.sgg_xtw_splits(R, M, Nn)
    ws = torch.empty(splits * (M * Nn + Nn), device=X.device, dtype=torch.float32)
    cs = torch.empty(Nn, device=X.device, dtype=torch.float32) if colsum else None
    def launch():
        N.check(lib.sgg_xtw(N.ptr(X), X.stride(0), N.ptr(Y), Y.stride(0), N.ptr(mask),
                            mask.stride(0) if mask is not None else 0, R, M, Nn, N.ptr(C), C.stride(0), int(trans_c),
                            N.ptr(cs), N.ptr(ws), ws.numel() * 4, N.stream_ptr()), "sgg_xtw")
    launch()
    if timer.active:
        timer.add("sgg::xtw_partial_kernel+xtw_reduce_kernel", (R, M, Nn, mask is not None), 2.0 * R * M * Nn,
                  4.0 * (R * M + R * Nn * (2 if mask is not None else 1) + M * Nn) + 8.0 * ws.numel(), launch)
    return (C, cs) if colsum else C


# ---------------------------------------------------------------------------
# input-embedding fold (sgg_fold_fwd / sgg_fold_bwd)
# ---------------------------------------------------------------------------
def fold_fwd(W, We, be, b1, b2=None):
    """A = W We (R x 2), bias = W be + b1 (+ b2); W may be a column block.
    Cached: the fold depends on weights only, so it is recomputed only after
    they change (torch's version counter, or an epoch ClipAdam bumps when it
    updates parameters through raw pointers) -- see prefold()."""
    key, ver = _fold_key(W, We, be, b1, b2)
    ent = _FOLD_CACHE.get(key)
    if _fold_hit(ent, ver, (W, We, be, b1, b2)):
        return ent[1], ent[2]
    prefold([(W, We, be, b1, b2)])
    ent = _FOLD_CACHE[key]
    return ent[1], ent[2]


# parameter data_ptr -> epoch, bumped by ClipAdam for every tensor it updates
# in place (its raw-pointer update does not move torch's version counter)
_EPOCH = {}
_FOLD_CACHE = {}


def _fold_key(W, We, be, b1, b2):
    ts = (W, We, be, b1, b2)
    key = tuple((t.data_ptr(), tuple(t.shape), t.stride(0)) if t is not None else None for t in ts)
    ver = tuple((t._version, _EPOCH.get(t.data_ptr(), 0)) if t is not None else None for t in ts)
    return key, ver


def _owner(t):
    return t._base if t._base is not None else t


def _fold_hit(ent, ver, ts):
    """A cached fold is current iff the weights' versions match AND the
    entry was made from these very weight tensors (weak references): a
    tensor that reuses a freed weight's address is a different tensor."""
    return (ent is not None and ent[0] == ver
            and all((r is None) if t is None else (r is not None and r() is _owner(t)) for r, t in zip(ent[4], ts)))


def _fold_purge():
    """Drop entries whose weights are gone (models built and discarded in one
    process: tests, sweeps, evaluating many checkpoints)."""
    dead = [k for k, e in _FOLD_CACHE.items() if any(r is not None and r() is None for r in e[4])]
    for k in dead:
        del _FOLD_CACHE[k]


def clear_fold_cache():
    """Drop every cached fold (a HIP-graph capture must start from an empty
    cache, so every fold its replays need is a node of the graph)."""
    _FOLD_CACHE.clear()


def prefold(specs):
    """Make sure the folds of `specs` [(W, We, be, b1, b2), ...] are cached and
    current, computing all missing / stale ones in ONE launch
    (sgg_fold_fwd_multi).  Called once per module set per forward (the
    generator's encoder + pooling + decoder, the discriminator's encoder +
    pooling), so a training iteration runs three fold launches instead of one
    per layer call."""
    todo = []
    for W, We, be, b1, b2 in specs:
        key, ver = _fold_key(W, We, be, b1, b2)
        if not _fold_hit(_FOLD_CACHE.get(key), ver, (W, We, be, b1, b2)):
            todo.append((key, ver, (W, We, be, b1, b2)))
    if not todo:
        return
    _fold_purge()
    arr = (N.Fold * len(todo))()
    outs = []
    for k, (key, ver, (W, We, be, b1, b2)) in enumerate(todo):
        W = _rows(W, "W")
        R, E = W.shape
        A = torch.empty(R, 2, device=W.device, dtype=torch.float32)
        bias = torch.empty(R, device=W.device, dtype=torch.float32)
        parts = (W, We.contiguous(), be.contiguous(), b1.contiguous(), b2.contiguous() if b2 is not None else None)
        arr[k] = N.Fold(N.ptr(parts[0]), W.stride(0), R, E, N.ptr(parts[1]), N.ptr(parts[2]), N.ptr(parts[3]),
                        N.ptr(parts[4]), N.ptr(A), N.ptr(bias))
        outs.append((key, ver, A, bias, parts))
    for i in range(0, len(todo), N.FOLD_MAX):
        chunk = (N.Fold * min(N.FOLD_MAX, len(todo) - i))(*arr[i:i + N.FOLD_MAX])
        N.check(_lib().sgg_fold_fwd_multi(chunk, len(chunk), N.stream_ptr()), "sgg_fold_fwd_multi")
    for (key, ver, A, bias, parts), (_, _, ts) in zip(outs, todo):
        # weak references to the caller's weights (the entry does not keep a
        # model alive); strong ones only to the contiguous copies made here
        refs = tuple(weakref.ref(_owner(t)) if t is not None else None for t in ts)
        copies = tuple(p for p, t in zip(parts, ts) if p is not None and p.data_ptr() != t.data_ptr())
        _FOLD_CACHE[key] = (ver, A, bias, copies, refs)


def lstm_fold_spec(lstm, emb):
    return (lstm.weight_ih_l0, emb.weight, emb.bias, lstm.bias_ih_l0, lstm.bias_hh_l0)


def pool_fold_spec(pool):
    l1, E = pool.mlp_pre_pool[0], pool.embedding_dim
    return (l1.weight[:, :E], pool.spatial_embedding.weight, pool.spatial_embedding.bias, l1.bias, None)


def fold_bwd(W, We, be, dA, dbias, dW=None, dbias_copy=None):
    """(dW, dWe, dbe) of fold_fwd; dW may be a preallocated column block;
    dbias_copy (optional) receives a copy of dbias in the same launch."""
    W = _rows(W, "W")
    R, E = W.shape
    dW = dW if dW is not None else torch.empty(R, E, device=W.device, dtype=torch.float32)
    dWe = torch.empty(E, 2, device=W.device, dtype=torch.float32)
    dbe = torch.empty(E, device=W.device, dtype=torch.float32)
    N.check(_lib().sgg_fold_bwd(N.ptr(W), W.stride(0), R, E, N.ptr(We.contiguous()), N.ptr(be.contiguous()),
                                N.ptr(dA.contiguous()), N.ptr(dbias.contiguous()), N.ptr(dW), dW.stride(0), N.ptr(dWe),
                                N.ptr(dbe), N.ptr(dbias_copy), N.stream_ptr()), "sgg_fold_bwd")
    return dW, dWe, dbe


# ---------------------------------------------------------------------------
# weight-gradient finish: a backward op's slab row sums + fold backwards in
# ONE launch (sgg_grad_finish)
# ---------------------------------------------------------------------------
def xtw_partial(X, Y, colsum=False):
    """sgg_xtw's split pass alone; returns (ws, splits): C's partials are the
    first splits x (M N) floats of ws, the column-sum partials the next
    splits x N.  The sums join a GradFinish."""
    lib = _lib()
    X = _rows(X, "X")
    Y = _rows(Y, "Y")
    R, M = X.shape
    Nn = Y.shape[1]
    assert Y.shape[0] == R and R > 0
    splits = lib.sgg_xtw_splits(R, M, Nn)
    ws = torch.empty(splits * (M * Nn + (Nn if colsum else 0)), device=X.device, dtype=torch.float32)

    def launch():
        N.check(lib.sgg_xtw_partial(N.ptr(X), X.stride(0), N.ptr(Y), Y.stride(0), None, 0, R, M, Nn, int(colsum),
                                    N.ptr(ws), ws.numel() * 4, N.stream_ptr()), "sgg_xtw_partial")
    launch()
    if timer.active:
        mt = 4 if M >= 64 else (M + 15) // 16
        timer.add("sgg::xtw_partial_kernel<%d>" % mt, (R, M, Nn), 2.0 * R * M * Nn,
                  4.0 * (R * M + R * Nn) + 4.0 * ws.numel(), launch)
    return ws, splits


class GradFinish:
    """Collects the row-sum jobs (SggRed) and fold backwards (SggFoldBwd) of
    one backward op and runs them through sgg_grad_finish: one launch for
    every row sum, one for the folds.  Inside defer_grad_finish() (the
    trainer's steps) run() only queues the jobs: grad_flush() issues the
    queued jobs of the whole backward pass together.  Results are
    bit-identical to sgg_slab_reduce / sgg_xtw / sgg_fold_bwd in turn."""

    def __init__(self):
        self.reds, self.folds, self.keep = [], [], []

    def _hold(self, *ts):
        """Keep the jobs' buffers alive until the launch -- by their STORAGE:
        a queued reference to an output tensor itself would raise its use
        count, and autograd's AccumulateGrad would then copy the (not yet
        written) gradient into .grad instead of taking the tensor."""
        self.keep += [t.untyped_storage() for t in ts if t is not None]

    def rowsum(self, src, rows, ld, col0, cols, out):
        """out[c] = sum over src's rows of src[:, col0 + c] (out contiguous)."""
        assert out.is_contiguous() and out.numel() == cols
        self.reds.append(N.Red(N.ptr(src), rows, ld, col0, cols, N.ptr(out), 0, 0, 0, 0))
        self._hold(src, out)

    def xtw_sums(self, ws, splits, M, Nn, C, trans_c=False, colsum=None):
        """C (M x Nn, or its transpose; row-strided view) and optionally the
        column sums from xtw_partial's workspace."""
        assert C.stride(1) == 1 and tuple(C.shape) == ((Nn, M) if trans_c else (M, Nn))
        self.reds.append(N.Red(N.ptr(ws), splits, M * Nn, 0, M * Nn, N.ptr(C), 1, Nn, C.stride(0), int(trans_c)))
        self._hold(ws, C)
        if colsum is not None:
            self.rowsum(ws[splits * M * Nn:], splits, Nn, 0, Nn, colsum)

    def fold(self, W, We, be, dA_src, dA_rows, dA_ld, dA_col0, db_src, db_rows, db_ld, db_col0, dW=None,
             dbias_copy=None):
        """fold_bwd with (dA, dbias) given as slab column row sums; returns
        (dW, dWe, dbe)."""
        W = _rows(W, "W")
        R, E = W.shape
        dW = dW if dW is not None else torch.empty(R, E, device=W.device, dtype=torch.float32)
        dWe = torch.empty(E, 2, device=W.device, dtype=torch.float32)
        dbe = torch.empty(E, device=W.device, dtype=torch.float32)
        We, be = We.contiguous(), be.contiguous()
        self.folds.append(N.FoldBwd(N.ptr(W), W.stride(0), R, E, N.ptr(We), N.ptr(be),
                                    N.ptr(dA_src), dA_rows, dA_ld, dA_col0, N.ptr(db_src), db_rows, db_ld, db_col0,
                                    N.ptr(dW), dW.stride(0), N.ptr(dWe), N.ptr(dbe), N.ptr(dbias_copy)))
        self._hold(W, We, be, dA_src, db_src, dW, dWe, dbe, dbias_copy)
        return dW, dWe, dbe

    def run(self):
        if not self.reds and not self.folds:
            return
        if _DEFER[0] > 0:
            _PENDING.append(self)
            return
        _finish_launch(self.reds, self.folds, self.keep)


_DEFER = [0]
_PENDING = []
# loss VALUES queued inside defer_grad_finish() (SggL2Job / SggBceJob): the
# training step only reports them, so they are formed in the flush's row-sum
# launch (one extra workgroup) instead of launches of their own
_LOSS = {"l2": [], "bce": [], "keep": [], "out": set()}


DEFER_LOSSES = os.environ.get("SGG_DEFER_LOSSES", "1") != "0"


def _loss_deferrable(kind):
    """May one more loss value of `kind` ("l2" / "bce") be queued?  The finish
    launch takes at most SGG_LOSSJOB_MAX jobs of EACH kind; past that the op
    forms its value in a launch of its own."""
    return DEFER_LOSSES and _DEFER[0] > 0 and not _NO_DEFER[0] and len(_LOSS[kind]) < N.LOSSJOB_MAX


@contextlib.contextmanager
def eager_losses():
    """Scope in which no loss value is queued: every loss op writes its value
    at once.  For callers that read a loss value before the backward (an
    eager add of two values): a queued value is formed only after the
    backward (the L2 value from the per-scene terms its backward writes)."""
    prev = _NO_DEFER[0]
    _NO_DEFER[0] = True
    try:
        yield
    finally:
        _NO_DEFER[0] = prev


_NO_DEFER = [False]


def _queue_loss(kind, job, keep, outs):
    _LOSS[kind].append(job)
    _LOSS["keep"] += [t.untyped_storage() for t in keep if t is not None]
    _LOSS["out"].update(t.data_ptr() for t in outs)


def _loss_pending(t):
    """Is t a queued (not yet written) loss value?"""
    return t is not None and t.data_ptr() in _LOSS["out"]


def _take_losses():
    l2, bce, keep = _LOSS["l2"], _LOSS["bce"], _LOSS["keep"]
    _LOSS.update(l2=[], bce=[], keep=[], out=set())
    return l2, bce, keep


def flush_losses():
    """Form the queued loss values now (their own one-workgroup launch)."""
    l2, bce, keep = _take_losses()
    if l2 or bce:
        _finish_launch([], [], keep, l2, bce)


@contextlib.contextmanager
def defer_grad_finish():
    """Scope in which the backward ops queue their weight-gradient finishes
    (GradFinish) instead of launching them; grad_flush() -- the trainer's,
    before the optimizer reads the gradients -- issues all of them in two
    launches (every row sum, every fold backward) where the ops would issue
    two each.  Leaving the scope flushes whatever is still queued.

    Invariant: inside the scope, the gradient tensors a backward op returns
    (views of its slab sums, dW / dWe / dbe) are NOT written until
    grad_flush().  Nothing may read them before that: not autograd's
    InputBuffer summing two contributions to one parameter (no parameter of
    the models feeds two ops), not a tensor / post-accumulate hook,
    retain_grad or an all-reduce hook during the backward.  GanTrainer leaves
    the scope out when a parameter has such a reader (_grad_observed); with
    SGG_CHECK_DEFER=1 every op flushes right after its backward (the deferred
    == immediate comparison of tests/test_gpu_parity.py runs both)."""
    if os.environ.get("SGG_CHECK_DEFER") == "1":
        yield
        return
    _DEFER[0] += 1
    try:
        yield
    finally:
        _DEFER[0] -= 1
        if _DEFER[0] == 0:
            grad_flush()


def grad_flush():
    """Issue every queued GradFinish (in queue order, as few sgg_grad_finish
    calls as the job limits allow); the queued loss values ride in the last
    one."""
    if not _PENDING:
        flush_losses()
    while _PENDING:
        reds, folds, keep = [], [], []
        while _PENDING and len(reds) + len(_PENDING[0].reds) <= N.RED_MAX \
                and len(folds) + len(_PENDING[0].folds) <= N.FOLDB_MAX:
            gf = _PENDING.pop(0)
            reds += gf.reds
            folds += gf.folds
            keep += gf.keep
        if not reds and not folds:   # one op alone over the limits: cannot happen (each op is within them)
            raise N.NativeError("grad_flush: a queued finish exceeds the job limits")
        l2, bce = [], []
        if not _PENDING:
            l2, bce, lkeep = _take_losses()
            keep = keep + lkeep
        _finish_launch(reds, folds, keep, l2, bce)


def _finish_launch(reds_l, folds_l, keep, l2_l=(), bce_l=()):
    lib = _lib()
    assert len(reds_l) <= N.RED_MAX and len(folds_l) <= N.FOLDB_MAX
    assert len(l2_l) <= N.LOSSJOB_MAX and len(bce_l) <= N.LOSSJOB_MAX
    reds = (N.Red * max(1, len(reds_l)))(*reds_l)
    folds = (N.FoldBwd * max(1, len(folds_l)))(*folds_l)
    l2 = (N.L2Job * max(1, len(l2_l)))(*l2_l)
    bce = (N.BceJob * max(1, len(bce_l)))(*bce_l)
    nr, nf, nl, nb = len(reds_l), len(folds_l), len(l2_l), len(bce_l)
    dev = keep[0].device
    scratch = torch.empty(max(1, sum(3 * f.R for f in folds_l)), device=dev, dtype=torch.float32)

    def launch(reds=reds, folds=folds, nr=nr, nf=nf, l2=l2, bce=bce, nl=nl, nb=nb, keep=list(keep)):
        N.check(lib.sgg_grad_finish_losses(reds, nr, folds, nf, N.ptr(scratch), scratch.numel() * 4, l2, nl, bce, nb,
                                           N.stream_ptr()), "sgg_grad_finish")
    launch()
    if timer.active:
        nb = sum(4.0 * r.rows * r.cols for r in reds_l) + sum(4.0 * 3 * f.R * max(f.dA_rows, f.db_rows)
                                                               for f in folds_l)
        timer.add("sgg::grad_finish_kernel", (nr, nf, tuple((r.rows, r.cols) for r in reds_l)), nb / 4.0, nb,
                  launch)


class _XW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, trans_w, act):
        y = xw_raw(x, w, bias, trans_w, act)
        ctx.trans_w, ctx.act, ctx.has_bias = trans_w, act, bias is not None
        ctx.save_for_backward(x, w, y if act else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        m = y if ctx.act else None    # ReLU backward dy * (y > 0), fused into the operands
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = xw_raw(dy, w, None, not ctx.trans_w, 0, mask=m, prec="fp32")
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            # X^T dY (K x N); nn.Linear-layout weights take it transposed (N x K)
            with side(x, dy, m):
                dw, cs = xtw(x, dy, colsum=True, trans_c=ctx.trans_w, mask=m)
            db = cs if ctx.has_bias else None
        return dx, dw, db, None, None


def xw(x, w, bias=None, trans_w=False, act=0):
    """act(x @ w + bias) (trans_w: w stored (N, K), i.e. nn.Linear layout)."""
    return _XW.apply(x, w, bias, trans_w, act)


def linear(x, lin, act=0):
    """nn.Linear through the MFMA node transform (weight is (out, in))."""
    return _XW.apply(x, lin.weight, lin.bias, True, act)


# ---------------------------------------------------------------------------
# discriminator scoring head (sgg_head_fwd / sgg_head_bwd)
# ---------------------------------------------------------------------------
def head_ok(seq):
    """real_classifier = make_mlp([K, N1, 1]) without BatchNorm / dropout, with
    ReLU or no activation after each Linear, in the shapes the fused head
    kernel takes: returns (lin1, lin2, act) or None."""
    mods = list(seq)
    lins = [m for m in mods if isinstance(m, torch.nn.Linear)]
    if len(lins) != 2 or any(not isinstance(m, (torch.nn.Linear, torch.nn.ReLU)) for m in mods):
        return None
    l1, l2 = lins
    if l2.out_features != 1 or l1.bias is None or l2.bias is None:
        return None
    if not _lib().sgg_head_ok(l1.in_features, l1.out_features):
        return None
    i1, i2 = mods.index(l1), mods.index(l2)
    relu1 = i1 + 1 < len(mods) and isinstance(mods[i1 + 1], torch.nn.ReLU)
    relu2 = i2 + 1 < len(mods) and isinstance(mods[i2 + 1], torch.nn.ReLU)
    if len(mods) != 2 + int(relu1) + int(relu2):
        return None
    return l1, l2, int(relu1) | (2 * int(relu2))


class BceLink:
    """Carries the BCE loss's backward arguments (upstream gradient, targets,
    split, weight) from _Bce / _BceTotal to the head backward, which forms the
    scores' gradient itself (sgg_head_bwd's bce_* arguments): one launch fewer
    per discriminator loss.  The BCE backward returns an unwritten placeholder
    as the scores' gradient; the head backward checks it received exactly that
    tensor (the scores had no other consumer)."""

    def __init__(self):
        self.pending = None
        self.forward_held = None   # the head's forward, waiting for the BCE forward (HEAD_FUSE)
        self.fused = None          # (seed, dx, slab) of the fused launch, when it ran

    def put(self, g, ya, yb, split, w, placeholder, nvalid=None):
        self.pending = (g, ya, yb, split, w, placeholder, nvalid)

    def take(self):
        p, self.pending = self.pending, None
        return p

    def run_fused(self, ya, yb, split, w, nvalid):
        """The BCE forward's call: issue the held head forward together with
        the head + BCE backward for the trainer's backward seed (the constant
        1.0 of const()) -- sgg_head_fwdbwd.  The BCE backward later confirms
        it received that seed (seed_ok); otherwise the head backward runs its
        own launches."""
        held, self.forward_held = self.forward_held, None
        if held is None:
            return
        x, W1, b1, W2, b2, act, y, wgrad = held
        lib = _lib()
        M, Kd = x.shape
        N1 = W1.shape[0]
        seed = const(1.0, x.device)
        dx = torch.empty(M, Kd, device=x.device, dtype=torch.float32)
        P = lib.sgg_head_slab_cols(Kd, N1)
        slab = torch.empty(max((M + 63) // 64, 1), P, device=x.device, dtype=torch.float32) if wgrad else None

        def launch():
            N.check(lib.sgg_head_fwdbwd(N.ptr(x), x.stride(0), M, Kd, N1, N.ptr(W1), N.ptr(b1), N.ptr(W2), N.ptr(b2),
                                        act, N.ptr(y), N.ptr(dx), dx.stride(0), N.ptr(slab), N.ptr(seed), N.ptr(ya),
                                        N.ptr(yb), int(split), float(w), N.ptr(nvalid), N.stream_ptr()),
                    "sgg_head_fwdbwd")
        launch()
        if timer.active and M > 0:
            timer.add("sgg::head_fwdbwd_kernel<%d, %d>" % (N1 // 16, Kd // 16), (M, Kd, N1, wgrad),
                      2.0 * M * N1 * (Kd + 1) + 2.0 * M * N1 * Kd * (2 if wgrad else 1),
                      4.0 * (M * Kd * (2 if wgrad else 1) + N1 * Kd + 2 * M + M * Kd
                             + (slab.numel() if wgrad else 0)), launch)
        self.fused = (seed, dx, slab)

    def flush_forward(self):
        """The held forward alone (no BCE forward came): sgg_head_fwd."""
        held, self.forward_held = self.forward_held, None
        if held is not None:
            x, W1, b1, W2, b2, act, y, _ = held
            _head_fwd(x, W1, b1, W2, b2, act, y, record=True)


HEAD_FUSE = os.environ.get("SGG_HEAD_FUSE", "1") != "0"
_HELD_HEADS = []   # links whose head forward is held (flushed when the handoff scope ends)


def _head_fwd(x, W1, b1, W2, b2, act, y, record=False):
    """sgg_head_fwd -> hid (Y into y)."""
    lib = _lib()
    M, Kd = x.shape
    N1 = W1.shape[0]
    hid = torch.empty(M, N1, device=x.device, dtype=torch.float32)

    def launch():
        N.check(lib.sgg_head_fwd(N.ptr(x), x.stride(0), M, Kd, N1, N.ptr(W1), N.ptr(b1), N.ptr(W2), N.ptr(b2),
                                 act, N.ptr(hid), N.ptr(y), N.stream_ptr()), "sgg_head_fwd")
    launch()
    if record and timer.active and M > 0:
        timer.add("sgg::head_fwd_kernel<%d, %d>" % (N1 // 16, Kd // 16), (M, Kd, N1), 2.0 * M * N1 * (Kd + 1),
                  4.0 * (M * Kd + N1 * Kd + M * N1 + M), launch)
    return hid


class _Head(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, act, bce_link=None):
        x = _rows(x, "x")
        if x.data_ptr() % 16 or x.stride(0) % 4:   # the kernel reads 16-byte blocks of a row
            x = x.contiguous()
        M, Kd = x.shape
        W1, W2 = W1.contiguous(), W2.contiguous()
        b1, b2 = b1.contiguous(), b2.contiguous()
        y = torch.empty(M, 1, device=x.device, dtype=torch.float32)
        wgrad = any(ctx.needs_input_grad[1:5])
        if bce_link is not None and HEAD_FUSE and M > 0:
            # held: the BCE forward on y issues it with the backward (BceLink.run_fused)
            bce_link.forward_held = (x, W1, b1, W2, b2, act, y, wgrad)
            _HELD_HEADS.append(bce_link)
            hid = None
        else:
            hid = _head_fwd(x, W1, b1, W2, b2, act, y, record=True)
        ctx.act = act
        ctx.bce_link = bce_link
        ctx.hid = hid
        ctx.save_for_backward(x, W1, b1, W2, b2, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib()
        x, W1, b1, W2, b2, y = ctx.saved_tensors
        need = ctx.needs_input_grad
        M, Kd = x.shape
        N1 = W1.shape[0]
        link = ctx.bce_link
        pend = link.take() if link is not None else None
        if link is not None and link.forward_held is not None:
            link.flush_forward()
        fused, hid = None, ctx.hid
        if link is not None and link.fused is not None:
            fused, link.fused = link.fused, None
        bce = None
        if pend is not None:
            g, ya, yb, split, w, ph, nvalid = pend
            if dy.data_ptr() != ph.data_ptr():
                raise N.NativeError("fused head + BCE backward: the scores have a consumer besides the BCE loss "
                                    "(set SGG_HEAD_BCE=0)")
            bce = (g.contiguous(), ya, yb, int(split), float(w), nvalid)
        else:
            dy = dy.contiguous()
        wgrad = any(need[1:5])
        P = lib.sgg_head_slab_cols(Kd, N1)
        rows = (M + 63) // 64
        if fused is not None and bce is not None and bce[0].data_ptr() == fused[0].data_ptr():
            # the BCE backward received the seed the fused launch assumed: dx and the slab are final
            dx, slab = fused[1], fused[2]
        else:
            if hid is None:   # (the fused launch kept no hidden layer: recompute it)
                hid = _head_fwd(x, W1, b1, W2, b2, ctx.act, torch.empty_like(y))
            dx = torch.empty(M, Kd, device=x.device, dtype=torch.float32)
            slab = torch.empty(max(rows, 1), P, device=x.device, dtype=torch.float32) if wgrad else None
            bg, bya, byb, bsp, bw, bnv = (N.ptr(bce[0]), N.ptr(bce[1]), N.ptr(bce[2]), bce[3], bce[4],
                                          N.ptr(bce[5])) if bce else (None, None, None, 0, 0.0, None)

            def launch():
                N.check(lib.sgg_head_bwd(N.ptr(x), x.stride(0), M, Kd, N1, N.ptr(W1), N.ptr(W2), N.ptr(hid),
                                         N.ptr(y), None if bce else N.ptr(dy), ctx.act, N.ptr(dx), dx.stride(0),
                                         N.ptr(slab), bg, bya, byb, bsp, bw, bnv, N.stream_ptr()), "sgg_head_bwd")
            launch()
            if timer.active and M > 0:
                timer.add("sgg::head_bwd_kernel<%d, %d>" % (N1 // 16, Kd // 16), (M, Kd, N1, wgrad),
                          2.0 * M * N1 * Kd * (2 if wgrad else 1),
                          4.0 * (M * Kd * (3 if wgrad else 2) + 2 * M * N1 + (slab.numel() if wgrad else 0)), launch)
        ctx.hid = None
        if not wgrad:
            return dx, None, None, None, None, None, None
        dW1 = torch.empty(N1, Kd, device=x.device, dtype=torch.float32)
        db1 = torch.empty(N1, device=x.device, dtype=torch.float32)
        dW2 = torch.empty(1, N1, device=x.device, dtype=torch.float32)
        db2 = torch.empty(1, device=x.device, dtype=torch.float32)
        if M == 0:
            for t in (dW1, db1, dW2, db2):
                t.zero_()
        else:
            gf = GradFinish()
            gf.rowsum(slab, rows, P, 0, N1 * Kd, dW1)
            gf.rowsum(slab, rows, P, N1 * Kd, N1, db1)
            gf.rowsum(slab, rows, P, N1 * Kd + N1, N1, dW2)
            gf.rowsum(slab, rows, P, N1 * Kd + 2 * N1, 1, db2)
            gf.run()
        return dx, dW1, db1, dW2, db2, None, None


HEAD_BCE = os.environ.get("SGG_HEAD_BCE", "1") != "0"
_BCE_HANDOFF = [0]


@contextlib.contextmanager
def bce_handoff():
    """Scope in which the discriminator head's scores may hand their BCE
    backward to the head's launch (BceLink).  Only the trainer's own steps
    open it: there the scores' gradient is never read by anyone but the head,
    whereas outside it a direct query (autograd.grad on the scores,
    retain_grad) must see a real gradient, not the handoff's placeholder."""
    _BCE_HANDOFF[0] += 1
    try:
        yield
    finally:
        _BCE_HANDOFF[0] -= 1
        if _BCE_HANDOFF[0] == 0:   # a held head forward no BCE forward took: issue it now
            while _HELD_HEADS:
                _HELD_HEADS.pop().flush_forward()


def head(x, spec):
    """real_classifier forward through the fused head (spec = head_ok(seq)).
    With autograd on inside bce_handoff(), the scores carry a BceLink: a
    K.bce_pair / K.bce_pair_total on them hands its backward to the head's
    launch."""
    l1, l2, act = spec
    link = BceLink() if (HEAD_BCE and _BCE_HANDOFF[0] > 0 and torch.is_grad_enabled()) else None
    y = _Head.apply(x, l1.weight, l1.bias, l2.weight, l2.bias, act, link)
    if link is not None:
        y._sgg_bce_link = link
    return y


# ---------------------------------------------------------------------------
# optimizer step
# ---------------------------------------------------------------------------
class ClipAdam:
    """[nn.utils.clip_grad_norm_(params, max_norm)] + optim.Adam.step() in two
    launches (sgg_adam_step; scripts/train.py:418-427, :472-482).

    The state lives in a torch.optim.Adam (capturable layout: per-parameter
    float32 device 'step', 'exp_avg', 'exp_avg_sq'), so `state_dict()` /
    `load_state_dict()` are torch's: a parameter gets its state the first
    time it has a gradient, exactly as torch's Adam (parameters whose grad is
    None are skipped and keep no state), so a state dict round-trips with a
    reference checkpoint's optimizer state (train.py:238, :363).  Graph-
    capturable: the tensor list is passed by value (the trainers warm up
    eagerly before capturing, which creates the state)."""

    MAX_TENSORS = 48

    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8):
        self.params = [p for p in params]
        self.opt = torch.optim.Adam(self.params, lr=lr, betas=betas, eps=eps, capturable=True)
        self._ws = None

    def _state(self, p):
        st = self.opt.state[p]
        if "exp_avg" not in st:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        elif not torch.is_tensor(st["step"]) or st["step"].device != p.device or st["step"].dtype != torch.float32:
            st["step"] = torch.as_tensor(float(st["step"]), dtype=torch.float32).to(p.device)
        return st

    @property
    def param_groups(self):
        return self.opt.param_groups

    def state_dict(self):
        return self.opt.state_dict()

    def load_state_dict(self, sd):
        """torch's Adam state dict, e.g. a reference checkpoint's
        g_optim_state / d_optim_state (host 'step' counters are moved to the
        device, the capturable layout the fused step reads)."""
        self.opt.load_state_dict(sd)
        for p in self.params:
            if self.opt.state.get(p):
                self._state(p)

    def zero_grad(self, set_to_none=True):
        self.opt.zero_grad(set_to_none=set_to_none)

    def step(self, max_norm=0.0):
        lib = _lib()
        grp = self.opt.param_groups[0]
        act = [p for p in self.params if p.grad is not None]
        if max_norm > 0:            # the norm spans every tensor: one call
            self._launch(lib, act, grp, max_norm)
            return
        for i in range(0, len(act), self.MAX_TENSORS):
            self._launch(lib, act[i:i + self.MAX_TENSORS], grp, 0.0)

    def _launch(self, lib, act, grp, max_norm):
        import ctypes
        if len(act) > self.MAX_TENSORS:
            raise N.NativeError("ClipAdam: %d tensors with gradients, the fused step takes <= %d (clipping needs "
                              "them in one call)" % (len(act), self.MAX_TENSORS))
        for p in act:
            for t in (p, p.grad):
                if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
                    raise N.NativeError("ClipAdam: parameters and grads must be contiguous fp32 device tensors")
        n = len(act)
        st = [self._state(p) for p in act]
        for p in act:    # in-place update through raw pointers: invalidate cached folds of these weights
            _EPOCH[p.data_ptr()] = _EPOCH.get(p.data_ptr(), 0) + 1
        arr = lambda xs: (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])
        numel = (ctypes.c_longlong * n)(*[p.numel() for p in act])
        total = sum(p.numel() for p in act)
        parts = lib.sgg_adam_parts(total)
        if self._ws is None or self._ws.numel() < parts:
            self._ws = torch.zeros(parts, device=act[0].device, dtype=torch.float32)   # (the ticket word: 0)
        b1, b2 = grp["betas"]
        N.check(lib.sgg_adam_step(arr(act), arr([p.grad for p in act]), arr([s["exp_avg"] for s in st]),
                                  arr([s["exp_avg_sq"] for s in st]), numel, n, float(grp["lr"]), float(b1),
                                  float(b2), float(grp["eps"]), float(max_norm), arr([s["step"] for s in st]),
                                  N.ptr(self._ws), self._ws.numel() * 4, N.stream_ptr()), "sgg_adam_step")


# ---------------------------------------------------------------------------
# social pooling
# ---------------------------------------------------------------------------
class OwnershipError(N.NativeError):
    """A re-issuable launch holds a raw device pointer (inside a ctypes
    descriptor) to memory it does not keep alive."""


def _storage_span(obj):
    """(begin, end) device address range of a tensor's / storage's memory."""
    s = obj.untyped_storage() if isinstance(obj, torch.Tensor) else obj
    b = s.data_ptr()
    return (b, b + s.nbytes())


def _walk_held(obj, spans, descs, seen, depth=0):
    """Everything a closure holds: memory spans of tensors / storages, and the
    ctypes descriptors (structs, arrays of them) whose pointer fields the
    launch hands to the device."""
    import ctypes
    if obj is None or isinstance(obj, (int, float, str, bytes, bool)) or depth > 6 or id(obj) in seen:
        return
    seen.add(id(obj))
    if isinstance(obj, (torch.Tensor, torch.UntypedStorage)):
        sp = _storage_span(obj)
        if sp is not None:
            spans.append(sp)
        return
    if isinstance(obj, (ctypes.Structure, ctypes.Array)):
        descs.append(obj)
        for v in getattr(obj, "__dict__", {}).values():   # an owned descriptor's kept buffers
            _walk_held(v, spans, descs, seen, depth + 1)
        return
    if isinstance(obj, (list, tuple, set, frozenset)):
        for v in obj:
            _walk_held(v, spans, descs, seen, depth + 1)
        return
    if isinstance(obj, dict):
        for v in obj.values():
            _walk_held(v, spans, descs, seen, depth + 1)
        return
    if isinstance(obj, functools.partial):
        for v in (obj.func, obj.args, obj.keywords):
            _walk_held(v, spans, descs, seen, depth + 1)
        return
    code = getattr(obj, "__code__", None)
    if code is not None:   # a function: its closure cells and bound defaults
        for c in obj.__closure__ or ():
            try:
                _walk_held(c.cell_contents, spans, descs, seen, depth + 1)
            except ValueError:   # an empty cell
                pass
        _walk_held(obj.__defaults__, spans, descs, seen, depth + 1)
        _walk_held(obj.__kwdefaults__, spans, descs, seen, depth + 1)
        return
    if hasattr(obj, "__self__") and hasattr(obj, "__func__"):   # a bound method
        _walk_held(obj.__self__, spans, descs, seen, depth + 1)
        return
    d = getattr(obj, "__dict__", None)
    if d is not None and not isinstance(obj, (type, torch.nn.Module)):
        _walk_held(d, spans, descs, seen, depth + 1)


def _desc_pointers(desc, path="", out=None):
    """[(field path, address)] of every non-null pointer field of a ctypes
    struct / array (nested structs and pointer arrays included)."""
    import ctypes
    out = [] if out is None else out
    if isinstance(desc, ctypes.Array):
        for i in range(len(desc)):
            v = desc[i]
            if isinstance(v, (ctypes.Structure, ctypes.Array)):
                _desc_pointers(v, "%s[%d]" % (path, i), out)
            elif desc._type_ is ctypes.c_void_p and v:
                out.append(("%s[%d]" % (path, i), v))
        return out
    for fname, ftype in desc._fields_:
        v = getattr(desc, fname)
        if isinstance(v, (ctypes.Structure, ctypes.Array)):
            _desc_pointers(v, path + "." + fname, out)
        elif ftype is ctypes.c_void_p and v:
            out.append((path + "." + fname, v))
    return out


def check_ownership(fn, name="launch"):
    """Assert that every device pointer a re-issuable launch `fn` passes
    through a ctypes descriptor lies in memory that `fn` itself keeps alive
    (a tensor or storage reachable from its closure, its bound defaults, or
    the descriptor's own kept buffers).  Arguments passed as N.ptr(t) are
    re-evaluated on tensors the closure holds, so they are owned by
    construction; a descriptor's pointers are raw integers, and a buffer that
    only the descriptor names can be freed and reused before a re-issue (the
    round-3 hipErrorIllegalAddress)."""
    spans, descs = [], []
    _walk_held(fn, spans, descs, set())
    spans.sort()
    for d in descs:
        for path, p in _desc_pointers(d, type(d).__name__):
            if not any(b <= p < e for b, e in spans):
                raise OwnershipError("%s: descriptor field %s points to 0x%x, which the re-issuable launch does "
                                     "not keep alive" % (name, path, p))


@contextlib.contextmanager
def capture_guard():
    """Around a HIP-graph capture: collect garbage first and keep the cyclic
    garbage collector off until the capture ends.  A CUDAGraph reachable only
    through a reference cycle is destroyed whenever the collector happens to
    run; if that is inside another capture, ~CUDAGraph's synchronisation is
    illegal on the capturing stream and the process aborts (the round-3
    hipErrorStreamCaptureUnsupported).  Nothing outlives
    the capture: the collector's state is restored as it was."""
    import gc
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def capture_error_mode():
    """The stream-capture mode of this process's HIP-graph captures:
    "thread_local" once a torch.distributed process group exists -- its
    watchdog thread polls collective events while we capture, which the
    global mode treats as an illegal call and answers by invalidating the
    capture -- else "global" (the strictest)."""
    import torch.distributed as dist
    return "thread_local" if dist.is_available() and dist.is_initialized() else "global"


@contextlib.contextmanager
def gc_frozen():
    """Scope in which every object alive at entry (captured graphs and the
    step state they keep) sits in the collector's permanent generation, so a
    full collection during a replay loop does not re-scan them (milliseconds
    of host time against sub-millisecond replays).  Opt-in and scoped: the
    objects frozen here are unfrozen at exit, so cyclic garbage among them is
    collected as usual afterwards.  When the process already froze objects
    itself, its freeze is left alone (nothing frozen or unfrozen here)."""
    import gc
    own = gc.get_freeze_count() == 0
    if own:
        gc.collect()
        gc.freeze()
    try:
        yield
    finally:
        if own:
            gc.unfreeze()


class LaunchTimer:
    """Per-kernel device timing of the hot ops (bench.py's roofline).

    While active, every instrumented launch (pooling, LSTM sequences, GAT
    encoder, node transforms, weight-gradient reductions) is recorded with
    its kernel name (as rocprofv3 lists it), its algorithmic FLOP and HBM
    bytes (work models in DESIGN.md section 4) and a closure that re-issues
    the identical launch on the same buffers (every instrumented op is
    idempotent: it rewrites its outputs from its inputs).  The closure must
    own every buffer it launches on: `add` checks that each pointer inside
    its ctypes descriptors lies in a tensor / storage reachable from the
    closure (check_ownership) and raises OwnershipError otherwise, so a
    recorded launch stays valid after the step's own tensors are dropped.
    `replay()` captures `reps` back-to-back re-issues of each distinct launch
    into a HIP graph and replays it between two HIP events on the current
    stream, so the device never waits for the host and elapsed / reps is the
    kernel's average device duration (an event pair around one eager launch
    would also count host launch latency)."""

    def __init__(self):
        self.active = False
        self.rec = []

    def start(self):
        self.active, self.rec = True, []

    def stop(self):
        self.active = False
        torch.cuda.synchronize()
        out, self.rec = self.rec, []
        return out

    def add(self, name, key, flop, nbytes, relaunch):
        if self.active:
            check_ownership(relaunch, name)
            self.rec.append((name, (name,) + tuple(key), float(flop), float(nbytes), relaunch))

    @staticmethod
    def replay(records, reps=20):
        """records -> {key: dict(name, launches, flop, bytes, ms)} with ms the
        average device time of one launch."""
        with capture_guard():   # (one collection for all the captures below)
            return LaunchTimer._replay(records, reps)

    @staticmethod
    def _replay(records, reps):
        res = {}
        cur = torch.cuda.current_stream()
        for name, key, fl, nb, fn in records:
            if key in res:
                res[key]["launches"] += 1
                continue
            # the re-issues are captured into a HIP graph and replayed, so the
            # events bracket device work only (an eager loop of ctypes launches
            # is host-bound for the few-us kernels)
            side = private_stream("timer")
            side.wait_stream(cur)
            graph = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.stream(side):
                    fn()                          # warm (instruction cache, L2)
                    graph.capture_begin(capture_error_mode=capture_error_mode())
                    for _ in range(reps):
                        fn()
                    graph.capture_end()
            except RuntimeError:
                graph = None
            cur.wait_stream(side)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if graph is not None:
                graph.replay()
            else:
                for _ in range(reps):
                    fn()
            e1.record()
            e1.synchronize()
            res[key] = dict(name=name, launches=1, flop=fl, bytes=nb, ms=e0.elapsed_time(e1) / reps)
            del graph
        return res


timer = LaunchTimer()


def _pool_flops(scenes, bn):
    import numpy as np
    sz = np.diff(scenes.host_off).astype(np.float64)
    return float((sz * sz).sum()) * 512.0 * (4 + 2 * bn)


def _pool_kname(bn, gpw, nchunks, bf16, dev, max_n=None, max_rows=None):
    """The forward kernel the library picks (pool.hip launch_fwd_g / launch_fwd_bf16)."""
    if bf16:
        g = 4 if gpw >= 4 and bn <= 48 else (2 if gpw >= 2 else 1)
        if max_n is not None and max_n >= 32 and os.environ.get("SGG_POOL_JB") != "0":
            # the j-block form, its wave groups from the plan's rows
            gj = "*" if max_rows is None else (4 if max_rows > 16 else (2 if max_rows > 8 else 1))
            return "sgg::pool_fwd_bf16_jb_kernel<%d, %s>" % (bn, gj)
        return "sgg::pool_fwd_bf16_kernel<%d, %d>" % (bn, g)
    if gpw <= 2 and 32 <= bn <= 48 and os.environ.get("SGG_POOL_X3", "1")[:1] != "0":
        return "sgg::pool_fwd_x3_kernel<%d, %d>" % (bn, gpw)
    small = gpw <= 2 and nchunks <= 4 * torch.cuda.get_device_properties(dev).multi_processor_count
    return "sgg::" + ("pool_fwd_v_kernel<%d, %d>" % (bn, gpw) if small else "pool_fwd_kernel<%d, %d, 2>" % (bn, gpw))


def _pool_wbytes(bn):
    return 4.0 * (1024 + bn * 512 + bn)     # A, W2, b2


class PoolRider:
    """pool_pair(): the block's first pooling forward (the discriminator
    step's generator pooling, scripts/train.py:400) is held; the next one of
    the same net and plan width (the generator step's, :443) issues both in
    ONE launch (sgg_pool_fwd2).  Nothing may read the held forward's outputs
    before that; a held forward nobody carried is issued on exit."""

    def __init__(self):
        self.held = None
        self.done = False
        self.carried = False

    def hold(self, batch, keep, weights, bn, bf16, gpw, nchunks, work, launch):
        self.held = (batch, keep, weights, bn, bf16, gpw, nchunks, work, launch)

    def fits(self, weights, bn, bf16, gpw):
        if self.held is None:
            return False
        _, _, wh, bnh, bfh, gph, _, _, _ = self.held
        return bnh == bn and bfh == bf16 and gph == gpw and all(a is b for a, b in zip(wh, weights))

    def carry(self, batch, keep, nchunks, work):
        """-> (the paired launch, (kernel name, S, B, flop, bytes, chunks) of both)."""
        a, keep_a, (A, W2, b2), bn, bf16, gpw, nch_a, work_a, _ = self.held
        self.held = None
        self.done = self.carried = True
        lib = _lib()
        b = batch

        def pl(k=(keep_a, keep, A, W2, b2)):
            N.check(lib.sgg_pool_fwd2(N.ctypes.byref(a), N.ctypes.byref(b), N.ptr(A), N.ptr(W2), N.ptr(b2), bn,
                                      int(bf16), N.stream_ptr()), "sgg_pool_fwd2")
        S2, B2 = work_a[0] + work[0], work_a[1] + work[1]
        return pl, (None, S2, B2, work_a[2] + work[2], work_a[3] + work[3], nch_a + nchunks)

    def flush(self):
        if self.held is not None:
            _, _, (A, W2, b2), bn, bf16, gpw, nch, work, launch = self.held
            self.held = None
            launch()
            if timer.active:
                timer.add(_pool_kname(bn, gpw, nch, bf16, A.device), work[:2], work[2], work[3] + _pool_wbytes(bn),
                          launch)
        self.done = True


_PRIDER = [None]


@contextlib.contextmanager
def pool_pair():
    """The block's first pooling forward rides with the next one (PoolRider)."""
    prev = _PRIDER[0]
    r = _PRIDER[0] = PoolRider()
    try:
        yield r
    finally:
        _PRIDER[0] = prev
        r.flush()


class _Pool(torch.autograd.Function):
    """PoolHiddenNet on raw parameters: W1 (512 x (E + Hd)) = [W1e | W1h], the
    spatial embedding (We, be), b1, W2 (bn x 512), b2.  Forward: one fold
    launch (A = W1e We, c = W1e be + b1), U = h W1h^T + c (sgg_xw on the W1h
    block in place), the fused pooling kernel.  Backward: the pooling
    backward, dW1 assembled in place (fold backward -> left block, X^T dU
    transposed -> right block)."""

    @staticmethod
    def forward(ctx, h, pos, W1, We, be, b1, W2, b2, scenes, link=None, U=None):
        lib = _lib()
        ctx.link = link
        h = _rows(h, "h")
        pos = _req(pos, "pos").contiguous()
        B, Hd = h.shape
        E = We.shape[0]
        bn = W2.shape[0]
        assert pos.shape == (B, 2) and scenes.B == B, (pos.shape, B, scenes.B)
        assert W1.shape == (512, E + Hd), (W1.shape, E, Hd)
        W1 = W1.contiguous()
        W2 = W2.contiguous()
        b2 = b2.contiguous()
        A, c = fold_fwd(W1[:, :E], We, be, b1)
        if U is None:
            U = xw_raw(h, W1[:, E:], c, trans_w=True)             # B x 512
        else:                                                     # from the encoder kernel's epilogue
            assert U.shape == (B, 512) and U.is_contiguous()
        out = torch.empty(B, bn, device=h.device, dtype=torch.float32)
        am = torch.empty(B, bn, device=h.device, dtype=torch.int32)
        # the opt-in bf16 precision: the 512 -> bn contraction on bf16 MFMA (its own chunk plan)
        bf16 = _PRECISION == "bf16"
        fwd = lib.sgg_pool_fwd_bf16 if bf16 else lib.sgg_pool_fwd
        plan = scenes.pool_plan(bn, bf16=bf16)
        chunks, nchunks, max_rows, gpw = plan[:4]
        ncd = plan[4] if len(plan) > 4 else None    # a fixed-capacity plan's device chunk count
        if bf16 and ncd is not None:
            gpw = 4   # (a fixed-capacity fp32 plan: its chunks run in passes of up to 512 pairs)

        def launch():
            N.check(fwd(N.ptr(U), N.ptr(pos), N.ptr(A), N.ptr(W2), N.ptr(b2), N.ptr(scenes.scene_off),
                        N.ptr(chunks), nchunks, max_rows, gpw, B, bn, scenes.max_n, N.ptr(out),
                        N.ptr(am), N.ptr(ncd), N.stream_ptr()), "sgg_pool_fwd")
        nb = 4.0 * (B * 512 + 2 * B) + 8.0 * B * bn     # + the weights, once per launch (_pool_timing)
        work = (scenes.S, B, _pool_flops(scenes, bn), nb)
        rider = _PRIDER[0]
        if rider is not None and not rider.done and rider.held is None:
            # the block's first pooling forward: held until the next one carries it
            batch = N.PoolBatch(N.ptr(U), N.ptr(pos), N.ptr(scenes.scene_off), N.ptr(chunks), nchunks, max_rows,
                                gpw, B, scenes.max_n, N.ptr(out), N.ptr(am), N.ptr(ncd))
            rider.hold(batch, (U, pos, scenes.scene_off, chunks, out, am, ncd), (A, W2, b2), bn, bf16, gpw,
                       nchunks, work, launch)
        elif rider is not None and rider.fits((A, W2, b2), bn, bf16, gpw):
            batch = N.PoolBatch(N.ptr(U), N.ptr(pos), N.ptr(scenes.scene_off), N.ptr(chunks), nchunks, max_rows,
                                gpw, B, scenes.max_n, N.ptr(out), N.ptr(am), N.ptr(ncd))
            pl, (name, S2, B2, fl2, nb2, nch2) = rider.carry(batch, (U, pos, scenes.scene_off, chunks, out, am, ncd),
                                                             nchunks, work)
            pl()
            if timer.active:
                timer.add(_pool_kname(bn, gpw, nch2, bf16, h.device, scenes.max_n, max_rows), (S2, B2, "pair"), fl2,
                          nb2 + _pool_wbytes(bn), pl)
        else:
            if rider is not None:
                rider.flush()
            launch()
            if timer.active:
                timer.add(_pool_kname(bn, gpw, nchunks, bf16, h.device, scenes.max_n, max_rows), (scenes.S, B), work[2],
                          nb + _pool_wbytes(bn), launch)
        ctx.scenes = scenes
        ctx.E = E
        ctx.save_for_backward(h, pos, W1, We, be, A, W2, U, out, am)
        ctx.mark_non_differentiable(am)
        ctx.set_materialize_grads(False)   # no zero-filled gradient for the argmax output
        return out, am

    @staticmethod
    def backward(ctx, dout, _dam):
        lib = _lib()
        h, pos, W1, We, be, A, W2, U, out, am = ctx.saved_tensors
        sc, E = ctx.scenes, ctx.E
        B, bn = out.shape
        dout = dout.contiguous()
        need = ctx.needs_input_grad
        wgrad = any(need[2:8])       # False: weights frozen (the G-step's discriminator), input gradient only
        P = bn * 512 + 1024 + bn
        dU = torch.empty(B, 512, device=h.device, dtype=torch.float32)
        part = torch.empty(lib.sgg_pool_bwd_grid(sc.S), P, device=h.device, dtype=torch.float32) if wgrad else None
        def launch():
            N.check(lib.sgg_pool_bwd(N.ptr(U), N.ptr(pos), N.ptr(A), N.ptr(W2), N.ptr(out), N.ptr(am), N.ptr(dout),
                                     N.ptr(sc.scene_off), sc.S, B, bn, sc.max_n, N.ptr(dU), N.ptr(part),
                                     N.stream_ptr()), "sgg_pool_bwd")
        launch()
        if timer.active:
            nb = 8.0 * B * 512 + 12.0 * B * bn + 4.0 * 512 * (2 + bn) + (4.0 * part.numel() if wgrad else 0.0)
            jq = max(1, min(8, 256 // sc.S)) if sc.S >= 1 else 1   # pool.hip pool_bwd_jq / launch_bwd
            stage = (sc.max_n + jq - 1) // jq + 1 <= 16
            timer.add("sgg::pool_bwd_kernel<%d, %s, %s>" % (bn, "true" if wgrad else "false",
                                                            "true" if stage else "false"), (sc.S, B),
                      8.0 * B * bn * 512, nb, launch)
        dh = None
        H = h.shape[1]
        dual = need[0] and wgrad and DUAL_POOL_BWD and not SIDE_STREAM and H <= 64
        if need[0]:
            base = ctx.link.take() if ctx.link is not None else None
            if dual:
                # dh = dU W1h (+ the other consumer's gradient of h) and the
                # h^T dU partials (+ column sums) in ONE launch
                dh = base if base is not None else torch.empty(B, H, device=h.device, dtype=torch.float32)
                splits = lib.sgg_xtw_splits(B, H, 512)
                ws = torch.empty(splits * (H * 512 + 512), device=h.device, dtype=torch.float32)
                W1h = W1[:, E:]
                acc = int(base is not None)

                def launch2():
                    N.check(lib.sgg_pool_dh_dw(N.ptr(dU), 512, N.ptr(W1h), W1h.stride(0), N.ptr(dh), dh.stride(0),
                                               acc, N.ptr(h), h.stride(0), B, H, N.ptr(ws), ws.numel() * 4,
                                               N.stream_ptr()), "sgg_pool_dh_dw")
                launch2()
                if timer.active:   # (re-issued like sgg_xw's accumulating launches: timing, not values)
                    mt = 4 if H >= 64 else (H + 15) // 16
                    timer.add("sgg::xw_xtw_kernel<%d>" % mt, (B, H), 4.0 * B * 512 * H,
                              4.0 * (2 * B * 512 + 512 * H + 2 * B * H) + 4.0 * ws.numel(), launch2)
            else:
                # dh = dU W1h (+ the other consumer's gradient of h, accumulated in the same launch)
                dh = xw_raw(dU, W1[:, E:], None, trans_w=False, prec="fp32", out=base, act=0 if base is None else 2)
        if not wgrad:
            return dh, None, None, None, None, None, None, None, None, None, None
        with side(part, h, dU, W1, We, be):
            # one launch after the dW1h partials: dW2, db2 (slab [dW2 | dA | db2]
            # row sums), dW1h = dU^T h, dc = sum_j dU_j, and the fold backward
            # of (dA, dc) -> dW1e, dWe, dbe
            rows = part.shape[0]
            if not dual:
                ws, splits = xtw_partial(h, dU, colsum=True)
            dW1 = torch.empty_like(W1)
            dW2 = torch.empty(bn, 512, device=h.device, dtype=torch.float32)
            db2 = torch.empty(bn, device=h.device, dtype=torch.float32)
            dc = torch.empty(512, device=h.device, dtype=torch.float32)
            gf = GradFinish()
            gf.rowsum(part, rows, P, 0, bn * 512, dW2)
            gf.rowsum(part, rows, P, bn * 512 + 1024, bn, db2)
            gf.xtw_sums(ws, splits, H, 512, dW1[:, E:], trans_c=True, colsum=dc)
            _, dWe, dbe = gf.fold(W1[:, :E], We, be, part, rows, P, bn * 512, ws[splits * H * 512:], splits, 512, 0,
                                  dW=dW1[:, :E])
            gf.run()
        return dh, None, dW1, dWe, dbe, dc, dW2, db2, None, None, None


class Handoff:
    """A one-shot slot passing a backward's arguments to the next backward
    that consumes them (see _Split2 / _LSTMSeq)."""

    def __init__(self):
        self.pending = None

    def put(self, *args):
        self.pending = args

    def take(self):
        p, self.pending = self.pending, None
        return p


class CopiesLink:
    """Carries the decoder-initial-state gradient of the best-of-k copies
    (decoder_init's backward) to the GAT encoder's backward, which sums the
    copies while loading dy (SggGatEncArgs.dy_copies) -- no separate sum
    launch.  decoder_init returns copy 0's rows (a view into the same
    buffer) as the autograd gradient."""

    def __init__(self):
        self.pending = None

    def put(self, base, copies, cstride, ld):
        self.pending = (base, copies, cstride, ld)

    def take(self):
        p, self.pending = self.pending, None
        return p


class GradLink:
    """Carries one input gradient from a backward to a LATER backward of the
    same tensor's other consumer, which adds it inside its own launch: the
    generator's encoder state feeds the pooling net and (as the first input
    block) the GAT encoder, whose backward runs first; the pooling backward's
    dh = dU W1h then accumulates it (sgg_xw act bit 1) instead of autograd
    summing the two gradients in an extra launch."""

    def __init__(self):
        self.grad = None

    def put(self, g):
        assert self.grad is None, "GradLink: gradient already pending"
        self.grad = g.contiguous()

    def take(self):
        g, self.grad = self.grad, None
        return g


def social_pool(h, pos, W1, We, be, b1, W2, b2, scenes, link=None, U=None):
    """PoolHiddenNet core (models.py:497-549) -> (B, bn); see sgg_pool_fwd.
    link: a GradLink whose pending gradient of h the backward adds to dh.
    U: h W1[:, E:]^T + c when the encoder kernel already produced it
    (pool_u_spec / lstm_sequence(proj_u=...))."""
    out, _ = _Pool.apply(h, pos, W1, We, be, b1, W2, b2, scenes, link, U)
    return out


def pool_u_spec(pool):
    """(Wu, cu) of a PoolHiddenNet for the encoder's projection epilogue:
    Wu = W1[:, E:] (in place), cu = W1[:, :E] be + b1 (the cached fold)."""
    l1, E = pool.mlp_pre_pool[0], pool.embedding_dim
    _, c = fold_fwd(l1.weight[:, :E], pool.spatial_embedding.weight, pool.spatial_embedding.bias, l1.bias)
    return l1.weight[:, E:], c


# ---------------------------------------------------------------------------
# graph attention
# ---------------------------------------------------------------------------
class _GatAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wh, a, bias, labels, seg_off, nseg, max_seg, alpha, mode, epi, heads):
        lib = _lib()
        wh = _req(wh, "wh").contiguous()
        n, HF = wh.shape
        F = HF // heads
        ctx.a_shape = a.shape
        a = a.contiguous().view(-1)
        if bias is not None:
            bias = bias.contiguous()
        # (rows past the last segment -- the zero-padded group buffers of the
        # complete-graph mode -- are written zero by the kernel)
        y = torch.empty(n, HF, device=wh.device, dtype=torch.float32)
        hp = torch.empty(n, HF, device=wh.device, dtype=torch.float32) if epi else None
        N.check(lib.sgg_gat_fwd(N.ptr(wh), heads, N.ptr(a), N.ptr(bias), N.ptr(labels), N.ptr(seg_off), nseg, n, F,
                                float(alpha), mode, epi, max_seg, N.ptr(hp), N.ptr(y), HF, N.stream_ptr()),
                "sgg_gat_fwd")
        ctx.meta = (labels, seg_off, nseg, max_seg, float(alpha), mode, epi, heads, bias is not None)
        ctx.save_for_backward(wh, a, hp, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib()
        wh, a, hp, y = ctx.saved_tensors
        labels, seg_off, nseg, max_seg, alpha, mode, epi, heads, has_bias = ctx.meta
        n, HF = wh.shape
        F = HF // heads
        dy = dy.contiguous()
        dWh = torch.empty(n, HF, device=wh.device, dtype=torch.float32)
        ds = torch.empty(n, heads, device=wh.device, dtype=torch.float32)
        dt = torch.empty(n, heads, device=wh.device, dtype=torch.float32)
        N.check(lib.sgg_gat_bwd(N.ptr(wh), heads, N.ptr(a), N.ptr(labels), N.ptr(seg_off), nseg, n, F, alpha, mode,
                                epi, max_seg, N.ptr(hp), N.ptr(y), N.ptr(dy), HF, N.ptr(dWh), N.ptr(ds), N.ptr(dt),
                                N.stream_ptr()), "sgg_gat_bwd")
        if not ctx.needs_input_grad[1] and not has_bias:
            return dWh, None, None, None, None, None, None, None, None, None, None
        dsdt = torch.cat([ds, dt], 1)                                       # n x [ds_h | dt_h]
        if heads == 1:
            da = xtw(wh, dsdt).t().reshape(ctx.a_shape)
        else:
            C = xtw(wh, dsdt).view(heads, F, 2, heads)                     # [h, f, src|dst, h']
            hh = torch.arange(heads, device=wh.device)
            da = C[hh, :, :, hh].permute(0, 2, 1).reshape(heads, 2 * F)    # diagonal blocks h == h'
        dbias = None
        if has_bias:
            dpre = dy if epi == 0 else dy * torch.where(hp > 0, torch.ones_like(hp), torch.exp(hp))
            # a near-cancelling sum (the next layer's instance norm removes
            # each feature's mean over the scene): accumulated in fp64
            dbias = dpre.view(n, heads, F).double().sum((0, 1)).float()
        return dWh, da, dbias, None, None, None, None, None, None, None, None


class _GatAttnEx(torch.autograd.Function):
    """The batched multi-head GAT's attention (sgg_gat_fwd_ex / _bwd_ex):
    a_src / a_dst as the module holds them, and their gradients and the
    bias's finished on the device (no host-side concatenation, products or
    reductions)."""

    @staticmethod
    def forward(ctx, wh, a_src, a_dst, bias, labels, seg_off, nseg, max_seg, alpha, mode, epi, heads):
        lib = _lib()
        wh = _req(wh, "wh").contiguous()
        n, HF = wh.shape
        F = HF // heads
        a_src, a_dst = a_src.contiguous(), a_dst.contiguous()
        if a_src.numel() != heads * F or a_dst.numel() != heads * F:
            raise ValueError("a_src / a_dst must hold heads x F = %d values" % (heads * F))
        if bias is not None:
            bias = bias.contiguous()
        y = torch.empty(n, HF, device=wh.device, dtype=torch.float32)
        hp = torch.empty(n, HF, device=wh.device, dtype=torch.float32) if epi else None
        N.check(lib.sgg_gat_fwd_ex(N.ptr(wh), heads, N.ptr(a_src), N.ptr(a_dst), N.ptr(bias), N.ptr(labels),
                                   N.ptr(seg_off), nseg, n, F, float(alpha), mode, epi, max_seg, N.ptr(hp), N.ptr(y),
                                   HF, N.stream_ptr()), "sgg_gat_fwd_ex")
        ctx.meta = (labels, seg_off, nseg, max_seg, float(alpha), mode, epi, heads, bias is not None, F)
        ctx.save_for_backward(wh, a_src, a_dst, hp, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib()
        wh, a_src, a_dst, hp, y = ctx.saved_tensors
        labels, seg_off, nseg, max_seg, alpha, mode, epi, heads, has_bias, F = ctx.meta
        n, HF = wh.shape
        dy = dy.contiguous()
        dWh = torch.empty(n, HF, device=wh.device, dtype=torch.float32)
        da_s = torch.empty_like(a_src)
        da_d = torch.empty_like(a_dst)
        dbias = torch.empty(F, device=wh.device, dtype=torch.float32) if has_bias else None
        work = torch.empty(max(16, int(lib.sgg_gat_bwd_ex_work_bytes(nseg, heads, F))), device=wh.device,
                           dtype=torch.uint8)
        _gat_bwd_ex_launch(wh, heads, a_src, a_dst, labels, seg_off, nseg, n, F, alpha, mode, epi, max_seg, hp, y, dy,
                           dWh, da_s, da_d, dbias, work)
        return dWh, da_s, da_d, dbias, None, None, None, None, None, None, None, None


def _gat_bwd_ex_launch(wh, heads, a_src, a_dst, labels, seg_off, nseg, n, F, alpha, mode, epi, max_seg, hp, y, dy,
                       dWh, da_s, da_d, dbias, work):
    lib = _lib()
    HF = heads * F

    def launch():
        N.check(lib.sgg_gat_bwd_ex(N.ptr(wh), heads, N.ptr(a_src), N.ptr(a_dst), N.ptr(labels), N.ptr(seg_off), nseg,
                                   n, F, alpha, mode, epi, max_seg, N.ptr(hp), N.ptr(y), N.ptr(dy), HF, N.ptr(dWh),
                                   N.ptr(da_s), N.ptr(da_d), N.ptr(dbias), N.ptr(work), N.stream_ptr()),
                "sgg_gat_bwd_ex")
    launch()
    if timer.active and n > 0:
        # per (segment, head): datt = dhp Wh^T, dWh = att^T dhp, the attention
        # recompute ~ 3 x 2 n^2 F (n^2 bounded by n * max_seg); operands
        # Wh, dy, hp (+ y) in, dWh out
        timer.add("sgg::gat_bwd_kernel+gat_param_reduce_kernel", (n, HF, heads, max_seg),
                  6.0 * n * max_seg * HF, 4.0 * n * HF * (4 if epi else 3), launch)


def gat_attention_ex(wh, a_src, a_dst, alpha, graph, epilogue, heads=1, bias=None):
    """gat_attention with a_src / a_dst separate (heads x F each, any shape
    of that size) and the parameter gradients finished in the kernels."""
    return _GatAttnEx.apply(wh, a_src, a_dst, bias, graph.labels, graph.seg_off, graph.nseg, graph.max_seg, alpha,
                            graph.mode, epilogue, heads)


class _GatLayer(torch.autograd.Function):
    """One batched-GAT layer of the sgangat family (instance norm over each
    segment's rows, then the multi-head attention layer) in one launch,
    sgg_gat_layer_fwd: the input as one or two column blocks (x2: [h |
    pool_h] without a concatenation), w in the module's (heads, K, F) layout.
    Backward: sgg_gat_bwd_ex (dWh and the attention parameters' gradients),
    the node transform's input / weight gradients as _XW's backward, then
    sgg_seg_norm_bwd."""

    @staticmethod
    def forward(ctx, x1, x2, w, a_src, a_dst, bias, seg_off, nseg, max_seg, eps, alpha, epi, grad_on=True):
        lib = _lib()
        x1 = _rows(x1, "x1")
        x2 = _rows(x2, "x2") if x2 is not None else None
        n, K1 = x1.shape
        K2 = x2.shape[1] if x2 is not None else 0
        K = K1 + K2
        H, Kw, F = w.shape
        if Kw != K:
            raise ValueError("gat_layer: w is (%d, %d, %d) for %d input features" % (H, Kw, F, K))
        w = _req(w, "w").contiguous()
        a_src, a_dst = a_src.contiguous(), a_dst.contiguous()
        bias = bias.contiguous() if bias is not None else None
        HF = H * F
        dev = x1.device
        # grad_on: the caller's grad mode (forward itself runs with grad off;
        # under no_grad needs_input_grad still reflects the parameters'
        # requires_grad, but no backward can follow: nothing is saved)
        save = grad_on and any(ctx.needs_input_grad[:6])
        y = torch.empty(n, HF, device=dev, dtype=torch.float32)
        hp = torch.empty(n, HF, device=dev, dtype=torch.float32) if epi else None
        xn = rstd = wh = None
        if save:
            xn = torch.empty(n, K, device=dev, dtype=torch.float32)
            rstd = torch.empty(nseg, K, device=dev, dtype=torch.float32)
            wh = torch.empty(n, HF, device=dev, dtype=torch.float32)
        bf16 = _PRECISION == "bf16"

        def launch():
            N.check(lib.sgg_gat_layer_fwd(N.ptr(x1), x1.stride(0), K1, N.ptr(x2), x2.stride(0) if x2 is not None else 0,
                                          K2, N.ptr(w), N.ptr(a_src), N.ptr(a_dst), N.ptr(bias), N.ptr(seg_off), nseg,
                                          n, H, F, float(alpha), float(eps), epi, max_seg, int(bf16), N.ptr(xn),
                                          N.ptr(rstd), N.ptr(wh), N.ptr(hp), N.ptr(y), HF, N.stream_ptr()),
                    "sgg_gat_layer_fwd")
        # norm 5 nK, transform 2 n K HF, attention 2 n^2 HF (n^2 bounded by
        # n * max_seg); x in, W, y (+ hp) out, the saved xn / Wh
        work = (5.0 * n * K + 2.0 * n * K * HF + 2.0 * n * max_seg * HF,
                4.0 * (n * K + n * HF * (2 if epi else 1) + (n * K + n * HF if save else 0)))
        rider = _GRIDER[0]
        shape = (H, F, K1, K2, epi, bf16, float(eps), float(alpha))
        weights = (w, a_src, a_dst, bias)
        lset = N.GatLayerSet(N.ptr(x1), x1.stride(0), K1, N.ptr(x2), x2.stride(0) if x2 is not None else 0, K2,
                             N.ptr(seg_off), nseg, n, max_seg, N.ptr(xn), N.ptr(rstd), N.ptr(wh), N.ptr(hp), N.ptr(y), HF)
        keep = (x1, x2, seg_off, xn, rstd, wh, hp, y)
        name = "sgg::gat_layer_fwd_kernel<%d, %s>" % (8 if max_seg <= 32 else 16 if max_seg <= 64 else 32,
                                                      "true" if bf16 else "false")
        if rider is not None and not save and rider.held is None and n > 0:
            # the discriminator step's batch: held for the generator step's
            rider.hold(lset, keep, weights, shape, launch, (name, (n, K, HF, H, max_seg, save)) + work)
        elif rider is not None and rider.fits(weights, shape) and n > 0:
            pl, (S2, wk2) = rider.carry(lset, keep, max_seg, work)
            pl()
            if timer.active:
                timer.add(name, (S2, K, HF, H, "pair"), wk2[0], wk2[1] + 4.0 * H * K * F, pl)
        else:
            launch()
            if timer.active and n > 0:
                timer.add(name, (n, K, HF, H, max_seg, save), work[0], work[1] + 4.0 * H * K * F, launch)
        ctx.meta = (seg_off, nseg, max_seg, float(alpha), epi, H, F, K1, K2, bias is not None)
        ctx.save_for_backward(xn, rstd, wh, hp, y, w, a_src, a_dst)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib()
        xn, rstd, wh, hp, y, w, a_src, a_dst = ctx.saved_tensors
        seg_off, nseg, max_seg, alpha, epi, H, F, K1, K2, has_bias = ctx.meta
        n = wh.shape[0]
        K, HF = K1 + K2, H * F
        dev = wh.device
        dy = dy.contiguous()
        dWh = torch.empty(n, HF, device=dev, dtype=torch.float32)
        da_s = torch.empty_like(a_src)
        da_d = torch.empty_like(a_dst)
        dbias = torch.empty(F, device=dev, dtype=torch.float32) if has_bias else None
        work = torch.empty(max(16, int(lib.sgg_gat_bwd_ex_work_bytes(nseg, H, F))), device=dev, dtype=torch.uint8)
        _gat_bwd_ex_launch(wh, H, a_src, a_dst, None, seg_off, nseg, n, F, alpha, 1, epi, max_seg, hp, y, dy, dWh,
                           da_s, da_d, dbias, work)
        # the node transform Wh = xn [w_0 | .. | w_{H-1}] (as _XW's backward)
        w_all = w.permute(1, 0, 2).reshape(K, HF)
        dxn = xw_raw(dWh, w_all, None, True, 0, prec="fp32")
        dw = None
        if ctx.needs_input_grad[2]:
            with side(xn, dWh):
                dw_all = xtw(xn, dWh)
            dw = dw_all.view(K, H, F).permute(1, 0, 2)
        dx = torch.empty(n, K, device=dev, dtype=torch.float32)
        N.check(lib.sgg_seg_norm_bwd(N.ptr(xn), K, N.ptr(dxn), K, K, N.ptr(seg_off), nseg, N.ptr(rstd), N.ptr(dx), K,
                                     N.stream_ptr()), "sgg_seg_norm_bwd")
        if timer.active and n > 0:
            timer.add("sgg::seg_norm_bwd_kernel", (n, K), 8.0 * n * K, 4.0 * 4 * n * K,
                      lambda: N.check(lib.sgg_seg_norm_bwd(N.ptr(xn), K, N.ptr(dxn), K, K, N.ptr(seg_off), nseg,
                                                           N.ptr(rstd), N.ptr(dx), K, N.stream_ptr()),
                                      "sgg_seg_norm_bwd"))
        dx1 = dx[:, :K1] if K2 else dx
        dx2 = dx[:, K1:] if K2 else None
        return dx1, dx2, dw, da_s, da_d, dbias, None, None, None, None, None, None, None


class GatLayerRider:
    """gat_layer_pair(): a no-grad batched-GAT layer forward (the
    discriminator step's generator, G.context_pair) is held; the next one of
    the same layer weights and shape (the generator step's) issues both in
    ONE launch (sgg_gat_layer_fwd2).  Layer by layer: the held layer's
    output is written by the carrying launch before the next layer of its
    batch is held.  A held forward nobody carried is issued on exit."""

    def __init__(self):
        self.held = None

    def hold(self, lset, keep, weights, shape, launch, timing):
        self.held = (lset, keep, weights, shape, launch, timing)

    def fits(self, weights, shape):
        if self.held is None:
            return False
        _, _, wh, sh, _, _ = self.held
        return sh == shape and all(a is b for a, b in zip(wh, weights))

    def carry(self, lset, keep, max_seg, work):
        """-> (the paired launch, (rows of both, (flop, bytes) of both))."""
        la, keep_a, (w, a_src, a_dst, bias), (H, F, _, _, epi, bf16, eps, alpha), _, timing = self.held
        self.held = None
        lib = _lib()

        def pl(k=(keep_a, keep, w, a_src, a_dst, bias)):
            N.check(lib.sgg_gat_layer_fwd2(N.ctypes.byref(la), N.ctypes.byref(lset), N.ptr(w), N.ptr(a_src),
                                           N.ptr(a_dst), N.ptr(bias), H, F, alpha, eps, epi, int(bf16),
                                           N.stream_ptr()), "sgg_gat_layer_fwd2")
        return pl, (la.n + lset.n, (timing[2] + work[0], timing[3] + work[1]))

    def flush(self):
        if self.held is not None:
            _, _, (w, _, _, _), (H, F, K1, K2, _, _, _, _), launch, timing = self.held
            self.held = None
            launch()
            if timer.active:
                timer.add(timing[0], timing[1], timing[2], timing[3] + 4.0 * H * (K1 + K2) * F, launch)


_GRIDER = [None]


@contextlib.contextmanager
def gat_layer_pair():
    """Batched-GAT layer forwards of two batches in shared launches (GatLayerRider)."""
    prev = _GRIDER[0]
    r = _GRIDER[0] = GatLayerRider()
    try:
        yield r
    finally:
        _GRIDER[0] = prev
        r.flush()


def gat_layer_ok(K, F, heads, max_seg, epi):
    """sgg_gat_layer_fwd's limits: the LDS plan, F, heads, the epilogue."""
    if not (1 <= F <= 128 and 1 <= heads <= 64 and epi in (0, 1) and 1 <= max_seg <= 128 and K <= 256):
        return False
    return int(_lib().sgg_gat_layer_lds_bytes(K, F, max_seg)) <= 160 * 1024


def gat_layer(x, w, a_src, a_dst, bias, graph, epilogue, eps=1e-5, alpha=0.2):
    """InstanceNorm1d over each segment's rows, then the multi-head attention
    layer (w: (heads, K, F); x: a tensor or (x1, x2) column blocks) in one
    launch (sgg_gat_layer_fwd); the complete graph of each segment."""
    x1, x2 = x if isinstance(x, tuple) else (x, None)
    return _GatLayer.apply(x1, x2, w, a_src, a_dst, bias, graph.seg_off, graph.nseg, graph.max_seg, eps, alpha,
                           epilogue, torch.is_grad_enabled())


def gat_attention(wh, a, alpha, graph, epilogue, heads=1, bias=None):
    """Masked-softmax attention + aggregation + epilogue over `graph`
    (a SegmentGraph).  epilogue: 0 none, 1 ELU, 2 log_softmax(ELU).
    Multi-head: wh is n x heads*F, a is heads x 2F, bias (F) shared by the
    heads and added before the epilogue (sgangat GAT, GAT.py:6-55 text)."""
    return _GatAttn.apply(wh, a, bias, graph.labels, graph.seg_off, graph.nseg, graph.max_seg, alpha, graph.mode,
                          epilogue, heads)


class _GatEnc(torch.autograd.Function):
    """The whole GATEncoder of every scene in one launch (sgg_gatenc_fwd);
    when a gradient is needed the forward also writes each scene's layer
    state (Wh of every layer, activations, group structure) to a saved buffer
    (sgg_gatenc_saved_floats) and the backward is one back-propagation launch
    over it (sgg_gatenc_bwd, no forward recompute) + the scene-ordered slab
    sum of the parameter gradients (sgg_slab_reduce).
    params: [W_h, a_h for each intra head], W_out, a_out (intra), the same for
    the inter GAT, out_embedding weight, bias -- the slab order of sgg.h."""

    @staticmethod
    def forward(ctx, x, labels, scenes, nh, alpha, x2, link, dy_link, save, comp, *params):
        lib = _lib()
        ctx.link = link
        ctx.dy_link = dy_link
        x = _rows(x, "x")
        B = x.shape[0]
        if x2 is not None:
            x2 = _rows(x2, "x2")
            assert x2.shape[0] == B and x.shape[1] + x2.shape[1] == 40, (x.shape, x2.shape)
        y = torch.empty(B, 24, device=x.device, dtype=torch.float32)
        ps = [_req(q, "gat weight").contiguous() for q in params]
        a = _gatenc_args(x, labels, scenes, nh, alpha, ps, x2)
        a.y, a.ldy = N.ptr(y), 24
        saved = None
        if save and any(ctx.needs_input_grad) and GATENC_SAVE:
            nf = int(lib.sgg_gatenc_saved_floats(max(scenes.S, 1), a.np, nh))
            saved = torch.empty(max(nf, 1), device=x.device, dtype=torch.float32)
            a.saved = N.ptr(saved)
        keep = (x, x2, y, labels, scenes, ps, saved)   # the replay closure holds every buffer `a` points to
        flops = _gatenc_flops(scenes, nh)
        nbytes = 4.0 * B * (40 + 1 + 24) + (_gatenc_saved_bytes(B, nh) if saved is not None else 0.0)
        ac = comp.args(nh, alpha, ps, a.np) if comp is not None else None
        if ac is not None:
            # the companion batch's scenes first, then this one's (sgg_gatenc_fwd2)
            keep = keep + comp.keep()
            flops += _gatenc_flops(comp.scenes, nh)
            nbytes += 4.0 * comp.x.shape[0] * (40 + 1 + 24)
            launch = lambda a=a, ac=ac, keep=keep: N.check(
                lib.sgg_gatenc_fwd2(N.ctypes.byref(ac), N.ctypes.byref(a), N.stream_ptr()), "sgg_gatenc_fwd2")
        else:
            if comp is not None:   # (different np: the companion runs alone, first)
                comp.run_alone(nh, alpha, ps)
            launch = lambda a=a, keep=keep: N.check(lib.sgg_gatenc_fwd(N.ctypes.byref(a), N.stream_ptr()),
                                                    "sgg_gatenc_fwd")
        launch()
        if timer.active:
            timer.add("sgg::gatenc_kernel<false>", (scenes.S, B, nh) + ((comp.scenes.S,) if ac is not None else ()),
                      flops, nbytes, launch)
        ctx.meta = (labels, scenes, nh, alpha)
        ctx.save_for_backward(x, x2, saved, *ps)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib()
        x, x2, saved, *ps = ctx.saved_tensors
        labels, scenes, nh, alpha = ctx.meta
        B = x.shape[0]
        pend = ctx.dy_link.take() if ctx.dy_link is not None else None
        copies = 1
        if pend is not None:
            base, copies, cstride, ld = pend
            if dy.data_ptr() == base.data_ptr() and dy.stride(0) == ld:
                dy = base   # rows 0 .. B of copy 0; the kernel adds the other copies
            else:           # autograd summed in another consumer's gradient: add the copies here
                dy = dy + sum(base.view(copies, B, ld)[c, :, :dy.shape[1]] for c in range(1, copies))
                copies = 1
        dy = _rows(dy, "dy")
        P = lib.sgg_gatenc_param_size(nh)
        dx = torch.empty(B, x.shape[1], device=x.device, dtype=torch.float32)
        dx2 = torch.empty(B, x2.shape[1], device=x.device, dtype=torch.float32) if x2 is not None else None
        slab = torch.empty(max(scenes.S, 1), P, device=x.device, dtype=torch.float32)
        a = _gatenc_args(x, labels, scenes, nh, alpha, ps, x2)
        a.dy, a.lddy = N.ptr(dy), dy.stride(0)
        if copies > 1:
            a.dy_copies, a.dy_cstride = copies, cstride
        a.dX, a.lddx = N.ptr(dx), dx.shape[1]
        if dx2 is not None:
            a.dX2, a.lddx2 = N.ptr(dx2), dx2.shape[1]
        a.slab = N.ptr(slab)
        a.saved = N.ptr(saved)
        N.check(lib.sgg_gatenc_bwd(N.ctypes.byref(a), N.stream_ptr()), "sgg_gatenc_bwd")
        if timer.active:
            keep = (x, x2, dy, dx, dx2, slab, labels, scenes, ps, saved)
            timer.add("sgg::gatenc_kernel<true>", (scenes.S, B, nh), 3.0 * _gatenc_flops(scenes, nh),
                      4.0 * (B * (40 + 1 + 24 + 40) + scenes.S * P) + _gatenc_saved_bytes(B, nh),
                      lambda a=a, keep=keep: N.check(lib.sgg_gatenc_bwd(N.ctypes.byref(a), N.stream_ptr()),
                                                     "sgg_gatenc_bwd"))
        flat = torch.empty(P, device=x.device, dtype=torch.float32)
        gf = GradFinish()   # the scene-ordered slab sum (sgg_slab_reduce's order), deferred in the trainer
        gf.rowsum(slab, scenes.S, P, 0, P, flat)
        gf.run()
        grads, o = [], 0
        for q in ps:
            grads.append(flat[o:o + q.numel()].view_as(q))
            o += q.numel()
        if ctx.link is not None and ctx.needs_input_grad[0]:
            ctx.link.put(dx)   # added by the pooling backward (the other consumer of x), which runs next
            dx = None
        return (dx, None, None, None, None, dx2, None, None, None, None) + tuple(grads)


class GatEncCompanion:
    """A second batch through the same GATEncoder forward, without autograd:
    the discriminator step's generator forward, launched together with the
    generator step's context (sgg_gatenc_fwd2; G's weights do not change
    between the two steps, scripts/train.py:395-484).  Its output is `y`
    once the launch carrying it has been issued."""

    def __init__(self, x, labels, scenes, x2=None):
        self.x = _rows(x, "x")
        self.x2 = _rows(x2, "x2") if x2 is not None else None
        self.labels = _req(labels, "labels").contiguous().view(-1)
        self.scenes = scenes
        self.y = None

    def keep(self):
        return (self.x, self.x2, self.labels, self.scenes, self.y)

    def args(self, nh, alpha, ps, np_other):
        """The companion's launch arguments when it can share the launch
        (same np as the batch carrying it), else None."""
        a = _gatenc_args(self.x, self.labels, self.scenes, nh, alpha, ps, self.x2)
        if a.np != np_other:
            return None
        self.y = torch.empty(self.x.shape[0], 24, device=self.x.device, dtype=torch.float32)
        a.y, a.ldy = N.ptr(self.y), 24
        return a

    def run_alone(self, nh, alpha, ps):
        lib = _lib()
        a = _gatenc_args(self.x, self.labels, self.scenes, nh, alpha, ps, self.x2)
        self.y = torch.empty(self.x.shape[0], 24, device=self.x.device, dtype=torch.float32)
        a.y, a.ldy = N.ptr(self.y), 24
        keep = self.keep() + (ps,)
        launch = lambda a=a, keep=keep: N.check(lib.sgg_gatenc_fwd(N.ctypes.byref(a), N.stream_ptr()),
                                                "sgg_gatenc_fwd")
        launch()
        if timer.active:
            timer.add("sgg::gatenc_kernel<false>", (self.scenes.S, self.x.shape[0], nh),
                      _gatenc_flops(self.scenes, nh), 4.0 * self.x.shape[0] * (40 + 1 + 24), launch)


def _gatenc_flops(scenes, nh):
    """GATEncoder forward FLOP (models.py:254-294) per scene of N peds, G
    groups: node transforms 2 N (40*72 nh + 72 nh*16) + 2 G (16*72 nh + 72 nh*16)
    + 2 N 32*24; attention (score + softmax + aggregate) ~ 3 F per edge over
    the N^2 intra pairs (F = 72 nh and 16) and G^2 inter pairs (upper bound N^2)."""
    import numpy as np
    n = np.diff(scenes.host_off).astype(np.float64)
    node = 2 * n * (40 * 72 * nh + 72 * nh * 16) + 2 * n * (16 * 72 * nh + 72 * nh * 16) + 2 * n * 32 * 24
    edge = 2 * n * n * 3 * (72 * nh + 16)
    return float((node + edge).sum())


def _gatenc_saved_bytes(B, nh):
    """Saved forward state per launch (upper bound: as many groups as peds):
    every layer's Wh (72 nh + 16, twice), H1 / G1 (72 nh each), the 16-wide
    activations (yI, preI, gin, preG, gout) and 5 words of group structure."""
    return 4.0 * B * (4 * 72 * nh + 2 * 16 + 5 * 16 + 5)


def _gatenc_args(x, labels, scenes, nh, alpha, ps, x2=None):
    a = N.GatEncArgs()
    a.X, a.ldx = N.ptr(x), x.stride(0)
    if x2 is not None:
        a.X2, a.ldx2, a.kx1 = N.ptr(x2), x2.stride(0), x.shape[1]
    a.labels, a.scene_off = N.ptr(labels), N.ptr(scenes.scene_off)
    a.S, a.np, a.nh, a.alpha = scenes.S, max(scenes.max_n, 1), nh, float(alpha)
    it = iter(ps)
    for h in range(nh):
        a.w.Wi[h], a.w.ai[h] = N.ptr(next(it)), N.ptr(next(it))
    a.w.Wio, a.w.aio = N.ptr(next(it)), N.ptr(next(it))
    for h in range(nh):
        a.w.Wg[h], a.w.ag[h] = N.ptr(next(it)), N.ptr(next(it))
    a.w.Wgo, a.w.ago = N.ptr(next(it)), N.ptr(next(it))
    a.w.Woe, a.w.boe = N.ptr(next(it)), N.ptr(next(it))
    return a


def gat_encoder_fused_ok(scenes, nh, need_grad):
    """The fused GATEncoder path holds a scene in one workgroup's LDS."""
    if not GATENC_FUSED or nh < 1 or nh > N.MAX_HEADS or scenes.max_n > 64:
        return False
    # the backward's plan: with the forward's saved state (compact for
    # 49 .. 64-ped scenes) or, SGG_GATENC_SAVE=0, the recomputing one
    plan = (1 if GATENC_SAVE else 2) if need_grad else 0
    return _lib().sgg_gatenc_lds_bytes(max(scenes.max_n, 1), nh, plan) <= 160 * 1024


def gat_encoder(x, labels, scenes, nh, alpha, params, x2=None, link=None, companion=None):
    """GATEncoder.forward (models.py:254-294) for all scenes: (B, 40) -> (B, 24).
    x2: the input as two column blocks [x | x2] (no concatenation copy).
    link: a GradLink that takes the gradient of x instead of returning it
    (x's other consumer, the pooling net, adds it in its own backward).
    companion: a GatEncCompanion whose batch runs in the same launch."""
    lab = _req(labels, "labels").contiguous().view(-1)
    dl = CopiesLink() if torch.is_grad_enabled() else None
    # the forward state is saved only when a backward can follow (not under
    # no_grad, e.g. the generator inside the discriminator step)
    y = _GatEnc.apply(x, lab, scenes, nh, alpha, x2, link, dl, torch.is_grad_enabled(), companion, *params)
    if dl is not None:
        y._sgg_copies_link = dl   # found by decoder_init (its only consumer in the generator)
    return y


# the one-launch GCNModule (sgg_gcnmod_*); "0" forces the per-op kernels
GCNMOD_FUSED = os.environ.get("SGG_GCNMOD_FUSED", "1") != "0"


class _GcnMod(torch.autograd.Function):
    """The whole GCNModule of every scene in one launch per direction
    (sgg_gcnmod_fwd / _bwd; the backward recomputes the forward in LDS) + the
    slab sum of the parameter gradients (sgg_slab_reduce).
    params: gcn_intra.W.0, gcn_intra.W.1, gcn_inter.W.0, gcn_inter.W.1,
    out_embedding weight, bias -- the slab order of sgg.h."""

    @staticmethod
    def forward(ctx, x, labels, scenes, x2, link, dy_link, bf16, comp, *params):
        lib = _lib()
        ctx.link, ctx.dy_link = link, dy_link
        x = _rows(x, "x")
        B = x.shape[0]
        if x2 is not None:
            x2 = _rows(x2, "x2")
            assert x2.shape[0] == B
        ps = [_req(q, "gcn weight").contiguous() for q in params]
        fe = ps[4].shape[0]
        y = torch.empty(B, fe, device=x.device, dtype=torch.float32)
        a = _gcnmod_args(x, x2, labels, scenes, ps, bf16)
        a.y, a.ldy = N.ptr(y), fe
        keep = (x, x2, y, labels, scenes, ps)
        flops = _gcnmod_flops(scenes, labels, a.fin, fe)
        nbytes = 4.0 * B * (a.fin + 1 + fe)
        ac = comp.args(ps, bf16, fe, a.np, a.fin) if comp is not None else None
        if ac is not None:
            # the companion batch's scenes first, then this one's (sgg_gcnmod_fwd2)
            keep = keep + comp.keep()
            flops += _gcnmod_flops(comp.scenes, comp.labels, a.fin, fe)
            nbytes += 4.0 * comp.x.shape[0] * (a.fin + 1 + fe)
            launch = lambda a=a, ac=ac, keep=keep: N.check(
                lib.sgg_gcnmod_fwd2(N.ctypes.byref(ac), N.ctypes.byref(a), N.stream_ptr()), "sgg_gcnmod_fwd2")
        else:
            if comp is not None:   # (different np: the companion runs alone, first)
                comp.run_alone(ps, bf16, fe)
            launch = lambda a=a, keep=keep: N.check(lib.sgg_gcnmod_fwd(N.ctypes.byref(a), N.stream_ptr()),
                                                    "sgg_gcnmod_fwd")
        launch()
        if timer.active:
            timer.add("sgg::gcnmod_fwd_kernel<%s>" % ("true" if bf16 else "false"),
                      (scenes.S, B, a.fin) + ((comp.scenes.S,) if ac is not None else ()), flops, nbytes, launch)
        ctx.meta = (labels, scenes, bf16)
        ctx.save_for_backward(x, x2, *ps)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib()
        x, x2, *ps = ctx.saved_tensors
        labels, scenes, bf16 = ctx.meta
        B = x.shape[0]
        pend = ctx.dy_link.take() if ctx.dy_link is not None else None
        copies, cstride = 1, 0
        if pend is not None:
            base, copies, cstride, ld = pend
            if dy.data_ptr() == base.data_ptr() and dy.stride(0) == ld:
                dy = base   # rows 0 .. B of copy 0; the kernel adds the other copies
            else:           # autograd summed in another consumer's gradient: add the copies here
                dy = dy + sum(base.view(copies, B, ld)[c, :, :dy.shape[1]] for c in range(1, copies))
                copies = 1
        dy = _rows(dy, "dy")
        a = _gcnmod_args(x, x2, labels, scenes, ps, bf16)
        P = lib.sgg_gcnmod_param_size(a.fin, a.fe)
        rows = lib.sgg_gcnmod_slab_rows(scenes.S)
        dx = torch.empty(B, x.shape[1], device=x.device, dtype=torch.float32)
        dx2 = torch.empty(B, x2.shape[1], device=x.device, dtype=torch.float32) if x2 is not None else None
        slab = torch.empty(rows, P, device=x.device, dtype=torch.float32)
        a.dy, a.lddy = N.ptr(dy), dy.stride(0)
        a.dy_copies, a.dy_cstride = copies, cstride
        a.dX, a.lddx = N.ptr(dx), dx.shape[1]
        if dx2 is not None:
            a.dX2, a.lddx2 = N.ptr(dx2), dx2.shape[1]
        a.slab = N.ptr(slab)
        N.check(lib.sgg_gcnmod_bwd(N.ctypes.byref(a), N.stream_ptr()), "sgg_gcnmod_bwd")
        if timer.active:
            keep = (x, x2, dy, dx, dx2, slab, labels, scenes, ps)
            timer.add("sgg::gcnmod_bwd_kernel<%s>" % ("true" if bf16 else "false"), (scenes.S, B, a.fin),
                      3.0 * _gcnmod_flops(scenes, labels, a.fin, a.fe),
                      4.0 * (B * (a.fin + 1 + a.fe + a.fin) + rows * P),
                      lambda a=a, keep=keep: N.check(lib.sgg_gcnmod_bwd(N.ctypes.byref(a), N.stream_ptr()),
                                                     "sgg_gcnmod_bwd"))
        flat = torch.empty(P, device=x.device, dtype=torch.float32)
        gf = GradFinish()   # the workgroup-ordered slab sum (sgg_slab_reduce's order), deferred in the trainer
        gf.rowsum(slab, rows, P, 0, P, flat)
        gf.run()
        grads, o = [], 0
        for q in ps:
            grads.append(flat[o:o + q.numel()].view_as(q))
            o += q.numel()
        if ctx.link is not None and ctx.needs_input_grad[0]:
            ctx.link.put(dx)   # added by the pooling backward (the other consumer of x), which runs next
            dx = None
        return (dx, None, None, dx2, None, None, None, None) + tuple(grads)


class GcnModCompanion:
    """A second batch through the same GCNModule forward without autograd,
    launched with the batch that carries it (sgg_gcnmod_fwd2); see
    GatEncCompanion.  Its output is `y` once that launch is issued."""

    def __init__(self, x, labels, scenes, x2=None):
        self.x = _rows(x, "x")
        self.x2 = _rows(x2, "x2") if x2 is not None else None
        self.labels = _req(labels, "labels").contiguous().view(-1)
        self.scenes = scenes
        self.y = None

    def keep(self):
        return (self.x, self.x2, self.labels, self.scenes, self.y)

    def _args(self, ps, bf16, fe):
        a = _gcnmod_args(self.x, self.x2, self.labels, self.scenes, ps, bf16)
        self.y = torch.empty(self.x.shape[0], fe, device=self.x.device, dtype=torch.float32)
        a.y, a.ldy = N.ptr(self.y), fe
        return a

    def args(self, ps, bf16, fe, np_other, fin_other):
        a = _gcnmod_args(self.x, self.x2, self.labels, self.scenes, ps, bf16)
        if a.np != np_other or a.fin != fin_other:
            return None
        return self._args(ps, bf16, fe)

    def run_alone(self, ps, bf16, fe):
        lib = _lib()
        a = self._args(ps, bf16, fe)
        keep = self.keep() + (ps,)
        launch = lambda a=a, keep=keep: N.check(lib.sgg_gcnmod_fwd(N.ctypes.byref(a), N.stream_ptr()),
                                                "sgg_gcnmod_fwd")
        launch()
        if timer.active:
            timer.add("sgg::gcnmod_fwd_kernel<%s>" % ("true" if bf16 else "false"),
                      (self.scenes.S, self.x.shape[0], a.fin), _gcnmod_flops(self.scenes, self.labels, a.fin, fe),
                      4.0 * self.x.shape[0] * (a.fin + 1 + fe), launch)


def _gcnmod_flops(scenes, labels, fin, fe):
    """GCNModule forward FLOP (models.py:628-712), minimal formulation: per
    scene of N peds the two intra layers on its G group rows 2 G (fin 72 + 72
    16), the inter layers on one row 2 (16 72 + 72 16), out_embedding 2 N 32 fe.
    G is bounded by N (the label structure is device data; the bound keeps the
    count host-only)."""
    import numpy as np
    n = np.diff(scenes.host_off).astype(np.float64)
    return float((2 * n * (fin * 72 + 72 * 16) + 2 * (16 * 72 + 72 * 16) * (n > 0) + 2 * n * 32 * fe).sum())


def _gcnmod_args(x, x2, labels, scenes, ps, bf16):
    a = N.GcnModArgs()
    a.X, a.ldx = N.ptr(x), x.stride(0)
    fin = x.shape[1]
    if x2 is not None:
        a.X2, a.ldx2, a.kx1 = N.ptr(x2), x2.stride(0), x.shape[1]
        fin += x2.shape[1]
    a.labels, a.scene_off = N.ptr(labels), N.ptr(scenes.scene_off)
    a.S, a.np, a.fin, a.fe, a.bf16 = scenes.S, max(scenes.max_n, 1), fin, ps[4].shape[0], int(bool(bf16))
    a.W0i, a.W1i, a.W0g, a.W1g, a.Woe, a.boe = [N.ptr(q) for q in ps]
    return a


def gcn_module_fused_ok(scenes, fin, fe, params_ok=True):
    """The fused GCNModule path holds a scene's group structure in one wavefront."""
    if not GCNMOD_FUSED or not params_ok or scenes.max_n > 64 or scenes.max_n < 1:
        return False
    return 0 <= _lib().sgg_gcnmod_lds_bytes(scenes.max_n, fin, fe, 1) <= 160 * 1024


def gcn_module(x, labels, scenes, params, x2=None, link=None, companion=None):
    """GCNModule.forward (models.py:628-712) for all scenes: (B, fin) -> (B, fe),
    the input optionally as two column blocks [x | x2]; link as gat_encoder;
    companion: a GcnModCompanion whose batch runs in the same launch."""
    lab = _req(labels, "labels").contiguous().view(-1)
    dl = CopiesLink() if torch.is_grad_enabled() else None
    y = _GcnMod.apply(x, lab, scenes, x2, link, dl, _PRECISION == "bf16", companion, *params)
    if dl is not None:
        y._sgg_copies_link = dl   # found by decoder_init (its only consumer in the generator)
    return y


class _SegNorm(torch.autograd.Function):
    """Per-segment instance normalisation (sgg_seg_norm_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, x, seg_off, nseg, eps):
        lib = _lib()
        x = _rows(x, "x")
        n, F = x.shape
        y = torch.empty(n, F, device=x.device, dtype=torch.float32)
        rstd = torch.empty(nseg, F, device=x.device, dtype=torch.float32)
        N.check(lib.sgg_seg_norm_fwd(N.ptr(x), x.stride(0), F, N.ptr(seg_off), nseg, float(eps), N.ptr(y), F,
                                     N.ptr(rstd), N.stream_ptr()), "sgg_seg_norm_fwd")
        ctx.meta = (seg_off, nseg)
        ctx.save_for_backward(y, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, rstd = ctx.saved_tensors
        seg_off, nseg = ctx.meta
        dy = _rows(dy, "dy")
        n, F = y.shape
        dx = torch.empty(n, F, device=y.device, dtype=torch.float32)
        N.check(_lib().sgg_seg_norm_bwd(N.ptr(y), F, N.ptr(dy), dy.stride(0), F, N.ptr(seg_off), nseg, N.ptr(rstd),
                                        N.ptr(dx), F, N.stream_ptr()), "sgg_seg_norm_bwd")
        return dx, None, None, None


def seg_instance_norm(x, seg_off, nseg, eps=1e-5):
    """InstanceNorm1d (affine=False) of each segment's rows, per feature."""
    return _SegNorm.apply(x, seg_off, nseg, eps)


class SegmentGraph:
    """Node segments for the attention kernel: mode 0 = label mask inside each
    scene (intra-group graph), mode 1 = complete graph (inter-group graph)."""

    def __init__(self, seg_off, nseg, max_seg, mode, labels=None):
        self.seg_off, self.nseg, self.max_seg, self.mode, self.labels = seg_off, nseg, max_seg, mode, labels
        # the kernels size their LDS plan by max_seg (and clamp a larger
        # segment, memory-safe but wrong): SGG_DEBUG=1 checks it against the
        # offsets (one device read per graph)
        if DEBUG and nseg > 0:
            big = int((seg_off[1:nseg + 1] - seg_off[:nseg]).max())
            if big > max_seg:
                raise ValueError("SegmentGraph: a segment of %d nodes exceeds max_seg %d" % (big, max_seg))


# ---------------------------------------------------------------------------
# segmented reduce / gather (group pool, un-pool, GCN aggregation)
# ---------------------------------------------------------------------------
def _seg_reduce_raw(x, seg_of_row, row_scale, range_off, seg_range, nseg_dev, cap, mean):
    x = _rows(x, "x")
    F = x.shape[1]
    out = torch.empty(cap, F, device=x.device, dtype=torch.float32)
    N.check(_lib().sgg_seg_reduce(N.ptr(x), x.stride(0), F, N.ptr(seg_of_row), N.ptr(row_scale), N.ptr(range_off),
                                  N.ptr(seg_range), N.ptr(nseg_dev), cap, int(mean), N.ptr(out), F, N.stream_ptr()),
            "sgg_seg_reduce")
    return out


def _seg_gather_raw(src, seg_of_row, row_scale, nrow_dev, n):
    src = _rows(src, "src")
    F = src.shape[1]
    out = torch.empty(n, F, device=src.device, dtype=torch.float32)
    N.check(_lib().sgg_seg_gather(N.ptr(src), src.stride(0), F, N.ptr(seg_of_row), N.ptr(row_scale),
                                  N.ptr(nrow_dev), n, N.ptr(out), F, N.stream_ptr()), "sgg_seg_gather")
    return out


class _SegReduce(torch.autograd.Function):
    """out[k] = post_k * sum_{rows of k} scale_i x_i ; backward gathers with
    bwd_scale_i = scale_i * post_{seg(i)} (given by the caller)."""

    @staticmethod
    def forward(ctx, x, seg_of_row, row_scale, range_off, seg_range, nseg_dev, cap, mean, bwd_scale, nrow_dev):
        ctx.meta = (seg_of_row, bwd_scale, nrow_dev, x.shape[0])
        return _seg_reduce_raw(x, seg_of_row, row_scale, range_off, seg_range, nseg_dev, cap, mean)

    @staticmethod
    def backward(ctx, dout):
        seg_of_row, bwd_scale, nrow_dev, n = ctx.meta
        dx = _seg_gather_raw(dout, seg_of_row, bwd_scale, nrow_dev, n)
        return dx, None, None, None, None, None, None, None, None, None


class _SegGather(torch.autograd.Function):
    """out[i] = scale_i * src[seg(i)] ; backward = segment sum of scale_i dout_i."""

    @staticmethod
    def forward(ctx, src, seg_of_row, row_scale, nrow_dev, n, range_off, seg_range, nseg_dev):
        ctx.meta = (seg_of_row, row_scale, range_off, seg_range, nseg_dev, src.shape[0])
        return _seg_gather_raw(src, seg_of_row, row_scale, nrow_dev, n)

    @staticmethod
    def backward(ctx, dout):
        seg_of_row, row_scale, range_off, seg_range, nseg_dev, cap = ctx.meta
        dsrc = _seg_reduce_raw(dout, seg_of_row, row_scale, range_off, seg_range, nseg_dev, cap, 0)
        return dsrc, None, None, None, None, None, None, None


def group_mean(x, groups):
    """R @ X with R the row-normalised distinct rows of M_intra
    (models.py:271-280): per-group mean of its members -> (cap, F), rows >= G zero."""
    sc = groups.scenes
    return _SegReduce.apply(x, groups.ped_gid, None, sc.scene_off, groups.group_scene, groups.n_groups_dev,
                            groups.cap, True, groups.ped_inv_size, None)


def group_unpool(gx, groups, scale=True):
    """R^T @ G (models.py:286): ped i receives G[g(i)] / |g(i)| (scale=True) or
    G[g(i)] (scale=False, the broadcast of the GCN's A @ H)."""
    sc = groups.scenes
    rs = groups.ped_inv_size if scale else None
    return _SegGather.apply(gx, groups.ped_gid, rs, None, sc.B, sc.scene_off, groups.group_scene,
                            groups.n_groups_dev)


def scene_mean_over_groups(gx, groups):
    """Complete-graph row-normalised A @ H over each scene's groups
    (models.py:688-694 with A = ones/M): every group row gets the mean of its
    scene's group rows.  Rows >= G stay zero."""
    sc = groups.scenes
    if not hasattr(groups, "_group_inv_ng"):
        ng = (groups.group_off[1:] - groups.group_off[:-1]).float().clamp(min=1)
        groups._group_inv_ng = ng.index_select(0, groups.group_scene.long()).reciprocal()
    sm = _SegReduce.apply(gx, groups.group_scene, None, groups.group_off, None, None, sc.S, True,
                          groups._group_inv_ng, groups.n_groups_dev)
    return _SegGather.apply(sm, groups.group_scene, None, groups.n_groups_dev, groups.cap, groups.group_off, None,
                            None)


# ---------------------------------------------------------------------------
# fused LSTM sequences (encoder / decoder rollout)
# ---------------------------------------------------------------------------
def _tkey(t):
    return (t.data_ptr(), tuple(t.shape), tuple(t.stride()))


class SharedPrefix:
    """The discriminator encoder's observed steps, run once (sgg.h
    SggLstmSeg).  Its input traj_rel = cat(obs_rel, pred) (train.py:404-407,
    456-459) starts with obs_rel for the real and the fake half alike, and
    obs_rel is exactly what the generator's encoder reads first: the
    generator's encoder launch on obs_rel also runs the discriminator's first
    obs_len steps on obs_rel's Bsrc peds (sgg_lstm_fwd_seg2), saving them at
    their positions of the discriminator's (T, copies Bsrc) state layout, and
    the discriminator's forward on traj_rel then runs the remaining steps on
    every column from there (sgg_lstm_fwd_seg, t0 = obs_len).  The backward
    reads the shared steps of column p from column p mod Bsrc
    (sgg_lstm_bwd_shared), so every result is the one of the full sequence.

    Armed by `shared_prefix(...)` around a training step; the two halves only
    meet when the generator's encoder runs on obs_rel itself and the
    discriminator on a traj_cat whose head was obs_rel (same tensor), with the
    discriminator's weights unchanged in between (fold versions)."""

    def __init__(self, lstm, emb, obs_rel, T, copies, fold_specs=None):
        self.lstm, self.emb, self.fold_specs = lstm, emb, fold_specs
        self.obs_rel = obs_rel
        self.key = _tkey(obs_rel)
        self.T_pre, self.Bsrc = int(obs_rel.shape[0]), int(obs_rel.shape[1])
        self.T, self.B = int(T), copies * self.Bsrc
        self.H = int(lstm.weight_hh_l0.shape[1])
        self.ran = self.used = False
        lib = _lib()
        self.ok = (lstm.num_layers == 1 and 0 < self.T_pre < self.T and self.Bsrc > 0
                   and (copies == 1 or self.Bsrc % 16 == 0)
                   and bool(lib.sgg_lstm_u_ok(self.T, self.B, self.H, 0, 1, 16))
                   and bool(lib.sgg_lstm_u_ok(self.T_pre, self.Bsrc, self.H, 0, 1, 16)))

    def arm(self, rel, H_g):
        """The generator encoder's launch on `rel`: the prefix rides along iff
        rel is obs_rel and the kernel pair is one launch (H_g = 32, H = 48)."""
        return self.ok and not self.ran and H_g == 32 and self.H == 48 and _tkey(rel) == self.key

    def arm_dec(self, H_dec):
        """A saving decoder launch before the discriminator's forward (the
        generator step's best / last samples, when no encoder launch of the
        step carried the prefix: G.context_pair formed the context at the
        discriminator step) carries it instead (sgg_lstm_fwd_dec_seg)."""
        return self.ok and not self.ran and H_dec == 32 and self.H == 48

    def segment(self, rel):
        """-> SggLstmSeg of the prefix (state buffers allocated here)."""
        lib = _lib()
        dev = rel.device
        T, B, H = self.T, self.B, self.H
        self.h_all = torch.empty(T + 1, B, H, device=dev, dtype=torch.float32)
        self.c_all = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 1)), device=dev, dtype=torch.float32)
        self.act = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 0)), device=dev, dtype=torch.float32)
        l = self.lstm
        if self.fold_specs is not None:   # all of the module's folds in one launch, as its forward would
            prefold(self.fold_specs())
        self.A, self.bias = fold_fwd(l.weight_ih_l0, self.emb.weight, self.emb.bias, l.bias_ih_l0, l.bias_hh_l0)
        self.Whh = l.weight_hh_l0.contiguous()
        self.fold_ver = _fold_key(*lstm_fold_spec(l, self.emb))[1]
        self.whh_ver = (l.weight_hh_l0._version, _EPOCH.get(l.weight_hh_l0.data_ptr(), 0))
        s = N.LstmSeg(N.ptr(rel), N.ptr(self.A), N.ptr(self.Whh), N.ptr(self.bias), None, None, self.T_pre,
                      self.Bsrc, B, 0, T, self.Bsrc, N.ptr(self.h_all), N.ptr(self.c_all), N.ptr(self.act),
                      None, 0, None, 0, None)
        s._keep = (rel, self.A, self.Whh, self.bias, self.h_all, self.c_all, self.act)   # (check_ownership)
        return s

    def matches(self, rel, W_hh, T, save):
        """The discriminator's forward on `rel` may continue from the prefix."""
        if not (self.ran and not self.used and save and T == self.T and W_hh is self.lstm.weight_hh_l0):
            return False
        if tuple(rel.shape) != (self.T, self.B, 2) or getattr(rel, "_sgg_head_key", None) != self.key:
            return False
        l = self.lstm
        return (_fold_key(*lstm_fold_spec(l, self.emb))[1] == self.fold_ver
                and (l.weight_hh_l0._version, _EPOCH.get(l.weight_hh_l0.data_ptr(), 0)) == self.whh_ver)


_PREFIX = [None]


@contextlib.contextmanager
def shared_prefix(D, obs_rel, T, copies):
    """Arm a SharedPrefix of the discriminator D's encoder for the duration of
    one step (see SharedPrefix); D's forward on traj_cat(obs_rel, ...) of T
    steps and copies x obs_rel's peds may then continue from it."""
    prev = _PREFIX[0]
    enc = D.encoder
    _PREFIX[0] = SharedPrefix(enc.encoder, enc.spatial_embedding, obs_rel, T, copies,
                              getattr(D, "fold_specs", None))
    try:
        yield _PREFIX[0]
    finally:
        _PREFIX[0] = prev


class EncoderRider:
    """encoder_pair(): the block's first encoder launch that carries a shared
    prefix (the discriminator step's generator encoder + the discriminator's
    observed steps) is held instead of launched; the next encoder launch with
    saved states (the generator step's encoder) issues all three segments in
    one launch (sgg_lstm_fwd_seg3).  Nothing may read the held launch's
    outputs before that; a held launch nobody carried is issued on exit."""

    def __init__(self):
        self.held = None     # ([(SggLstmSeg, H), ...], its own launch, its timer entry)
        self.timing = None
        self.done = False

    def hold(self, segs, launch, timing):
        self.held = (segs, launch)
        self.timing = timing

    def carry(self, own, H):
        (a, Ha), (b, Hb) = self.held[0]
        self.held = None
        self.done = True
        lib = _lib()
        return lambda: N.check(lib.sgg_lstm_fwd_seg3(N.ctypes.byref(a), Ha, N.ctypes.byref(b), Hb,
                                                     N.ctypes.byref(own), H, N.stream_ptr()), "sgg_lstm_fwd_seg3")

    def flush(self):
        if self.held is not None:
            segs, launch = self.held
            self.held = None
            launch()
            if timer.active:
                name, key, fl, nb = self.timing
                timer.add(name, key, fl, nb, launch)
        self.done = True


_RIDER = [None]


class DecoderRider:
    """decoder_pair(): the block's first no-grad decoder launch with a fused
    start that writes the discriminator input (the discriminator step's
    generator decoder, four-wave or -- at >= 4096 peds -- batch-MFMA
    family) is held; the next no-grad
    decoder launch of the same weights on the batch-MFMA family (the
    generator step's best-of-k rollout) issues both (sgg_lstm_fwd_dec2).
    Nothing may read the held launch's outputs before that -- its
    discriminator input is taken by traj_cat without a launch; a held launch
    nobody carried is issued on exit."""

    def __init__(self):
        self.held = None
        self.timing = None
        self.done = False

    def hold(self, di, rel_out, to, B, H, T, weights, keep, launch):
        self.held = (di, rel_out, to, B, H, T, weights, keep, launch)

    def fits(self, H, T, *weights):
        if self.held is None:
            return False
        _, _, _, _, Hh, Th, wh, _, _ = self.held
        return Hh == H and Th == T and all(a is b for a, b in zip(wh, weights))

    def carry(self, di, A, Whh, bias, Wp, bp, T, B, H, rel_out, keep):
        di2, rel2, to2, B2, _, _, _, keep2, _ = self.held
        self.held = None
        self.done = True
        lib = _lib()
        return lambda k=(keep, keep2): lib.sgg_lstm_fwd_dec2(
            N.ctypes.byref(di), N.ctypes.byref(di2), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(Wp), N.ptr(bp), T, B,
            B2, H, N.ptr(rel_out), N.ptr(rel2), N.ctypes.byref(to2) if to2 is not None else None, N.stream_ptr())

    def flush(self):
        if self.held is not None:
            launch = self.held[-1]
            self.held = None
            launch()
            if timer.active:
                timer.add(*self.timing, launch)
        self.done = True


_DRIDER = [None]


@contextlib.contextmanager
def decoder_pair():
    """The discriminator step's decoder launch rides with the rollout's
    (DecoderRider)."""
    prev = _DRIDER[0]
    r = _DRIDER[0] = DecoderRider()
    try:
        yield r
    finally:
        _DRIDER[0] = prev
        r.flush()


@contextlib.contextmanager
def encoder_pair():
    """The first prefix-carrying encoder launch inside the block rides with
    the next saved-state encoder launch (EncoderRider)."""
    prev = _RIDER[0]
    r = _RIDER[0] = EncoderRider()
    try:
        yield r
    finally:
        _RIDER[0] = prev
        r.flush()


class _LSTMSeq(torch.autograd.Function):
    """Fused LSTM sequence on the raw parameters of Linear(2, E) + LSTM(E, H)
    (+ hidden2pos for the decoder): the embedding fold is one launch
    (sgg_fold_fwd), the T-step recurrence another; the backward returns
    the raw parameters' gradients (sgg_fold_bwd maps dA, dbias back).  Where
    the library accumulates the weight gradients inside the backward kernel
    (sgg_lstm_wpart_rows > 0) the gate gradients never reach HBM: one slab
    row per workgroup, summed by sgg_slab_reduce; otherwise dG is written
    and reduced by sgg_xtw."""

    @staticmethod
    def forward(ctx, rel, W_ih, W_hh, b_ih, b_hh, We, be, h0, c0, Wp, bp, decoder, T, save, u=None, slink=None):
        lib = _lib()
        ctx.t_stop = int(getattr(rel, "_sgg_grad_from", 0))
        pfx = _PREFIX[0]
        rel_in = rel
        rel = _req(rel, "rel").contiguous()
        H = W_hh.shape[1]
        B = rel.shape[-2]
        dev = rel.device
        A, bias = fold_fwd(W_ih, We, be, b_ih, b_hh)
        # the discriminator's shared observed-steps prefix: this launch carries
        # it (generator encoder), or this sequence continues from it
        carry = pfx is not None and not decoder and h0 is None and c0 is None and pfx.arm(rel_in, H)
        cont = (pfx is not None and not decoder and h0 is None and c0 is None and not carry
                and pfx.matches(rel_in, W_hh, T, save))
        ctx.t_sh, ctx.bsrc = (pfx.T_pre, pfx.Bsrc) if cont and pfx.Bsrc < B else (0, 0)
        if cont:
            h_all, c_all, act = pfx.h_all, pfx.c_all, pfx.act
            pfx.used = True
        else:
            h_all = torch.empty(T + 1, B, H, device=dev, dtype=torch.float32)
            # saved states in the layout of the kernel family (H, B) picks
            c_all = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 1)), device=dev, dtype=torch.float32)
            act = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 0)), device=dev, dtype=torch.float32) \
                if save else None
        rel_out = torch.empty(T, B, 2, device=dev, dtype=torch.float32) if decoder else None
        # a no-grad decoder rollout whose final state nobody reads
        # (final_state_unused(): the best-of-k samples) writes rel_out only
        no_final = (_NO_FINAL[0] and decoder and not save and not cont and h0 is not None and c0 is None
                    and getattr(h0, "_sgg_dinit", None) is not None)
        if no_final:
            h_all = c_all = None
        Whh = W_hh.contiguous()
        h0c = h0.contiguous() if h0 is not None else None
        c0c = c0.contiguous() if c0 is not None else None
        Wpc = Wp.contiguous() if Wp is not None else None
        U = None
        Wu = cu = None
        if u is not None:
            # the pooling MLP's U = h_T Wu^T + cu from the kernel's epilogue
            Wu, cu = u
            Wu = _rows(Wu, "Wu")
            cu = cu.contiguous()
            U = torch.empty(B, Wu.shape[0], device=dev, dtype=torch.float32)

        def seg(t0, Tn, Bsrc):
            s = N.LstmSeg(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(h0c), N.ptr(c0c), Tn, B, B, t0, T,
                          Bsrc, N.ptr(h_all), N.ptr(c_all), N.ptr(act), N.ptr(Wu),
                          Wu.stride(0) if Wu is not None else 0, N.ptr(cu), Wu.shape[0] if Wu is not None else 0,
                          N.ptr(U))
            # the descriptor owns what it points to (a re-issue outlives this frame)
            s._keep = (rel, A, Whh, bias, h0c, c0c, h_all, c_all, act, Wu, cu, U)
            return s
        pfx_seg = pfx.segment(rel) if carry else None
        if carry:
            pfx.ran = True
        kname = None
        launch_done = False
        dheld = dcarried = False
        if carry:
            ga, gb = seg(0, T, B), pfx_seg
            kname = "sgg::lstm_mw_fwd2_kernel<32, %s, 48, true>" % ("true" if save else "false")

            def launch():
                N.check(lib.sgg_lstm_fwd_seg2(N.ctypes.byref(ga), H, N.ctypes.byref(gb), pfx.H, N.stream_ptr()),
                        "sgg_lstm_fwd_seg2")
        elif cont:
            gs = seg(pfx.T_pre, T - pfx.T_pre, pfx.Bsrc)

            def launch():
                N.check(lib.sgg_lstm_fwd_seg(N.ctypes.byref(gs), H, N.stream_ptr()), "sgg_lstm_fwd_seg")
        elif u is not None:
            def launch():
                N.check(lib.sgg_lstm_fwd_u(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(h0c), N.ptr(c0c), T,
                                           B, H, N.ptr(h_all), N.ptr(c_all), N.ptr(act), N.ptr(Wu), Wu.stride(0),
                                           N.ptr(cu), Wu.shape[0], N.ptr(U), N.stream_ptr()), "sgg_lstm_fwd_u")
        else:
            def launch():
                N.check(lib.sgg_lstm_fwd(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(h0c), N.ptr(c0c),
                                         N.ptr(Wpc), N.ptr(bp), T, B, H, int(decoder), N.ptr(h_all), N.ptr(c_all),
                                         N.ptr(act), N.ptr(rel_out), N.stream_ptr()), "sgg_lstm_fwd")
            dinit = getattr(h0, "_sgg_dinit", None) if (decoder and h0 is not None and c0 is None) else None
            if dinit is not None:
                # the decoder's h0 / rel0 built in the kernel's prologue (one
                # launch fewer); where no kernel takes it, materialise them first
                di, dkeep, materialize = dinit
                ta = _TRAJ[0]
                to = ta.desc(T, B) if ta is not None else None
                # the closure holds every buffer the descriptors and the
                # arguments point to (the bench's timer re-issues it later)
                fkeep = (dkeep, A, Whh, bias, Wpc, bp, h_all, c_all, act, rel_out, rel,
                         (ta.out, ta.start, ta.head, ta.b, ta.pos0) if to is not None else None)
                dcarry = pfx is not None and save and pfx.arm_dec(H)
                if dcarry:
                    # the discriminator's observed-steps prefix of this step rides along
                    pseg = pfx.segment(pfx.obs_rel)
                    pfx.ran = True
                    kname = "sgg::lstm_mw_fwd2d_kernel<32, true, 48, true>"
                    fused = lambda k=fkeep, to=to, pseg=pseg, Hp=pfx.H: lib.sgg_lstm_fwd_dec_seg(
                        N.ctypes.byref(di), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(Wpc), N.ptr(bp), T, B, H,
                        N.ptr(h_all), N.ptr(c_all), N.ptr(act), N.ptr(rel_out), N.ptr(rel),
                        N.ctypes.byref(to) if to is not None else None, N.ctypes.byref(pseg), Hp, N.stream_ptr())
                else:
                    fused = lambda k=fkeep, to=to: lib.sgg_lstm_fwd_dec(
                        N.ctypes.byref(di), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(Wpc), N.ptr(bp), T, B, H,
                        N.ptr(h_all), N.ptr(c_all), N.ptr(act), N.ptr(rel_out), N.ptr(rel) if save else None,
                        N.ctypes.byref(to) if to is not None else None, N.stream_ptr())
                drider = _DRIDER[0]
                if drider is not None and not save and not dcarry and h_all is None and Wpc is not None:
                    mfma = "mfma" in lib.sgg_lstm_kernel_name(H, B, 1, 0, 0).decode()
                    if to is not None and drider.held is None and not drider.done:
                        # the discriminator step's decoder (either family): held for the rollout's launch
                        dheld = True
                    elif mfma and drider.fits(H, T, A, Whh, bias, Wpc, bp):
                        fused = drider.carry(di, A, Whh, bias, Wpc, bp, T, B, H, rel_out, fkeep)
                        dcarried = True
                if dheld:
                    rc = 0
                else:
                    rc = fused()
                if rc != 0 and (dcarry or dcarried):   # (owed to a later consumer: no fallback)
                    N.check(rc, "sgg_lstm_fwd_dec_seg" if dcarry else "sgg_lstm_fwd_dec2")
                if rc != 0 and to is not None:   # no family writes the discriminator input here
                    to = None
                    fused = functools.partial(fused, to=None)
                    rc = fused()
                if rc == 0:
                    if to is not None:   # traj_cat on these columns finds them written
                        ta.filled = (rel_out.data_ptr() + 8 * ta.col0, rel_out.stride(0))
                    launch = lambda: N.check(fused(), "sgg_lstm_fwd_dec")
                    if dheld:
                        drider.hold(di, rel_out, to, B, H, T, (A, Whh, bias, Wpc, bp), fkeep, launch)
                else:
                    if h_all is None:   # (sgg_lstm_fwd writes the final state)
                        h_all = torch.empty(T + 1, B, H, device=dev, dtype=torch.float32)
                        c_all = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 1)), device=dev,
                                            dtype=torch.float32)
                    h0d, r0d = h0.detach(), rel
                    materialize(h0d, r0d)
                    plain = launch
                    launch = lambda: (materialize(h0d, r0d), plain())
                    plain()
                launch_done = True
            else:
                launch_done = False
        # an encoder pair (encoder_pair(): G.context_pair): the first encoder
        # launch of the block is held, the next one carries it
        rider = _RIDER[0]
        held = carried = False
        if rider is not None and not launch_done and not decoder:
            if carry and rider.held is None and not rider.done:
                held = True
            elif (u is not None and save and not carry and not cont and rider.held is not None
                  and len(rider.held[0]) == 2):
                own = seg(0, T, B)
                launch = rider.carry(own, H)
                carried = True
        if not launch_done and not held:
            launch()
        if timer.active or held or dheld:
            # per ped-step: gates 2 4H (H + 3) FLOP + ~12 H cell / activation; bytes: inputs, saved states
            Ts = T - pfx.T_pre if cont else T    # the steps this launch runs
            fl = Ts * B * (8.0 * H * (H + 3) + 12.0 * H) + (2.0 * B * H * U.shape[1] if U is not None else 0.0)
            nb = 4.0 * (Ts * B * 2 + ((act.numel() + c_all.numel()) * Ts / T + (Ts + 1) * B * H if save else
                                      (0 if no_final else 2 * B * H))
                        + 4 * H * (H + 3) + (T * B * 2 if decoder else 0) + (U.numel() if U is not None else 0))
            if carry or (decoder and kname is not None):   # + the prefix: T_pre steps of Bsrc peds, states saved
                Hp, Tp, Bp = pfx.H, pfx.T_pre, pfx.Bsrc
                fl += Tp * Bp * (8.0 * Hp * (Hp + 3) + 12.0 * Hp)
                nb += 4.0 * (Tp * Bp * 2 + Tp * Bp * 5 * Hp + (Tp + 1) * Bp * Hp + 4 * Hp * (Hp + 3))
            name = kname or lib.sgg_lstm_kernel_name(H, B, int(decoder), int(save), 0).decode()
            key = (Ts, B, int(decoder), int(save)) + ((pfx.T_pre,) if (carry or cont) else ())
            if dheld:
                drider.timing = (name, key, fl, nb)
            elif dcarried:
                hname, hkey, hfl, hnb = drider.timing
                timer.add(name, key + hkey, fl + hfl, nb + hnb, launch)
            elif held:
                rider.hold([(ga, H), (gb, pfx.H)], launch, (name, key, fl, nb))
            elif carried:
                hname, hkey, hfl, hnb = rider.timing
                timer.add("sgg::lstm_mw_fwd3_kernel<32, false, 48, true, 32, true>", hkey + key, hfl + fl, hnb + nb,
                          launch)
            else:
                timer.add(name, key, fl, nb, launch)
        ctx.meta = (decoder, T, B, H, h0 is not None)
        ctx.slink = slink
        ctx.set_materialize_grads(False)   # unused outputs (the decoder's h_last) get None, not a zero fill
        if save:
            ctx.save_for_backward(rel, W_ih, We, be, A, Whh, Wpc, h_all, c_all, act, rel_out)
        h_last = h_all[T] if h_all is not None else rel.new_empty(0, H)
        if U is not None:
            ctx.mark_non_differentiable(U)   # its gradient is the pooling backward's business (dh = dU Wu)
            return h_last, U
        if decoder:
            return h_last, rel_out
        return h_last, h_last.new_empty(0)

    @staticmethod
    def backward(ctx, dh_last, drel_out):
        lib = _lib()
        decoder, T, B, H, has_h0 = ctx.meta
        rel, W_ih, We, be, A, Whh, Wp, h_all, c_all, act, rel_out = ctx.saved_tensors
        dev = rel.device
        need = ctx.needs_input_grad
        wgrad = any(need[1:7])
        rows = int(lib.sgg_lstm_wpart_rows(H, B))
        G4 = 4 * H
        P = G4 * H + G4 + 2 * G4
        # the decoder's rows also carry [dWp (2 x H) | dbp (2)] (lstm_mw.hip)
        PW = P + (2 * H + 2 if decoder else 0)
        wpart = torch.empty(rows, PW, device=dev, dtype=torch.float32) if (wgrad and rows > 0) else None
        dG = torch.empty(T, B, G4, device=dev, dtype=torch.float32) if rows == 0 else None
        drel_in = torch.empty(T, B, 2, device=dev, dtype=torch.float32)
        dh0 = torch.empty(B, H, device=dev, dtype=torch.float32) if has_h0 else None
        drel_tot = torch.empty(T, B, 2, device=dev, dtype=torch.float32) if decoder else None
        split = None
        if decoder and ctx.slink is not None:
            pend = ctx.slink.take()
            if pend is not None:
                ga, gb, bsplit, ph = pend
                if drel_out is None or drel_out.data_ptr() != ph.data_ptr():
                    raise N.NativeError("decoder backward: the split rollout output has another consumer")
                if rows > 0 and wgrad:   # the four-wave kernel reads the two blocks in place
                    split = (ga, gb, bsplit)
                else:
                    drel_out = torch.cat([ga, gb], 1)
        if decoder:
            if split is not None:
                dout = split[0]
            else:
                dout = drel_out.contiguous() if drel_out is not None else torch.zeros(T, B, 2, device=dev)
            dhl = None  # the decoder's final state feeds nothing in the generator (models.py:925)
        else:
            dout = None
            dhl = dh_last.contiguous() if dh_last is not None else None
        tail = (not decoder and not wgrad and not has_h0 and rows > 0 and 0 < ctx.t_stop < T)
        if ctx.t_sh > 0:   # steps < t_sh saved once for column p mod bsrc (SharedPrefix)
            def launch():
                N.check(lib.sgg_lstm_bwd_shared(N.ptr(A), N.ptr(Whh), N.ptr(h_all), N.ptr(c_all), N.ptr(act),
                                                N.ptr(rel), N.ptr(dhl), T, B, H, ctx.t_sh, ctx.bsrc, N.ptr(drel_in),
                                                N.ptr(wpart), N.stream_ptr()), "sgg_lstm_bwd_shared")
        elif tail:   # input gradients of steps t_stop .. T-1 only (the rest are not wanted)
            def launch():
                N.check(lib.sgg_lstm_bwd_tail(N.ptr(A), N.ptr(Whh), N.ptr(h_all), N.ptr(c_all), N.ptr(act),
                                              N.ptr(rel), N.ptr(dhl), T, B, H, ctx.t_stop, N.ptr(drel_in),
                                              N.stream_ptr()), "sgg_lstm_bwd_tail")
        elif split is not None:
            def launch():
                N.check(lib.sgg_lstm_bwd_split(N.ptr(A), N.ptr(Whh), N.ptr(Wp), N.ptr(h_all), N.ptr(c_all),
                                               N.ptr(act), N.ptr(rel), N.ptr(rel_out), N.ptr(split[0]),
                                               N.ptr(split[1]), split[2], T, B, H, N.ptr(dh0), N.ptr(drel_in),
                                               N.ptr(drel_tot), N.ptr(wpart), N.stream_ptr()), "sgg_lstm_bwd_split")
        else:
            def launch():
                N.check(lib.sgg_lstm_bwd(N.ptr(A), N.ptr(Whh), N.ptr(Wp), N.ptr(h_all), N.ptr(c_all), N.ptr(act),
                                         N.ptr(rel), N.ptr(rel_out), N.ptr(dhl), N.ptr(dout), T, B, H, int(decoder),
                                         N.ptr(dG), N.ptr(dh0), N.ptr(drel_in), N.ptr(drel_tot), N.ptr(wpart),
                                         N.stream_ptr()), "sgg_lstm_bwd")
        launch()
        if timer.active:
            # per ped-step: dh = W^T dG 2 4H H, cell gradient ~30 H, in-kernel
            # weight gradient 2 4H (H + 3); bytes: saved states read, input
            # gradients written, dG or the slab written
            fl = T * B * (8.0 * H * H + 30.0 * H + (8.0 * H * (H + 3) if wpart is not None else 0.0))
            nb = 4.0 * (act.numel() + c_all.numel() + T * B * 2 + (B * H if has_h0 else 0)
                        + ((T * B * (H + 2) + wpart.numel()) if wpart is not None else 0)
                        + (dG.numel() if dG is not None else 0) + (T * B * 4 if decoder else 0))
            timer.add(lib.sgg_lstm_kernel_name(H, B, int(decoder), int(wpart is not None), 1).decode(),
                      (T, B, int(decoder), int(wpart is not None)), fl, nb, launch)
        dW_ih = dW_hh = db_ih = db_hh = dWe = dbe = dWp = dbp = None
        side_ctx = side(wpart, dG, h_all, rel, rel_out, drel_tot, W_ih, We, be) if wgrad or decoder \
            else contextlib.nullcontext()
        with side_ctx:
            need_p = decoder and (need[9] or need[10])
            if wpart is not None:
                # one launch: dW_hh, dbias (slab [dW_hh | dbias | dA] row sums),
                # the fold backward of (dA, dbias) -> dW_ih, dWe, dbe (+ the b_hh
                # copy), and the decoder's dWp, dbp from their split partials
                gf = GradFinish()
                if need_p:   # accumulated by the kernel into the slab rows
                    dWp = torch.empty(2, H, device=dev, dtype=torch.float32)
                    dbp = torch.empty(2, device=dev, dtype=torch.float32)
                    gf.rowsum(wpart, rows, PW, P, 2 * H, dWp)
                    gf.rowsum(wpart, rows, PW, P + 2 * H, 2, dbp)
                dW_hh = torch.empty(G4, H, device=dev, dtype=torch.float32)
                db_ih = torch.empty(G4, device=dev, dtype=torch.float32)
                db_hh = torch.empty(G4, device=dev, dtype=torch.float32)
                gf.rowsum(wpart, rows, PW, 0, G4 * H, dW_hh)
                gf.rowsum(wpart, rows, PW, G4 * H, G4, db_ih)
                dW_ih, dWe, dbe = gf.fold(W_ih, We, be, wpart, rows, PW, G4 * H + G4, wpart, rows, PW, G4 * H,
                                          dbias_copy=db_hh)
                gf.run()
            else:
                if wgrad:
                    dW_ih, dW_hh, db_ih, db_hh, dWe, dbe = _lstm_wgrads(lib, wpart, rows, P, G4, H, T, B, dG, h_all,
                                                                        rel, rel_out, decoder, W_ih, We, be, dev)
                if need_p:
                    dr = drel_tot.view(T * B, 2)
                    dWp, dbp = xtw(h_all[1:].reshape(T * B, H), dr, colsum=True, trans_c=True)
        if decoder:
            drel = drel_in[0]
        else:
            drel = drel_in
        return (drel, dW_ih, dW_hh, db_ih, db_hh, dWe, dbe, (dh0 if has_h0 else None), None, dWp, dbp,
                None, None, None, None, None)


def _lstm_wgrads(lib, wpart, rows, P, G4, H, T, B, dG, h_all, rel, rel_out, decoder, W_ih, We, be, dev):
    """dW_ih, dW_hh, db_ih, db_hh, dWe, dbe of an LSTM sequence from the
    kernel's slab (or from dG for the families that write it)."""
    if wpart is not None:
        flat = torch.empty(P, device=dev, dtype=torch.float32)     # [dW_hh | dbias | dA]
        N.check(lib.sgg_slab_reduce(N.ptr(wpart), rows, P, N.ptr(flat), N.stream_ptr()), "sgg_slab_reduce")
        dW_hh = flat[:G4 * H].view(G4, H)
        dbias = flat[G4 * H:G4 * H + G4]
        dA = flat[G4 * H + G4:].view(G4, 2)
    else:
        dGf = dG.view(T * B, G4)
        # dW_hh = dG^T h_{t-1} (4H x H, transposed reduction), dbias = sum dG
        dW_hh, dbias = xtw(h_all[:T].reshape(T * B, H), dGf, colsum=True, trans_c=True)
        rel_in = torch.cat([rel.unsqueeze(0), rel_out[:-1]], 0) if decoder else rel
        dA = xtw(rel_in.reshape(T * B, 2), dGf, trans_c=True)                   # 4H x 2
    db_hh = torch.empty_like(dbias)          # two leaves: no shared gradient storage
    dW_ih, dWe, dbe = fold_bwd(W_ih, We, be, dA, dbias, dbias_copy=db_hh)
    return dW_ih, dW_hh, dbias, db_hh, dWe, dbe


def lstm_u_ok(T, B, H, save, NU):
    return bool(_lib().sgg_lstm_u_ok(T, B, H, 0, int(save), NU))


def lstm_sequence(rel, lstm, emb, h0=None, c0=None, proj=None, decoder=False, T=None, proj_u=None):
    """Fused Linear(2, E) + 1-layer LSTM over T steps (see sgg_lstm_fwd);
    `proj` is the decoder's hidden2pos.  Returns (h_last, rel_out).
    proj_u = (Wu, cu) (encoder): returns (h_last, U) with U = h_last Wu^T + cu
    from the kernel's epilogue, or (h_last, None) where the kernel family
    the sizes select has no such epilogue."""
    T = T if T is not None else rel.shape[0]
    W_ih, W_hh, b_ih, b_hh = lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0
    Wp = proj.weight if proj is not None else None
    bp = proj.bias if proj is not None else None
    ins = (rel, W_ih, W_hh, b_ih, b_hh, emb.weight, emb.bias, h0, Wp, bp)
    save = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ins)
    if c0 is not None and c0.requires_grad and torch.is_grad_enabled():
        raise NotImplementedError("gradient w.r.t. the initial cell state")
    if proj_u is not None:
        if decoder or not lstm_u_ok(T, rel.shape[-2], W_hh.shape[1], save, proj_u[0].shape[0]):
            h_last, _ = _LSTMSeq.apply(rel, W_ih, W_hh, b_ih, b_hh, emb.weight, emb.bias, h0, c0, Wp, bp,
                                       bool(decoder), T, save)
            return h_last, None
        return _LSTMSeq.apply(rel, W_ih, W_hh, b_ih, b_hh, emb.weight, emb.bias, h0, c0, Wp, bp, bool(decoder), T,
                              save, proj_u)
    slink = Handoff() if (decoder and save) else None
    h_last, rel_out = _LSTMSeq.apply(rel, W_ih, W_hh, b_ih, b_hh, emb.weight, emb.bias, h0, c0, Wp, bp,
                                     bool(decoder), T, save, None, slink)
    if slink is not None:
        rel_out._sgg_split_link = slink   # split2 of the best-of-k copies hands both gradient blocks over
    return h_last, (rel_out if decoder else None)


# ---------------------------------------------------------------------------
# adversarial loss (losses.py:5-49) -> sgg_bce_fwd / sgg_bce_bwd
# ---------------------------------------------------------------------------
class _Bce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ya, yb, split, w, nvalid):
        ctx.shape = x.shape
        ctx.bce_link = getattr(x, "_sgg_bce_link", None)
        if ctx.bce_link is not None:   # the held head forward + its backward, one launch
            ctx.bce_link.run_fused(ya, yb, split, w, nvalid)
        x = _req(x, "scores").contiguous().view(-1)
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        if _loss_deferrable("bce"):   # formed with the weight gradients
            _queue_loss("bce", N.BceJob(N.ptr(x), x.numel(), split, N.ptr(ya), N.ptr(yb), float(w), N.ptr(loss), None,
                                        None, N.ptr(nvalid)), (x, ya, yb, loss, nvalid), (loss,))
        else:
            N.check(_lib().sgg_bce_fwd(N.ptr(x), x.numel(), split, N.ptr(ya), N.ptr(yb), float(w), N.ptr(loss),
                                       None, None, N.ptr(nvalid), N.stream_ptr()), "sgg_bce_fwd")
        ctx.meta = (split, float(w), nvalid)
        ctx.save_for_backward(x, ya, yb)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, ya, yb = ctx.saved_tensors
        split, w, nvalid = ctx.meta
        if ctx.bce_link is not None:   # the head backward forms the scores' gradient (BceLink)
            ph = torch.empty(ctx.shape, device=x.device, dtype=torch.float32)
            ctx.bce_link.put(g, ya, yb, split, w, ph, nvalid)
            return ph, None, None, None, None, None
        g = g.contiguous()
        dx = torch.empty_like(x)
        N.check(_lib().sgg_bce_bwd(N.ptr(x), x.numel(), split, N.ptr(ya), N.ptr(yb), w, N.ptr(g), N.ptr(dx),
                                   N.ptr(nvalid), N.stream_ptr()), "sgg_bce_bwd")
        return dx.view(ctx.shape), None, None, None, None, None


_CONST = {}
_CONST_VALUES = (0.0, 1.0)


def const(v, device):
    """A cached device scalar for the FIXED constants 0 and 1 (no fill launch
    per use; created on first use, outside graph capture: the trainers warm up
    before capturing).  Any other value gets a fresh tensor: caching per value
    would keep one device scalar per random label-smoothing draw forever."""
    v = float(v)
    if v not in _CONST_VALUES:
        return torch.full((), v, device=device, dtype=torch.float32)
    key = (str(device), v)
    t = _CONST.get(key)
    if t is None:
        t = _CONST[key] = torch.full((), v, device=device, dtype=torch.float32)
    return t


def _scalar_dev(y, device):
    if torch.is_tensor(y):
        return y.to(device=device, dtype=torch.float32).reshape(())
    return const(y, device)


class _BceTotal(torch.autograd.Function):
    """(bce, bce + addend) in one launch: the generator's adversarial term
    and its total loss with the L2 term (no separate add launch)."""

    @staticmethod
    def forward(ctx, x, ya, yb, split, w, addend, nvalid):
        ctx.shape = x.shape
        ctx.bce_link = getattr(x, "_sgg_bce_link", None)
        if ctx.bce_link is not None:   # the held head forward + its backward, one launch
            ctx.bce_link.run_fused(ya, yb, split, w, nvalid)
        x = _req(x, "scores").contiguous().view(-1)
        addend = _req(addend, "addend").reshape(())
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        total = torch.empty((), device=x.device, dtype=torch.float32)
        if _loss_deferrable("bce"):   # after a queued L2 addend, in the same workgroup
            _queue_loss("bce", N.BceJob(N.ptr(x), x.numel(), split, N.ptr(ya), N.ptr(yb), float(w), N.ptr(loss),
                                        N.ptr(addend), N.ptr(total), N.ptr(nvalid)),
                        (x, ya, yb, loss, addend, total, nvalid), (loss, total))
        else:
            if _loss_pending(addend):   # (a queued L2 value exists only after the backward)
                raise N.NativeError("bce total: the addend is a queued loss value")
            N.check(_lib().sgg_bce_fwd(N.ptr(x), x.numel(), split, N.ptr(ya), N.ptr(yb), float(w), N.ptr(loss),
                                       N.ptr(addend), N.ptr(total), N.ptr(nvalid), N.stream_ptr()), "sgg_bce_fwd")
        ctx.meta = (split, float(w), nvalid)
        ctx.save_for_backward(x, ya, yb)
        ctx.set_materialize_grads(False)
        return loss, total

    @staticmethod
    def backward(ctx, g_loss, g_total):
        x, ya, yb = ctx.saved_tensors
        split, w, nvalid = ctx.meta
        g = g_total if g_loss is None else (g_loss if g_total is None else g_loss + g_total)
        dx = None
        if g is not None and ctx.needs_input_grad[0] and ctx.bce_link is not None:
            dx = torch.empty(ctx.shape, device=x.device, dtype=torch.float32)   # the head backward forms it
            ctx.bce_link.put(g, ya, yb, split, w, dx, nvalid)
        elif g is not None and ctx.needs_input_grad[0]:
            g = g.contiguous()
            dx = torch.empty_like(x)
            N.check(_lib().sgg_bce_bwd(N.ptr(x), x.numel(), split, N.ptr(ya), N.ptr(yb), w, N.ptr(g), N.ptr(dx),
                                       N.ptr(nvalid), N.stream_ptr()), "sgg_bce_bwd")
            dx = dx.view(ctx.shape)
        return dx, None, None, None, None, g_total, None


def bce_pair_total(scores, split, y_a, y_b, w, addend, nvalid=None):
    """(bce_pair(...), bce_pair(...) + addend) from one launch; the backward of
    the total passes its gradient to the addend unchanged."""
    dev = scores.device
    return _BceTotal.apply(scores, _scalar_dev(y_a, dev), _scalar_dev(y_b, dev), int(split), w, addend, nvalid)


def bce_pair(scores, split, y_a, y_b, w=1.0, nvalid=None):
    """w * (bce_loss(scores[:split], y_a) + bce_loss(scores[split:], y_b)) with
    scalar targets (python floats or device scalars); split = len -> one term.
    nvalid (device int32 scalar, a padded batch's PaddedScenes.nvalid): only
    the first *nvalid scores of each range are real."""
    dev = scores.device
    return _Bce.apply(scores, _scalar_dev(y_a, dev), _scalar_dev(y_b, dev), int(split), w, nvalid)


# ---------------------------------------------------------------------------
# training-step glue (glue.hip)
# ---------------------------------------------------------------------------
# the discriminator input written by the decoder launch that produces its
# generated half (SggTrajOut, sgg_lstm_fwd_dec): armed by traj_ahead around
# the decoder's call, taken by traj_cat when its arguments are the armed ones
# (one launch fewer per step); "0" disables
TRAJ_AHEAD = os.environ.get("SGG_TRAJ_AHEAD", "1") != "0"
_TRAJ = [None]


def _pairs_rows(t):
    """t is rows of (x, y) pairs with a free step stride (sgg_traj_cat's layout)."""
    return t is not None and t.dim() == 3 and t.stride(1) == 2 and t.stride(2) == 1


class TrajAhead:
    """traj_cat(head, <decoder output columns col0 .. col0 + ncol>, b, pos0),
    allocated before the decoder runs (see traj_ahead)."""

    def __init__(self, head, T1, ncol, col0=0, b=None, pos0=None):
        self.head, self.b, self.pos0 = head, b, pos0
        self.T0, self.T1, self.ncol, self.col0 = int(head.shape[0]), int(T1), int(ncol), int(col0)
        NB = 2 * self.ncol if b is not None else self.ncol
        dev = head.device
        self.out = torch.empty(self.T0 + self.T1, NB, 2, device=dev, dtype=torch.float32)
        self.start = torch.empty(1, NB, 2, device=dev, dtype=torch.float32) if pos0 is not None else None
        self.filled = None   # (address, step stride) of the decoder output columns it holds
        self.ok = (head.is_cuda and head.dtype == torch.float32 and _pairs_rows(head)
                   and tuple(head.shape[1:]) == (self.ncol, 2)
                   and (b is None or (b.dtype == torch.float32 and _pairs_rows(b)
                                      and tuple(b.shape) == (self.T1, self.ncol, 2)))
                   and (pos0 is None or (pos0.dtype == torch.float32 and pos0.is_contiguous()
                                         and pos0.numel() == 2 * self.ncol)))

    def desc(self, T, B):
        """-> N.TrajOut for a decoder launch of T steps x B columns, or None."""
        if not self.ok or self.filled is not None or T != self.T1 or self.col0 + self.ncol > B:
            return None
        b, p0 = self.b, self.pos0
        t = N.TrajOut(N.ptr(self.out), self.out.shape[1], self.T0, self.col0, self.ncol, N.ptr(self.head),
                      self.head.stride(0), N.ptr(b), b.stride(0) if b is not None else 0, N.ptr(p0),
                      N.ptr(self.start))
        t._keep = (self.out, self.head, b, p0, self.start)   # (check_ownership)
        return t

    def taken_by(self, head, a, b, pos0):
        key = lambda t: None if t is None else _tkey(t)
        if (self.filled is None or key(head) != key(self.head) or key(b) != key(self.b)
                or key(pos0) != key(self.pos0)):
            return False
        return (tuple(a.shape) == (self.T1, self.ncol, 2) and (a.data_ptr(), a.stride(0)) == self.filled
                and a.stride(1) == 2 and a.stride(2) == 1)


@contextlib.contextmanager
def traj_ahead(head, T1, ncol, col0=0, b=None, pos0=None):
    """Arm a TrajAhead for the decoder launch inside the block; traj_cat(head,
    a, b, pos0) on that launch's output columns then returns it unlaunched."""
    prev = _TRAJ[0]
    _TRAJ[0] = TrajAhead(head, T1, ncol, col0, b, pos0) if TRAJ_AHEAD else None
    try:
        yield _TRAJ[0]
    finally:
        _TRAJ[0] = prev


class _TrajCat(torch.autograd.Function):
    """cat over time of head (T0 x B x 2, repeated for both halves when b is
    given) and a | b (T1 x B x 2 each, side by side); a may be a batch slice
    of a wider tensor.  Gradient flows to `a` only (the generator output).
    With pos0 (B x 2) the same launch also returns the start positions of
    every column (pos0 repeated for both halves: the discriminator's traj[0])."""

    @staticmethod
    def forward(ctx, head, a, b, pos0):
        T0, B = head.shape[0], head.shape[1]
        head_key = _tkey(head)
        T1 = a.shape[0]
        ta = _TRAJ[0]
        if ta is not None and ta.taken_by(head, a, b, pos0):   # written by the decoder launch
            out, start = ta.out, ta.start
            ta.filled = ()   # taken once
            ctx.dims = (T0, B)
            if not head.requires_grad:
                out._sgg_grad_from = T0
            out._sgg_head_key = head_key
            if start is None:
                return out
            ctx.mark_non_differentiable(start)
            return out, start
        # rows of (x, y) pairs with a free step stride; anything else (e.g. the
        # permuted views seq_collate yields, trajectories_GCN.py:33) is copied
        fix = lambda t: t if t is None or (t.stride(1) == 2 and t.stride(2) == 1) else t.contiguous()
        head, a, b = fix(head), fix(a), fix(b)
        for t, nm in ((head, "head"), (a, "a")) + (((b, "b"),) if b is not None else ()):
            _req(t, nm)
            assert t.shape[1:] == (B, 2) and t.stride(1) == 2 and t.stride(2) == 1, (nm, t.shape, t.stride())
        NB = 2 * B if b is not None else B
        out = torch.empty(T0 + T1, NB, 2, device=a.device, dtype=torch.float32)
        start = None
        if pos0 is not None:
            pos0 = _req(pos0, "pos0").reshape(B, 2).contiguous()
            start = torch.empty(1, NB, 2, device=a.device, dtype=torch.float32)
        N.check(_lib().sgg_traj_cat(N.ptr(head), head.stride(0), T0, N.ptr(a), a.stride(0), N.ptr(b),
                                    b.stride(0) if b is not None else 0, T1, B, N.ptr(out), N.ptr(pos0),
                                    N.ptr(start), N.stream_ptr()), "sgg_traj_cat")
        ctx.dims = (T0, B)
        if not head.requires_grad:
            out._sgg_grad_from = T0   # the consumer's backward may skip the head steps' input gradients
        out._sgg_head_key = head_key   # every column starts with `head` (SharedPrefix)
        if start is None:
            return out
        ctx.mark_non_differentiable(start)
        return out, start

    @staticmethod
    def backward(ctx, dout, *_):
        T0, B = ctx.dims
        return None, dout[T0:, :B], None, None


def traj_cat(head, a, b=None, pos0=None):
    """-> traj_rel, or (traj_rel, start) when pos0 is given."""
    return _TrajCat.apply(head, a, b, pos0)


_NO_FINAL = [False]


@contextlib.contextmanager
def final_state_unused():
    """The no-grad decoder rollouts inside skip their final-state stores
    (h_T, c_T): the caller reads the predicted displacements only."""
    prev = _NO_FINAL[0]
    _NO_FINAL[0] = True
    try:
        yield
    finally:
        _NO_FINAL[0] = prev


# the decoder's h0 / rel0 built in the decoder LSTM's prologue
# (sgg_lstm_fwd_dec) instead of by a sgg_decoder_init launch; "0" disables
DEC_INIT_FUSED = os.environ.get("SGG_DEC_INIT_FUSED", "1") != "0"


class _DecoderInit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cvec, z, best, first_k, copies, scenes, last_rel, lazy):
        ctx.dy_link = getattr(cvec, "_sgg_copies_link", None)
        cvec = _rows(cvec, "ctx")
        B, Dc = cvec.shape
        nz = z.shape[-1] if z is not None else 0
        h0 = torch.empty(copies * B, Dc + nz, device=cvec.device, dtype=torch.float32)
        rel0 = torch.empty(copies * B, 2, device=cvec.device, dtype=torch.float32)
        zc = _req(z, "z").contiguous() if z is not None else None
        last = _req(last_rel, "last_rel").contiguous()
        # the kernels index z[k][s] and last_rel[p] without bounds: shapes checked here
        if B != scenes.B or tuple(last.shape) != (B, 2):
            raise ValueError("decoder_init: context rows %d / last_rel %s vs the scenes' %d peds"
                             % (B, tuple(last.shape), scenes.B))
        if zc is not None:
            need_k = first_k + copies - (1 if best is not None else 0)
            if zc.dim() != 3 or zc.shape[1] != scenes.S or zc.shape[0] < max(need_k, 1):
                raise ValueError("decoder_init: noise %s must be (>= %d draws, %d scenes, nz)"
                                 % (tuple(zc.shape), need_k, scenes.S))
            if best is not None and (best.numel() != scenes.S or best.dtype != torch.int64):
                raise ValueError("decoder_init: best must be the %d scenes' int64 sample indices" % scenes.S)
        ps = scenes.ped_scene_i32()
        args = (N.ptr(cvec), cvec.stride(0), Dc, N.ptr(zc), nz, N.ptr(best), int(first_k), int(copies), N.ptr(ps),
                scenes.S, B, N.ptr(last), N.ptr(h0), N.ptr(rel0))

        # every buffer the launches read, held by storage only (no autograd
        # graph kept alive, no reference back to h0: a cycle through h0 would
        # keep this iteration's graph alive into the next one)
        keep = tuple(t.detach() for t in (cvec, zc, best, ps, last) if t is not None)

        def materialize(h0_buf, rel0_buf, keep=keep):
            N.check(_lib().sgg_decoder_init(*args[:-2], N.ptr(h0_buf), N.ptr(rel0_buf), N.stream_ptr()),
                    "sgg_decoder_init")
        if lazy:
            # h0 / rel0 stay unwritten: the decoder LSTM (their one consumer)
            # builds them in its prologue from this descriptor, or calls
            # materialize(h0, rel0) first where its kernel family cannot
            di = N.DecInit(N.ptr(cvec), cvec.stride(0), Dc, N.ptr(zc), nz, N.ptr(best), int(first_k), N.ptr(ps),
                           scenes.S, B, N.ptr(last))
            di._keep = keep   # (check_ownership: the descriptor owns what it points to)
            h0._sgg_dinit = (di, keep, materialize)
        else:
            materialize(h0, rel0)
        ctx.dims = (copies, B, Dc)
        ctx.mark_non_differentiable(rel0)
        ctx.set_materialize_grads(False)   # no zero-filled gradient for rel0
        return h0, rel0

    @staticmethod
    def backward(ctx, dh0, _drel0):
        copies, B, Dc = ctx.dims
        d = dh0.view(copies, B, -1)[:, :, :Dc]
        if copies > 1 and ctx.dy_link is not None and dh0.is_contiguous():
            # the GAT encoder's backward sums the copies while loading dy
            ctx.dy_link.put(dh0, copies, B * dh0.shape[1], dh0.shape[1])
            return d[0], None, None, None, None, None, None, None
        return (d[0] if copies == 1 else d.sum(0)), None, None, None, None, None, None, None


def decoder_init(cvec, z, best, first_k, copies, scenes, last_rel, lazy=False):
    """add_noise (global mix) + the decoder's first input for `copies` samples:
    z is (K, S, nz); copy r takes sample best[s] (r = 0, when best is given)
    or first_k + r (- 1 with best).  -> (h0 (copies*B, Dc+nz), rel0).
    lazy: h0 / rel0 are left for the decoder LSTM (lstm_sequence) to build in
    its prologue -- pass them to nothing else."""
    return _DecoderInit.apply(cvec, z, best, first_k, copies, scenes, last_rel, bool(lazy and DEC_INIT_FUSED))


def l2_select(pred, gt, mask, scenes, k):
    """best-of-k sample per scene (train.py:443-464) -> int64 (S,)."""
    best = torch.empty(scenes.S, device=pred.device, dtype=torch.int64)
    pred = _req(pred, "pred").contiguous()
    N.check(_lib().sgg_l2_select(N.ptr(pred), N.ptr(_req(gt, "gt").contiguous()), N.ptr(mask), mask.stride(0),
                                 N.ptr(scenes.scene_off), scenes.S, gt.shape[0], scenes.B, int(k), N.ptr(best),
                                 N.stream_ptr()), "sgg_l2_select")
    return best


class _L2Loss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, mask, scenes, w):
        _req(pred, "pred")
        assert pred.stride(1) == 2 and pred.stride(2) == 1 and mask.stride(1) == 1
        gt = _req(gt, "gt").contiguous()
        T, B = gt.shape[0], gt.shape[1]
        loss = torch.empty((), device=pred.device, dtype=torch.float32)
        term = None
        if _loss_deferrable("l2"):
            # the backward forms the mask sums and the per-scene terms itself
            # (sgg_l2_loss_bwd_scenes); the value is their sum, formed with the
            # weight gradients (SggL2Job) -- inside the trainer's step, whose
            # backward always runs
            term = torch.empty(max(scenes.S, 1), device=pred.device, dtype=torch.float32)
            _queue_loss("l2", N.L2Job(N.ptr(term), scenes.S, N.ptr(loss)), (term, loss), (loss,))
            msum = None
        else:
            msum = torch.empty(scenes.S, device=pred.device, dtype=torch.float32)
            term = torch.empty(scenes.S, device=pred.device, dtype=torch.float32)
            N.check(_lib().sgg_l2_loss_fwd(N.ptr(pred), pred.stride(0), N.ptr(gt), N.ptr(mask), mask.stride(0),
                                           N.ptr(scenes.scene_off), scenes.S, T, B, float(w), N.ptr(loss),
                                           N.ptr(msum), N.ptr(term), N.stream_ptr()), "sgg_l2_loss_fwd")
        ctx.save_for_backward(pred, gt, mask, msum, term)
        ctx.meta = (scenes, float(w))
        return loss

    @staticmethod
    def backward(ctx, g):
        pred, gt, mask, msum, term = ctx.saved_tensors
        scenes, w = ctx.meta
        T, B = gt.shape[0], gt.shape[1]
        dpred = torch.empty(T, B, 2, device=pred.device, dtype=torch.float32)
        if msum is None:   # (the value was queued: the scenes' mask sums are formed here)
            N.check(_lib().sgg_l2_loss_bwd_scenes(N.ptr(pred), pred.stride(0), N.ptr(gt), N.ptr(mask), mask.stride(0),
                                                  N.ptr(scenes.scene_off), scenes.S, T, B, w, N.ptr(g.contiguous()),
                                                  N.ptr(dpred), 2 * B, N.ptr(term), N.stream_ptr()),
                    "sgg_l2_loss_bwd_scenes")
        else:
            N.check(_lib().sgg_l2_loss_bwd(N.ptr(pred), pred.stride(0), N.ptr(gt), N.ptr(mask), mask.stride(0),
                                           N.ptr(scenes.ped_scene_i32()), N.ptr(msum), T, B, w,
                                           N.ptr(g.contiguous()), N.ptr(dpred), 2 * B, N.stream_ptr()),
                    "sgg_l2_loss_bwd")
        return dpred, None, None, None, None


def l2_loss(pred, gt, mask, scenes, w=1.0):
    """sum_s w * l2_loss(pred, gt, mask, 'raw') summed over the peds of s /
    sum(mask of s) (train.py:459-464 for the selected sample)."""
    return _L2Loss.apply(pred, gt, mask, scenes, w)


class _Split2(torch.autograd.Function):
    """(x[:, :B], x[:, B:]) with ONE concatenating launch in the backward
    (autograd's slice backward would zero-fill and copy per slice)."""

    @staticmethod
    def forward(ctx, x, B):
        ctx.meta = (x.shape, B)
        ctx.slink = getattr(x, "_sgg_split_link", None)
        return x[:, :B], x[:, B:]

    @staticmethod
    def backward(ctx, ga, gb):
        shape, B = ctx.meta
        if ctx.slink is not None and ga is not None and gb is not None:
            # x is the decoder rollout's output: its backward reads the two
            # blocks in place (sgg_lstm_bwd_split), no concatenation
            ph = torch.empty(shape, device=ga.device, dtype=ga.dtype)
            ctx.slink.put(ga.contiguous(), gb.contiguous(), B, ph)
            return ph, None
        if ga is None:
            ga = torch.zeros(shape[0], B, *shape[2:], device=gb.device, dtype=gb.dtype)
        if gb is None:
            gb = torch.zeros(shape[0], shape[1] - B, *shape[2:], device=ga.device, dtype=ga.dtype)
        return torch.cat([ga, gb], 1), None


def split2(x, B):
    return _Split2.apply(x, B)
