"""Micro-benchmarks of single kernels on the training shapes (HIP events on
the launch stream).  Usage: python tools/bench_kernels.py [pool|big|lstm]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sgan import _native as N  # noqa: E402
from sgan import kernels as K  # noqa: E402
from sgan.scene import SceneIndex  # noqa: E402


def run(S, n, hd, bn, gpws=(0,), reps=20):
    torch.manual_seed(0)
    dev = "cuda"
    B = S * n
    sc = SceneIndex(np.arange(0, B + 1, n), dev)
    h = torch.randn(B, hd, device=dev)
    pos = torch.rand(B, 2, device=dev) * 15
    W1h = torch.randn(512, hd, device=dev) * 0.1
    A = torch.randn(512, 2, device=dev) * 0.3
    c = torch.randn(512, device=dev) * 0.1
    W2 = torch.randn(bn, 512, device=dev) * 0.05
    b2 = torch.randn(bn, device=dev) * 0.1
    U = K.xw_raw(h, W1h, c, trans_w=True)
    W2c = W2.contiguous()
    lib = N.load()
    flops = float(S * n * n) * 512 * (4 + 2 * bn)
    for gpw in gpws:
        sc.POOL_MAX_GPW = gpw
        sc.__dict__.pop("_pool_plans", None)
        chunks, nchunks, max_rows, g = sc.pool_plan(bn)
        out = torch.empty(B, bn, device=dev)
        am = torch.empty(B, bn, device=dev, dtype=torch.int32)
        call = lambda: N.check(lib.sgg_pool_fwd(N.ptr(U), N.ptr(pos), N.ptr(A), N.ptr(W2c), N.ptr(b2),
                                                N.ptr(sc.scene_off), N.ptr(chunks), nchunks, max_rows, g, B, bn,
                                                sc.max_n, N.ptr(out), N.ptr(am), None, N.stream_ptr()), "pool")
        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print("pool_fwd S=%5d n=%2d bn=%2d chunks=%5d gpw=%d  %8.1f us  %6.1f TF/s" % (
            S, n, bn, nchunks, g, us, flops / us / 1e6), flush=True)


def lstm(B, T, H, decoder, reps=10, save=False):
    torch.manual_seed(0)
    dev = "cuda"
    lib = N.load()
    rel = torch.randn(1 if decoder else T, B, 2, device=dev).squeeze(0) * 0.3
    A = torch.randn(4 * H, 2, device=dev) * 0.3
    Whh = torch.randn(4 * H, H, device=dev) * 0.2
    bias = torch.randn(4 * H, device=dev) * 0.1
    h0 = torch.randn(B, H, device=dev) * 0.5
    Wp = torch.randn(2, H, device=dev) * 0.2
    bp = torch.randn(2, device=dev) * 0.1
    h_all = torch.empty(T + 1, B, H, device=dev)
    c_all = torch.empty(T + 1, B, H, device=dev)
    act = torch.empty(T, B, 4 * H, device=dev)
    rel_out = torch.empty(T, B, 2, device=dev)
    call = lambda: N.check(lib.sgg_lstm_fwd(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(h0), None,
                                            N.ptr(Wp), N.ptr(bp), T, B, H, int(decoder), N.ptr(h_all), N.ptr(c_all),
                                            N.ptr(act) if save else None, N.ptr(rel_out), N.stream_ptr()), "lstm")
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    flops = 2.0 * T * B * 4 * H * (H + 2)
    print("lstm_fwd B=%6d T=%2d H=%2d dec=%d save=%d  %8.1f us  %6.1f TF/s (gate GEMM)" % (
        B, T, H, decoder, save, us, flops / us / 1e6), flush=True)


def lstm_ab(B, T, H, decoder, reps=20):
    """sgg_lstm_fwd / _bwd with the four-wave MFMA form (SGG_LSTM_MW=all)
    against the previous forms (SGG_LSTM_MW=0)."""
    torch.manual_seed(0)
    dev = "cuda"
    lib = N.load()
    rel = torch.randn(1 if decoder else T, B, 2, device=dev).squeeze(0) * 0.3
    A = torch.randn(4 * H, 2, device=dev) * 0.3
    Whh = torch.randn(4 * H, H, device=dev) * 0.2
    bias = torch.randn(4 * H, device=dev) * 0.1
    h0 = torch.randn(B, H, device=dev) * 0.5
    Wp = torch.randn(2, H, device=dev) * 0.2
    bp = torch.randn(2, device=dev) * 0.1
    h_all = torch.empty(T + 1, B, H, device=dev)
    c_all = torch.empty(T + 1, B, H, device=dev)
    act = torch.empty(T, B, 4 * H, device=dev)
    rel_out = torch.empty(T, B, 2, device=dev)
    dG = torch.empty(T, B, 4 * H, device=dev)
    drel_in = torch.empty(T, B, 2, device=dev)
    drel_tot = torch.empty(T, B, 2, device=dev)
    dh0 = torch.empty(B, H, device=dev)
    dout = torch.randn(T, B, 2, device=dev)
    dhl = torch.randn(B, H, device=dev)
    fwd = lambda: N.check(lib.sgg_lstm_fwd(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(h0), None, N.ptr(Wp),
                                           N.ptr(bp), T, B, H, int(decoder), N.ptr(h_all), N.ptr(c_all), N.ptr(act),
                                           N.ptr(rel_out), N.stream_ptr()), "lstm_fwd")
    bwd = lambda: N.check(lib.sgg_lstm_bwd(N.ptr(A), N.ptr(Whh), N.ptr(Wp), N.ptr(c_all), N.ptr(act),
                                           None if decoder else N.ptr(dhl), N.ptr(dout) if decoder else None, T, B,
                                           H, int(decoder), N.ptr(dG), N.ptr(dh0), N.ptr(drel_in),
                                           N.ptr(drel_tot), N.stream_ptr()), "lstm_bwd")
    res = []
    for mode in ("0", "all"):
        os.environ["SGG_LSTM_MW"] = mode
        res.append((timeit(fwd, reps), timeit(bwd, reps)))
    os.environ.pop("SGG_LSTM_MW")
    print("lstm B=%5d T=%2d H=%2d dec=%d  old fwd %6.1f bwd %6.1f us | mw fwd %6.1f bwd %6.1f us" % (
        B, T, H, decoder, res[0][0], res[0][1], res[1][0], res[1][1]), flush=True)


def lstm_bwd_w(B, T, H, reps=20):
    """The four-wave backward with in-kernel weight gradients (the
    discriminator encoder's launch: sgg_lstm_bwd with wpart), after a saving
    forward; HIP events around back-to-back launches."""
    torch.manual_seed(0)
    dev = "cuda"
    lib = N.load()
    rel = torch.randn(T, B, 2, device=dev) * 0.3
    A = torch.randn(4 * H, 2, device=dev) * 0.3
    Whh = torch.randn(4 * H, H, device=dev) * 0.2
    bias = torch.randn(4 * H, device=dev) * 0.1
    h0 = torch.randn(B, H, device=dev) * 0.5
    h_all = torch.empty(T + 1, B, H, device=dev)
    c_all = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 1)), device=dev)
    act = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 0)), device=dev)
    drel_in = torch.empty(T, B, 2, device=dev)
    dhl = torch.randn(B, H, device=dev)
    rows = int(lib.sgg_lstm_wpart_rows(H, B))
    wpart = torch.empty(rows * (4 * H * H + 12 * H + 2 * H + 2), device=dev)
    N.check(lib.sgg_lstm_fwd(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(h0), None, None, None, T, B, H, 0,
                             N.ptr(h_all), N.ptr(c_all), N.ptr(act), None, N.stream_ptr()), "lstm_fwd")
    bwd = lambda: N.check(lib.sgg_lstm_bwd(N.ptr(A), N.ptr(Whh), None, N.ptr(h_all), N.ptr(c_all), N.ptr(act),
                                           N.ptr(rel), None, N.ptr(dhl), None, T, B, H, 0, None, None,
                                           N.ptr(drel_in), None, N.ptr(wpart), N.stream_ptr()), "lstm_bwd")
    us = timeit(bwd, reps)
    print("lstm_bwd+w B=%5d T=%2d H=%2d  %7.2f us  (%s)" % (B, T, H, us, os.environ.get("SGG_LIB", "tree")),
          flush=True)


def timeit(call, reps=20):
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def dense():
    """sgg_xw / sgg_xtw on the training step's shapes."""
    dev = "cuda"
    for (M, Kd, Nn, tw) in [(2560, 40, 72, False), (2560, 72, 16, False), (1280, 32, 512, True), (2560, 64, 48, True),
                            (25600, 40, 72, False), (1280, 512, 32, False), (2560, 48, 64, True)]:
        x = torch.randn(M, Kd, device=dev)
        w = torch.randn(Nn, Kd, device=dev) if tw else torch.randn(Kd, Nn, device=dev)
        us = timeit(lambda: K.xw_raw(x, w, None, trans_w=tw))
        print("xw   M=%6d K=%4d N=%4d trans=%d  %7.1f us" % (M, Kd, Nn, tw, us), flush=True)
    for (R, M, Nn) in [(1280, 32, 512), (2560, 48, 512), (51200, 48, 192), (20480, 32, 128), (2560, 40, 72),
                       (1280, 64, 1), (2560, 2, 192)]:
        X = torch.randn(R, M, device=dev)
        Y = torch.randn(R, Nn, device=dev)
        us = timeit(lambda: K.xtw(X, Y, colsum=True))
        print("xtw  R=%6d M=%4d N=%4d  %7.1f us  (splits %d)" % (R, M, Nn, us, N.load().sgg_xtw_splits(R, M, Nn)),
              flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "pool"
    if what == "big":     # one config (profiling)
        run(1280, 20, 32, 8, reps=5)
        sys.exit(0)
    if what == "dense":
        dense()
        sys.exit(0)
    if what == "ab":
        for args in ((2560, 20, 48, False), (1280, 20, 48, False), (1280, 8, 32, False), (2560, 12, 32, True),
                     (1280, 12, 32, True)):
            lstm_ab(*args)
        dense()
        sys.exit(0)
    if what == "roll":    # the no-grad decoder rollout against its batch (waves per SIMD)
        for B in (4096, 8192, 16384, 20480, 25600, 32768, 49152):
            lstm(B, 12, 32, True, reps=20)
        sys.exit(0)
    if what == "rollb":   # the rollout over batch sizes: waves per SIMD 0.5 .. 2
        for B in (8192, 16384, 20480, 25600, 26880, 32768):
            lstm(B, 12, 32, True, reps=10)
        sys.exit(0)
    if what == "roll2":   # one / two waves per SIMD (counter runs: tools/gpu_sq_rollwaves.sh)
        for B in (16384, 25600):
            lstm(B, 12, 32, True, reps=5)
        sys.exit(0)
    if what == "mwf":     # the four-wave forward of the discriminator's encoder (H 48), saving / not
        for B in (2560, 1280):
            for save in (True, False):
                lstm(B, 12, 48, False, save=save)
        sys.exit(0)
    if what == "dpool":   # the discriminator's pooling (bn 48) at the training shapes
        for (S, n) in ((128, 20), (64, 20), (256, 20), (128, 57)):
            run(S, n, 48, 48)
        sys.exit(0)
    if what == "lbwd":    # the discriminator encoder's backward with weight gradients
        for (B, T, H) in ((2560, 20, 48), (1280, 20, 48), (2560, 12, 32), (8192, 20, 48)):
            lstm_bwd_w(B, T, H)
        sys.exit(0)
    if what == "lstm":
        for B in (1280, 2560, 4096, 25600):
            for save in (False, True):
                lstm(B, 8, 32, False, save=save)
                lstm(B, 12, 32, True, save=save)
        for B in (1280, 2560):
            lstm(B, 20, 48, False, save=True)
        sys.exit(0)
    run(1280, 20, 32, 8, gpws=(0, 1, 2, 4))
    run(64, 20, 32, 8, gpws=(0, 1, 2))
    run(128, 20, 32, 8)
    run(128, 20, 48, 48)
    run(256, 57, 32, 8)
