"""Four-wave LSTM encoder forward at the discriminator's shape (H 48, 2560
peds) for T = 1 .. 20, with / without the U epilogue and saved states:
per-launch time of 50 back-to-back launches (HIP events) -> fixed cost and
per-step cost.  usage: python tools/lstm_seg_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))

import torch  # noqa: E402

from sgan import _native as N  # noqa: E402


def main():
    lib = N.load()
    dev = "cuda"
    torch.manual_seed(0)
    H, B, NU = 48, int(os.environ.get("PROBE_B", 2560)), 512
    f = lambda *s: (torch.randn(*s, device=dev) * 0.2).contiguous()
    A, Whh, bias, Wu, cu = f(4 * H, 2), f(4 * H, H), f(4 * H), f(NU, H), f(NU)
    for T in (1, 2, 4, 8, 12, 20):
        rel = f(T, B, 2)
        h_all = torch.empty(T + 1, B, H, device=dev)
        c_all = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 1)), device=dev)
        act = torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, 0)), device=dev)
        U = torch.empty(B, NU, device=dev)
        res = []
        for save, withu in ((True, True), (True, False), (False, False)):
            def go():
                if withu:
                    N.check(lib.sgg_lstm_fwd_u(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, T, B, H,
                                               N.ptr(h_all), N.ptr(c_all), N.ptr(act if save else None), N.ptr(Wu),
                                               H, N.ptr(cu), NU, N.ptr(U), N.stream_ptr()), "u")
                else:
                    N.check(lib.sgg_lstm_fwd(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, None, None,
                                             T, B, H, 0, N.ptr(h_all), N.ptr(c_all), N.ptr(act if save else None),
                                             None, N.stream_ptr()), "f")
            for _ in range(5):
                go()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                go()
            e1.record()
            e1.synchronize()
            res.append(e0.elapsed_time(e1) / 50 * 1e3)
        print("T=%2d  save+U %.1f us  save %.1f us  nosave %.1f us" % (T, *res), flush=True)


if __name__ == "__main__":
    main()
