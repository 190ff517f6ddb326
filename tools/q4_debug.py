"""Per-step comparison of the four-peds encoder backward against the
four-wave one on the same saved states (diagnostics for lstm_q4.hip).
usage: python tools/q4_debug.py [H B T]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "group-gan-gcn-gat_amd"))
from sgan import _native as N  # noqa: E402


def main():
    H, B, T = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (48, 64, 6)
    lib = N.load()
    dev = "cuda"
    torch.manual_seed(1)
    f = lambda *s, sc=0.3: (torch.randn(*s, device=dev) * sc).contiguous()
    A, Whh, bias = f(4 * H, 2), f(4 * H, H, sc=0.2), f(4 * H)
    rel, h0, c0, dh_last = f(T, B, 2), f(B, H), f(B, H), f(B, H)
    sf = lambda w: torch.zeros(int(lib.sgg_lstm_state_floats(T, B, H, w)), device=dev)
    lib.sgg_lstm_q4_enable(0)
    h_all, c_all, act = torch.zeros(T + 1, B, H, device=dev), sf(1), sf(0)
    sg = N.LstmSeg(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), N.ptr(h0), N.ptr(c0), T, B, B, 0, T, B,
                   N.ptr(h_all), N.ptr(c_all), N.ptr(act), None, 0, None, 0, None)
    N.check(lib.sgg_lstm_fwd_seg(N.ctypes.byref(sg), H, N.stream_ptr()), "seg")
    out = []
    for q4 in (1, 0):
        for dl in (dh_last, None):
            lib.sgg_lstm_q4_enable(q4)
            drel, dh0 = torch.zeros(T, B, 2, device=dev), torch.zeros(B, H, device=dev)
            N.check(lib.sgg_lstm_bwd(N.ptr(A), N.ptr(Whh), None, N.ptr(h_all), N.ptr(c_all), N.ptr(act), N.ptr(rel),
                                     None, N.ptr(dl), None, T, B, H, 0, None, N.ptr(dh0), N.ptr(drel), None, None,
                                     N.stream_ptr()), "bwd")
            torch.cuda.synchronize()
            out.append((drel, dh0))
    (a, ad), (_, _), (b, bd), _ = out
    for t in range(T - 1, -1, -1):
        print("t=%2d drel max|q4-mw| %.3g  max|mw| %.3g" % (t, (a[t] - b[t]).abs().max().item(), b[t].abs().max().item()))
    print("dh0 max|q4-mw| %.3g max|mw| %.3g" % ((ad - bd).abs().max().item(), bd.abs().max().item()))
    e = (a[T - 1] - b[T - 1]).abs()
    print("step T-1 worst peds:", torch.topk(e.max(1)[0], 5))


if __name__ == "__main__":
    main()
