"""Debug: segment-split LSTM forward vs full sequence, per step / unit / ped."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
import torch  # noqa: E402

DEV = "cuda"


def main():
    from sgan import _native as N
    lib = N.load()
    torch.manual_seed(2)
    T, T0, Bs, C, H, NU = 11, 5, 32, 3, 48, 64
    B = Bs * C
    f = lambda *s, sc=0.3: (torch.randn(*s, device=DEV) * sc).contiguous()
    A, Whh, bias = f(4 * H, 2), f(4 * H, H, sc=0.2), f(4 * H)
    Wu, cu = f(NU, H), f(NU)
    head = f(T0, Bs, 2)
    rel = torch.cat([head.repeat(1, C, 1), f(T - T0, B, 2)], 0).contiguous()
    sf = lambda w: torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, w)), device=DEV)

    def run(mode):
        h_all, c_all, act = torch.zeros(T + 1, B, H, device=DEV), sf(1), sf(0)
        U = torch.empty(B, NU, device=DEV)
        if mode == "seg2":
            A2, W2, b2 = f(128, 2), f(128, 32, sc=0.2), f(128)
            h2 = torch.empty(T0 + 1, Bs, 32, device=DEV)
            g2 = N.LstmSeg(N.ptr(head), N.ptr(A2), N.ptr(W2), N.ptr(b2), None, None, T0, Bs, Bs, 0, T0, Bs,
                           N.ptr(h2), None, None, None, 0, None, 0, None)
            pre = N.LstmSeg(N.ptr(head), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, T0, Bs, B, 0, T, Bs,
                            N.ptr(h_all), N.ptr(c_all), N.ptr(act), None, 0, None, 0, None)
            N.check(lib.sgg_lstm_fwd_seg2(N.ctypes.byref(g2), 32, N.ctypes.byref(pre), H, N.stream_ptr()), "seg2")
        elif mode == "seg1":
            pre = N.LstmSeg(N.ptr(head), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, T0, Bs, B, 0, T, Bs,
                            N.ptr(h_all), N.ptr(c_all), N.ptr(act), None, 0, None, 0, None)
            N.check(lib.sgg_lstm_fwd_seg(N.ctypes.byref(pre), H, N.stream_ptr()), "seg")
        if mode != "full":
            suf = N.LstmSeg(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, T - T0, B, B, T0, T, Bs,
                            N.ptr(h_all), N.ptr(c_all), N.ptr(act), N.ptr(Wu), Wu.stride(0), N.ptr(cu), NU, N.ptr(U))
            N.check(lib.sgg_lstm_fwd_seg(N.ctypes.byref(suf), H, N.stream_ptr()), "seg")
        else:
            N.check(lib.sgg_lstm_fwd_u(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, T, B, H,
                                       N.ptr(h_all), N.ptr(c_all), N.ptr(act), N.ptr(Wu), Wu.stride(0), N.ptr(cu),
                                       NU, N.ptr(U), N.stream_ptr()), "fwd_u")
        torch.cuda.synchronize()
        return h_all.clone(), c_all.clone(), act.clone()
    full = run("full")
    # the continuation alone from the FULL run's state at step T0
    h_all, c_all, act = full[0].clone(), full[1].clone(), full[2].clone()
    U = torch.empty(B, NU, device=DEV)
    suf = N.LstmSeg(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, T - T0, B, B, T0, T, B,
                    N.ptr(h_all), N.ptr(c_all), N.ptr(act), N.ptr(Wu), Wu.stride(0), N.ptr(cu), NU, N.ptr(U))
    N.check(lib.sgg_lstm_fwd_seg(N.ctypes.byref(suf), H, N.stream_ptr()), "seg")
    torch.cuda.synchronize()
    for t in range(T0, T + 1):
        d = (h_all[t] - full[0][t]).abs()
        print("cont-from-full step %2d h max %.3e" % (t, d.max().item()))
    # one step only: T0 .. T0 + 1
    h2, c2, a2 = full[0].clone(), full[1].clone(), full[2].clone()
    suf = N.LstmSeg(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, 1, B, B, T0, T, B,
                    N.ptr(h2), N.ptr(c2), N.ptr(a2), None, 0, None, 0, None)
    N.check(lib.sgg_lstm_fwd_seg(N.ctypes.byref(suf), H, N.stream_ptr()), "seg")
    torch.cuda.synchronize()
    d = (h2[T0 + 1] - full[0][T0 + 1]).abs()
    print("one step from full: max %.3e  nbad %d" % (d.max().item(), int((d > 0).sum())))
    # float64 reference of that one step from the full run's state
    hp = full[0][T0].double()                         # h_{T0-1} (B x H)
    # c at index T0 of the tile-native layout: c[((blk (T+1) + t) 4 + g) 64 + lane) 3 + i], unit slot_unit(g 3 + i, q)
    cst = full[1].view(-1)
    cprev = torch.empty(B, H, dtype=torch.float64, device=DEV)
    for blk in range(B // 16):
        for g in range(4):
            for lane in range(64):
                q, c16 = lane >> 4, lane & 15
                for i in range(3):
                    j = g * 3 + i
                    u = 16 * (j >> 2) + 4 * q + (j & 3)
                    cprev[blk * 16 + c16, u] = cst[(((blk * (T + 1) + T0) * 4 + g) * 64 + lane) * 3 + i].double()
    pre = hp @ Whh.double().t() + rel[T0].double() @ A.double().t() + bias.double()
    i_, f_, g_, o_ = pre.split(H, 1)
    cn = torch.sigmoid(f_) * cprev + torch.sigmoid(i_) * torch.tanh(g_)
    hn = torch.sigmoid(o_) * torch.tanh(cn)
    print("full  vs f64: %.3e" % (full[0][T0 + 1].double() - hn).abs().max().item())
    print("cont  vs f64: %.3e" % (h2[T0 + 1].double() - hn).abs().max().item())
    if hasattr(lib, "sgg_dbg_hx"):
        import numpy as np
        hx = np.zeros((2, 4, 64, 2, 3, 4), np.uint32)
        acc = np.zeros((2, 4, 64, 3, 4), np.float32)
        import ctypes
        lib.sgg_dbg_hx.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.sgg_dbg_hx(hx.ctypes.data, acc.ctypes.data)
        d = hx[0] != hx[1]
        print("hx differ:", int(d.sum()), "of", d.size)
        if d.any():
            idx = np.argwhere(d)[:12]
            for w, ln, cc, p_, e in idx:
                print("  wave %d lane %d chunk %d piece %d word %d: %08x vs %08x" % (w, ln, cc, p_, e, hx[0, w, ln, cc, p_, e], hx[1, w, ln, cc, p_, e]))
        da = np.abs(acc[0] - acc[1])
        print("acc max diff %.3e  n %d" % (da.max(), int((da > 0).sum())))
    for mode in ("seg1", "seg2"):
        x = run(mode)
        print("==", mode)
        for t in range(T + 1):
            d = (x[0][t] - full[0][t]).abs()
            bad = (d > 0).nonzero()
            units = sorted(set(bad[:, 1].tolist()))
            peds = sorted(set(bad[:, 0].tolist()))
            print("step %2d h max %.3e  units %s  peds %s" % (t, d.max().item(), units[:48], peds[:10]))
        # cells of the prefix blocks (peds < 32: blocks 0, 1), steps 0..T0
        per = (T + 1) * 4 * 64 * 3
        for b in range(2):
            for t in range(T0 + 2):
                o = b * per + t * 4 * 64 * 3
                d = (x[1][o:o + 4 * 64 * 3] - full[1][o:o + 4 * 64 * 3]).abs().max().item()
                if d > 0:
                    print("c block %d step %d max %.3e" % (b, t, d))


if __name__ == "__main__":
    main()
