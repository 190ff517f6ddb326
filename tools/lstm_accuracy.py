"""Accuracy of the four-wave encoder forward against float64: max |h - h64| over
all steps for H 32 / 48 (the lib under SGG_LIB or the default)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
import torch  # noqa: E402


def main():
    from sgan import _native as N
    lib = N.load()
    dev = "cuda"
    for H in (32, 48):
        torch.manual_seed(H)
        T, B = 20, 1280
        f = lambda *s, sc=0.3: (torch.randn(*s, device=dev) * sc).contiguous()
        A, Whh, bias = f(4 * H, 2), f(4 * H, H, sc=0.3), f(4 * H)
        rel = f(T, B, 2, sc=0.5)
        h_all = torch.empty(T + 1, B, H, device=dev)
        sf = lambda w: torch.empty(int(lib.sgg_lstm_state_floats(T, B, H, w)), device=dev)
        c_all, act = sf(1), sf(0)
        N.check(lib.sgg_lstm_fwd(N.ptr(rel), N.ptr(A), N.ptr(Whh), N.ptr(bias), None, None, None, None, T, B, H, 0,
                                 N.ptr(h_all), N.ptr(c_all), N.ptr(act), None, N.stream_ptr()), "fwd")
        torch.cuda.synchronize()
        # float64 and float32 torch references of the same recurrence
        errs = {}
        for dt in (torch.float64, torch.float32):
            h = torch.zeros(B, H, dtype=dt, device=dev)
            c = torch.zeros(B, H, dtype=dt, device=dev)
            hs = [h]
            for t in range(T):
                pre = h @ Whh.to(dt).t() + rel[t].to(dt) @ A.to(dt).t() + bias.to(dt)
                i_, f_, g_, o_ = pre.split(H, 1)
                c = torch.sigmoid(f_) * c + torch.sigmoid(i_) * torch.tanh(g_)
                h = torch.sigmoid(o_) * torch.tanh(c)
                hs.append(h)
            errs[dt] = torch.stack(hs)
        e_hip = (h_all.double() - errs[torch.float64]).abs().max().item()
        e_t32 = (errs[torch.float32].double() - errs[torch.float64]).abs().max().item()
        print("H %d: |hip - f64| %.3e   |torch fp32 - f64| %.3e" % (H, e_hip, e_t32), flush=True)


if __name__ == "__main__":
    main()
