"""LSTM sequence kernels at the training shapes, alone (for rocprofv3 kernel
traces / PMC passes): the discriminator encoder (H 48, T 20) at the D-step
(B 2560, weight gradients) and G-step (B 1280, input gradients only) sizes,
and the generator's H 32 encoder / decoder.  Prints HIP-event times.
usage: python tools/lstm_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))

import torch  # noqa: E402

from sgan import kernels as K  # noqa: E402
from sgan import models as M  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.manual_seed(0)
    dev = "cuda"
    cases = [("D enc wgrad", 48, 20, 2560, False, True), ("D enc frozen", 48, 20, 1280, False, False),
             ("G enc", 32, 8, 1280, False, True), ("G dec", 32, 12, 2560, True, True)]
    if os.environ.get("LSTM_PROBE_BOK"):   # the best-of-k rollout alone (20 samples x 1280 peds, no grad)
        cases = [("G dec bok", 32, 12, 25600, True, False)]
    if os.environ.get("LSTM_PROBE_MORE"):   # batch-size vs weight-gradient effects of the D encoder
        cases += [("D wgrad 1280", 48, 20, 1280, False, True), ("D frozen 2560", 48, 20, 2560, False, False)]
    for name, H, T, B, dec, wgrad in cases:
        if dec:
            mod = M.Decoder(T, 16, H, 64, 1, False).to(dev)
        else:
            mod = M.Encoder(16, H).to(dev)
        for p in mod.parameters():
            p.requires_grad_(wgrad)
        if dec:
            h0 = (torch.randn(1, B, H, device=dev) * 0.5).requires_grad_(wgrad)
            lp, lr = torch.randn(B, 2, device=dev), torch.randn(B, 2, device=dev) * 0.3
            fwd = lambda: mod(lp, lr, (h0, None), None)[0]
        else:
            rel = (torch.randn(T, B, 2, device=dev) * 0.3).requires_grad_(True)
            fwd = lambda: mod(rel)
        dy = None
        times = {}
        for _ in range(3):
            y = fwd()
            dy = torch.randn_like(y)
            if y.requires_grad:
                y.backward(dy)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tf = tb = 0.0
        for _ in range(reps):
            e[0].record()
            y = fwd()
            e[1].record()
            if y.requires_grad:
                y.backward(dy)
            e[2].record()
            e[2].synchronize()
            tf += e[0].elapsed_time(e[1])
            tb += e[1].elapsed_time(e[2])
        print("%-14s H=%d T=%d B=%d  fwd %.1f us  bwd %.1f us (incl. host launch gaps)"
              % (name, H, T, B, tf / reps * 1e3, tb / reps * 1e3), flush=True)


if __name__ == "__main__":
    main()
