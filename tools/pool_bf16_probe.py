"""The bf16 pooling forward on S scenes of n peds (configs[4]'s shape by
default), for rocprofv3 counter passes and timing.
usage: python tools/pool_bf16_probe.py [bn] [S] [n] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "group-gan-gcn-gat_amd"))
from sgan import kernels as K  # noqa: E402
from sgan.models import PoolHiddenNet  # noqa: E402
from sgan.scene import SceneIndex  # noqa: E402


def main():
    bn = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    import numpy as np
    dev = "cuda"
    torch.manual_seed(0)
    H = 48 if bn == 48 else 32
    mod = PoolHiddenNet(embedding_dim=16, h_dim=H, mlp_dim=64, bottleneck_dim=bn, batch_norm=False).to(dev)
    sc = SceneIndex(np.arange(S + 1) * n, dev)
    h = torch.randn(S * n, H, device=dev)
    pos = torch.rand(S * n, 2, device=dev) * 10
    K.set_precision(os.environ.get("PREC", "bf16"))
    with torch.no_grad():
        for _ in range(2):
            mod(h, None, pos, scenes=sc)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            mod(h, None, pos, scenes=sc)
        e1.record()
        e1.synchronize()
    print("bn %d S %d n %d %s: %.1f us per forward (fold + U + pool)" % (bn, S, n, K.precision(), e0.elapsed_time(e1) * 1e3 / reps))


if __name__ == "__main__":
    main()
