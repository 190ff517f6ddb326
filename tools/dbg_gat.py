import sys, os
sys.path.insert(0, "group-gan-gcn-gat_amd")
import numpy as np, torch
from sgan import kernels as K
from sgan.models import GATEncoder
from sgan.scene import SceneIndex
DEV = "cuda"
torch.manual_seed(0)
mod = GATEncoder([40, 16, 40], 1, 0.0, 0.2).to(DEV)
for sizes in ([20] * 4, [5, 9], [30, 10], [40], [48], [57], [64]):
    B = sum(sizes)
    sc = SceneIndex(np.concatenate([[0], np.cumsum(sizes)]), DEV)
    lab = torch.randint(0, 4, (B, 1), device=DEV).float()
    x = torch.randn(B, 40, device=DEV)
    outs = []
    for fused in (True, False):
        K.GATENC_FUSED = fused
        with torch.no_grad():
            outs.append(mod(x, None, None, lab, scenes=sc))
    K.GATENC_FUSED = True
    err = (outs[0] - outs[1]).abs().max().item()
    print(sizes[:3], "lds_fwd", K._lib().sgg_gatenc_lds_bytes(max(sizes), 1, 0), "err %.3e" % err, flush=True)
