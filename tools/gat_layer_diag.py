"""Fused (sgg_gat_layer_fwd) vs per-op batched-GAT layer: where do the two
paths' forward values and gradients part (diagnostic, GPU)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "group-gan-gcn-gat_amd"))
from sgan import kernels as K  # noqa: E402
from sgan.models import BatchGAT, BatchGATEncoder  # noqa: E402
from sgan.scene import SceneIndex  # noqa: E402

DEV = "cuda"
torch.manual_seed(4)
mod = BatchGATEncoder([40, 16, 40], [4, 1], 0.0, 0.2).to(DEV)
with torch.no_grad():
    for l in mod.gat_net.layer_stack:
        l.bias.normal_(0, 0.1)
sizes = [64] * 9
sc = SceneIndex(np.concatenate([[0], np.cumsum(sizes)]), DEV)
x = torch.randn(sum(sizes), 40, device=DEV)
dy = torch.randn(sum(sizes), 40, device=DEV)
res = {}
for fused in (True, False):
    BatchGAT.LAYER_FUSED = fused
    acts = []
    hooks = []
    mod.zero_grad(set_to_none=True)
    xi = x.clone().requires_grad_(True)
    graph = K.SegmentGraph(sc.scene_off, sc.S, sc.max_n, 1, None)
    h = xi
    outs = []
    for i, layer in enumerate(mod.gat_net.layer_stack):
        epi = 0 if i + 1 == len(mod.gat_net.layer_stack) else 1
        if fused:
            h = K.gat_layer(h, layer.w, layer.a_src, layer.a_dst, layer.bias, graph, epi)
        else:
            h = layer(K.seg_instance_norm(h, graph.seg_off, graph.nseg), graph, epi)
        h.retain_grad()
        outs.append(h)
    (h * dy).sum().backward()
    res[fused] = ([o.detach().clone() for o in outs], [o.grad.clone() for o in outs], xi.grad.clone(),
                  {k: p.grad.clone() for k, p in mod.named_parameters()})
BatchGAT.LAYER_FUSED = True
for i in range(2):
    a, b = res[True][0][i], res[False][0][i]
    print("layer %d out   max|diff| %.3e  scale %.3e" % (i, (a - b).abs().max(), b.abs().max()))
    a, b = res[True][1][i], res[False][1][i]
    print("layer %d dout  max|diff| %.3e  scale %.3e" % (i, (a - b).abs().max(), b.abs().max()))
print("dx max|diff| %.3e scale %.3e" % ((res[True][2] - res[False][2]).abs().max(), res[False][2].abs().max()))
for k in res[True][3]:
    a, b = res[True][3][k], res[False][3][k]
    print("%-40s max|diff| %.3e scale %.3e" % (k, (a - b).abs().max(), b.abs().max()))
