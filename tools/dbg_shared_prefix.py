"""Debug: shared-prefix vs full D encoder (test_shared_prefix_is_bit_identical), every mismatching tensor."""
import contextlib
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from test_gpu_parity import build_models  # noqa: E402


def main():
    from sgan import kernels as K
    from sgan.data.synthetic import synthetic_batch
    from sgan.scene import SceneIndex
    from sgan.train_step import GanTrainer, KernelOps
    sizes = [20, 7, 13, 20, 4]
    batch = synthetic_batch(sizes, seed=5, device="cuda")
    sc = SceneIndex.from_seq_start_end(batch[-1], "cuda")

    class Full(KernelOps):
        shared_prefix = None
    res = []
    for ops in (KernelOps(), Full()):
        g, d = build_models("gat")
        tr = GanTrainer(g, d, ops=ops)
        torch.manual_seed(3)
        random.seed(3)
        out = {}
        ld = tr.d_step(batch, sc)
        out.update({"d." + k: p.grad.detach().clone() for k, p in d.named_parameters() if p.grad is not None})
        lg = tr.g_step(batch, sc)
        out.update({"g." + k: p.grad.detach().clone() for k, p in g.named_parameters() if p.grad is not None})
        out.update({"loss." + k: torch.tensor(float(v)) for k, v in list(ld.items()) + list(lg.items())})
        res.append(out)
    a, b = res
    for k in sorted(a):
        dd = (a[k].float() - b[k].float()).abs().max().item()
        print("%-45s %s %.3e" % (k, "==" if torch.equal(a[k], b[k]) else "!=", dd))


if __name__ == "__main__":
    main()
