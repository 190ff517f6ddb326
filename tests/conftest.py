import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "group-gan-gcn-gat_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels through the C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def load_family(model, sd):
    """Load a reference-built generator state (committed GAT layout:
    gatencoder.gat_intra/inter + gcn_module) into a model of any checkpoint
    family.  Keys the family lacks (the group GAT for 'gcn') are dropped;
    the only keys allowed to stay at init are mlp_decoder_context.*, which
    those families carry but never call."""
    own = model.state_dict()
    take = {k: v for k, v in sd.items() if k in own}
    missing = [k for k in own if k not in take]
    assert all(k.startswith("mlp_decoder_context.") for k in missing), missing
    model.load_state_dict(take, strict=False)
    return model


class RecordingAdam:
    """Mixin factory: an optimizer class whose step() first records every
    parameter's .grad (after backward and clipping, before the update) -- the
    test-side mirror of make_golden.py's _RecordingAdam."""

    @staticmethod
    def make(named, **kw):
        import torch

        class _Rec(torch.optim.Adam):
            def __init__(self, named):
                self.named = list(named)
                self.rec = []
                super().__init__([p for _, p in self.named], **kw)

            def step(self, closure=None):
                self.rec.append({k: p.grad.detach().cpu().clone() for k, p in self.named if p.grad is not None})
                return super().step(closure)
        return _Rec(named)


def check_step_grads(rec, f, it, kind, rtol=1e-3):
    """Compare recorded gradients with the fixture's it%d/grad{D,G}/<param>:
    max |a - b| <= rtol * max(|b|, 1 % of the largest gradient of the step)."""
    import numpy as np
    prefix = "it%d/grad%s/" % (it, kind)
    keys = [k for k in f.files if k.startswith(prefix)]
    assert keys, prefix
    floor = 1e-2 * max(np.abs(f[k]).max() for k in keys)
    rec = {n: (v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)) for n, v in rec.items()}
    for k in keys:
        name = k[len(prefix):]
        assert name in rec, (kind, name, "no gradient")
        a = np.asarray(rec[name], np.float64)
        b = np.asarray(f[k], np.float64)
        err = np.abs(a - b).max() / max(np.abs(b).max(), floor)
        assert err <= rtol, "it%d grad%s %s: max rel err %.3e" % (it, kind, name, err)
    extra = [n for n in rec if prefix + n not in f.files and float(abs(rec[n]).max()) != 0.0]
    assert not extra, ("gradients the reference does not have", extra)
