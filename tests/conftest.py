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
