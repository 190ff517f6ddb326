"""Every kernel of libsgg.so runs without scratch memory (CPU test: hipcc's
kernel-resource-usage remarks for gfx950, tools/kernel_resources.py).

Scratch is per-lane private memory in HBM: register spills, arrays the
compiler could not keep in registers, frames of calls left out of line.  In
a kernel's loop it is memory traffic the algorithm does not have (round 4:
the bf16 pooling forward wrote 6.8x its outputs, the GAT encoder backward
spilled).  The only kernels allowed scratch are listed with the reason they
are never dispatched at the reference's configurations.
"""
import os
import re
import shutil
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))

# (kernel-name regex, why it may keep scratch)
ALLOWED = [
    (r"lstm_unit_(fwd|bwd)_kernel<", "row-per-ped LSTM family, only reachable with the SGG_LSTM_MW=0 A/B switch"),
    (r"lstm_mw_bwd_kernel<64, ", "H = 64 LSTM backward: no reference configuration has a 64-wide LSTM"),
    (r"lstm_mw_bwd_kernel<48, true, ", "a 48-wide DECODER: the reference's decoders are 32 wide (train.py:53)"),
]


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not available")
def test_no_kernel_uses_scratch():
    import kernel_resources as KR
    rows = KR.collect()
    names = [r["name"] for r in rows]
    # the hot kernels of round 4's verdict are among those checked
    for must in ("pool_fwd_bf16_kernel<48, 4>", "gatenc_kernel<true, 1>", "lstm_fwd_mfma_kernel<32, true, true>",
                 "pool_fwd_kernel<48, 4, 2>", "lstm_mw_bwd_kernel<48, false, true>", "pool_fwd_x3_kernel<48, 2>"):
        assert any(must in n for n in names), must
    bad = []
    for r in rows:
        if r.get("scratch", 0) == 0 and r.get("vspill", 0) == 0:
            continue
        if any(re.search(p, r["name"]) for p, _ in ALLOWED):
            continue
        bad.append("%s: %d B/lane scratch, %d VGPRs spilled (%s)" % (KR.short(r["name"]), r.get("scratch", 0),
                                                                      r.get("vspill", 0), r["file"]))
    assert not bad, "kernels with scratch:\n" + "\n".join(bad)
