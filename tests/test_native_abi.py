"""CPU-side checks of the C-ABI library: it loads (no GPU needed to dlopen)
and exports every entry point include/sgg.h declares, with the ctypes
signature table covering exactly those.  No compute calls."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sgg.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sgg_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    names = declared()
    for n in ("sgg_xw", "sgg_pool_fwd", "sgg_pool_bwd", "sgg_gat_fwd", "sgg_gat_bwd", "sgg_group_index",
              "sgg_seg_reduce", "sgg_seg_gather"):
        assert n in names


def test_library_exports_header_symbols():
    from sgan import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libsgg.so not built (run __graft_entry__.build())")
    lib = _native.load(require_gpu=False)
    for n in declared():
        assert hasattr(lib, n), n
    assert set(declared()) == set(_native.SIGNATURES), "ctypes table out of sync with include/sgg.h"
    assert lib.sgg_version() >= 1
    assert lib.sgg_pool_bwd_grid(10) == 10 and lib.sgg_pool_bwd_grid(100000) == 256


def test_product_path_has_no_cpu_fallback():
    import torch
    from sgan import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libsgg.so not built")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_native.NativeError):
        _native.load(require_gpu=True)
    from sgan import kernels
    with pytest.raises(_native.NativeError):
        kernels.xw(torch.ones(4, 4), torch.ones(4, 4))
