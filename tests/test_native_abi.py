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
    # S x jq (scene, j-range) units, jq = clamp(256 / S, 1, 8), capped at 256 workgroups
    assert lib.sgg_pool_bwd_grid(10) == 80 and lib.sgg_pool_bwd_grid(64) == 256
    assert lib.sgg_pool_bwd_grid(100000) == 256 and lib.sgg_pool_bwd_grid(0) == 1


def test_library_built_from_this_tree():
    """sgg_source_hash() (compiled in by build_native.py) equals the hash of
    the csrc/ + include/sgg.h sources here; load() refuses a stale binary."""
    from sgan import _native
    from sgan._srchash import source_files, source_hash
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libsgg.so not built")
    assert any(f.endswith("sgg.h") for f in source_files()) and len(source_files()) > 10
    lib = _native.load(require_gpu=False)
    assert lib.sgg_source_hash().decode() == source_hash()


def test_load_refuses_stale_library(monkeypatch):
    from sgan import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libsgg.so not built")
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "_LIB_EXPLICIT", False)
    monkeypatch.setattr(_native, "source_hash", lambda: "0" * 64)
    with pytest.raises(_native.NativeError, match="other sources"):
        _native.load(require_gpu=False)


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


def test_pool_plan_covers_every_row_once():
    """sgg_pool_plan (host function of the C ABI): chunks are whole i-rows of
    one scene, cover every (scene, row) exactly once, respect the pair cap."""
    import ctypes
    import numpy as np
    from sgan import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libsgg.so not built")
    lib = _native.load(require_gpu=False)
    rng = np.random.default_rng(0)
    for bn in (8, 48):
        for sizes in ([20] * 64, [1, 2, 64, 57, 3, 20, 0, 5], list(rng.integers(1, 65, size=300))):
            off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
            S = len(sizes)
            for target in (1, 64, 1024, 100000):
                cap = int(off[-1]) + S + 1
                tab = np.zeros((cap, 4), np.int32)
                mr, gpw = ctypes.c_int(0), ctypes.c_int(0)
                nc = lib.sgg_pool_plan(off.ctypes.data_as(ctypes.c_void_p), S, bn, target, 0,
                                       tab.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(mr), ctypes.byref(gpw))
                assert nc > 0 and gpw.value in (1, 2, 4, 8)
                cap_pairs = max(64 * gpw.value, 64)
                seen = {}
                for s, i0, i1, _ in tab[:nc]:
                    n = sizes[s]
                    assert 0 <= i0 < i1 <= n and i1 - i0 <= 64
                    assert (i1 - i0) * n <= cap_pairs or i1 - i0 == 1
                    assert i1 - i0 <= mr.value
                    for i in range(i0, i1):
                        assert (s, i) not in seen
                        seen[(s, i)] = 1
                assert len(seen) == int(off[-1])


def test_rccl_binding_symbols():
    """The captured all-reduce's direct RCCL binding (sgan/rccl.py) resolves
    its entry points in torch's own librccl.so (no GPU needed to load it)."""
    import os
    import torch
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if not os.path.exists(path):
        pytest.skip("torch without a bundled librccl.so")
    from sgan import rccl
    lib = rccl._rccl()
    for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclCommDestroy", "ncclGetErrorString"):
        assert hasattr(lib, f), f
    assert rccl.NCCL_FLOAT32 == 7 and rccl.NCCL_SUM == 0
    assert lib.ncclGetErrorString(0) is not None


def test_gatenc_saved_floats_carries_the_weight_image():
    """sgg_gatenc_saved_floats(S, np, nh) = S per-scene blocks + the weights'
    staged LDS image (round 5: the backward copies it instead of restaging the
    parameters) -- a fixed tail independent of S, growing with the heads."""
    from sgan import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libsgg.so not built")
    lib = _native.load(require_gpu=False)
    for nh in (1, 2, 4):
        tail = lib.sgg_gatenc_saved_floats(0, 20, nh)
        per = lib.sgg_gatenc_saved_floats(1, 20, nh) - tail
        assert tail > 0 and tail % 4 == 0 and per > 0
        assert lib.sgg_gatenc_saved_floats(64, 20, nh) == 64 * per + tail
    assert lib.sgg_gatenc_saved_floats(0, 20, 2) > lib.sgg_gatenc_saved_floats(0, 20, 1)
