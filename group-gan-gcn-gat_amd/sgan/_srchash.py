"""Source hash of libsgg.so: SHA-256 over the kernel sources it is built from.

build_native.py compiles this hash into the library (`sgg_source_hash()`);
`_native.load` recomputes it from the tree it runs in and refuses a library
built from other sources, so a green GPU run proves the kernels of HEAD and
not a stale prebuilt binary.  The compile flags are part of the hash (they
live here, and build_native.py takes them from here): a library built with
other flags -- e.g. without lstm_mfma.hip's VGPR-form accumulators -- is
refused too.  No torch import: the build script uses it too.
"""
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
HEADER = os.path.join(os.path.dirname(PKG), "include", "sgg.h")

# hipcc flags of every object, and per-source extra flags: the batch-MFMA
# rollout keeps its accumulators in VGPRs (MFMA VGPR form): the AGPR form read
# every gate value back with a v_accvgpr_read per step (32 VALU instructions
# per step on its critical path)
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wall", "-Wno-unused-result",
         "-munsafe-fp-atomics"]
FILE_FLAGS = {"lstm_mfma.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def source_files():
    """csrc/*.hip, csrc/*.h and include/sgg.h, in a fixed order."""
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    return [os.path.join(CSRC, f) for f in names] + [HEADER]


def source_hash():
    h = hashlib.sha256()
    h.update(repr((FLAGS, sorted(FILE_FLAGS.items()))).encode())
    h.update(b"\0")
    for path in source_files():
        h.update(os.path.relpath(path, os.path.dirname(PKG)).encode())
        h.update(b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()
