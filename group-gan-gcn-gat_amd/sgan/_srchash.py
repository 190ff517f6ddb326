"""Source hash of libsgg.so: SHA-256 over the kernel sources it is built from.

build_native.py compiles this hash into the library (`sgg_source_hash()`);
`_native.load` recomputes it from the tree it runs in and refuses a library
built from other sources, so a green GPU run proves the kernels of HEAD and
not a stale prebuilt binary.  No torch import: the build script uses it too.
"""
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
HEADER = os.path.join(os.path.dirname(PKG), "include", "sgg.h")


def source_files():
    """csrc/*.hip, csrc/*.h and include/sgg.h, in a fixed order."""
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    return [os.path.join(CSRC, f) for f in names] + [HEADER]


def source_hash():
    h = hashlib.sha256()
    for path in source_files():
        h.update(os.path.relpath(path, os.path.dirname(PKG)).encode())
        h.update(b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()
