"""Build libsgg.so (gfx950) in-tree with hipcc: one shared library, C ABI.

    python group-gan-gcn-gat_amd/build_native.py [--jobs N]

Objects are compiled in parallel and linked into sgan/_lib/libsgg.so, which
is git-ignored but travels to the GPU box with the repo snapshot.
"""
import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "sgan", "_lib")
LIB = os.path.join(OUT_DIR, "libsgg.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wall", "-Wno-unused-result",
         "-munsafe-fp-atomics"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _compile(src, obj):
    cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, r.stdout, r.stderr))
    return obj


def build(jobs=8, verbose=True):
    os.makedirs(OUT_DIR, exist_ok=True)
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    srcs = sources()
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs.append(os.path.join(os.path.dirname(HERE), "include", "sgg.h"))
    newest_hdr = max(os.path.getmtime(h) for h in hdrs)
    todo = [(s, o) for s, o in zip(srcs, objs)
            if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), newest_hdr)]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for o in ex.map(lambda so: _compile(*so), todo):
            if verbose:
                print("compiled", os.path.basename(o))
    if todo or not os.path.exists(LIB):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
        if verbose:
            print("linked", LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    build(a.jobs)
