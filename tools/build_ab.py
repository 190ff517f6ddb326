"""Build a variant of libsgg.so for an A/B run: every csrc/*.hip compiled
with extra defines into tools/abx/<name>/, linked to tools/abx/libsgg_<name>.so
(git-ignored; it travels to the GPU box).  Load it with SGG_LIB=<path> (that
skips the source-hash check).

usage: python tools/build_ab.py NAME [-DMACRO=V ...]"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "group-gan-gcn-gat_amd")
sys.path.insert(0, PKG)
from sgan._srchash import FILE_FLAGS, FLAGS  # noqa: E402

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    out = os.path.join(ROOT, "tools", "abx", name)
    os.makedirs(out, exist_ok=True)
    csrc = os.path.join(PKG, "csrc")
    srcs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".hip"))

    def comp(src):
        obj = os.path.join(out, os.path.basename(src) + ".o")
        cmd = [HIPCC] + FLAGS + FILE_FLAGS.get(os.path.basename(src), []) + defs + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return obj
    with cf.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(comp, srcs))
    hsrc = os.path.join(out, "hash.hip")
    with open(hsrc, "w") as f:
        f.write('extern "C" const char* sgg_source_hash(void) { return "ab-%s"; }\n' % name)
    objs.append(comp(hsrc))
    lib = os.path.join(ROOT, "tools", "abx", "libsgg_%s.so" % name)
    subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main()
