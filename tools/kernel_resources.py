"""Register / scratch / occupancy report of every kernel in libsgg.so's sources
(hipcc's kernel-resource-usage remarks, gfx950, the build's flags).

usage: python tools/kernel_resources.py [out.txt] [--files pool.hip,gat_encoder.hip]

ScratchSize is the per-lane private memory a kernel needs: register spills,
stack-resident arrays (e.g. a struct copied under a condition) and the frames
of calls the inliner left out of line.  Every byte of it is memory traffic
inside the kernel's loops, so the product's kernels are kept at 0
(tests/test_kernel_resources.py checks the hot ones).
"""
import concurrent.futures as cf
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "group-gan-gcn-gat_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-munsafe-fp-atomics",
         "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/dev/null"]
FIELDS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"), ("ScratchSize [bytes/lane]", "scratch"),
          ("VGPRs Spill", "vspill"), ("SGPRs Spill", "sspill"), ("Occupancy [waves/SIMD]", "occ"),
          ("LDS Size [bytes/block]", "lds")]


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


def resources(src):
    """[{name, vgpr, agpr, sgpr, scratch, vspill, sspill, occ, lds}] of one source file."""
    sys.path.insert(0, os.path.join(ROOT, "group-gan-gcn-gat_amd"))
    from build_native import FILE_FLAGS   # the build's per-source flags
    extra = FILE_FLAGS.get(os.path.basename(src), [])
    r = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + extra + [src], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, r.stderr[-2000:]))
    rows, cur = [], None
    keys = dict(FIELDS)
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = {"mangled": t.split(":", 1)[1].strip(), "file": os.path.basename(src)}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            if k.strip() in keys:
                try:
                    cur[keys[k.strip()]] = int(v.strip())
                except ValueError:
                    pass
    for row, name in zip(rows, demangle([x["mangled"] for x in rows])):
        row["name"] = name
    return rows


def collect(files=None, jobs=8):
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    if files:
        srcs = [s for s in srcs if os.path.basename(s) in files]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        return [row for rows in ex.map(resources, srcs) for row in rows]


def short(name):
    """kernel name without the argument list"""
    name = name.replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i].replace("void ", "")
    return name


def report(rows):
    out = ["# kernel resources (hipcc -O3 --offload-arch=gfx950 -Rpass-analysis=kernel-resource-usage), "
           "tools/kernel_resources.py",
           "# %d kernels; nonzero scratch: %d" % (len(rows), sum(1 for r in rows if r.get("scratch", 0))),
           "%-16s %5s %5s %5s %7s %6s %6s %4s %6s  %s" % ("file", "VGPR", "AGPR", "SGPR", "scratch", "vspill",
                                                          "sspill", "occ", "LDS", "kernel")]
    for r in sorted(rows, key=lambda r: (r["file"], r["name"])):
        out.append("%-16s %5d %5d %5d %7d %6d %6d %4d %6d  %s" % (
            r["file"], r.get("vgpr", 0), r.get("agpr", 0), r.get("sgpr", 0), r.get("scratch", 0),
            r.get("vspill", 0), r.get("sspill", 0), r.get("occ", 0), r.get("lds", 0), short(r["name"])))
    return "\n".join(out) + "\n"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--files")]
    files = None
    for a in sys.argv[1:]:
        if a.startswith("--files"):
            files = a.split("=", 1)[1].split(",")
    text = report(collect(files))
    if args:
        with open(args[0], "w") as f:
            f.write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
