"""Per-kernel register / occupancy table of one HIP source (hipcc's
kernel-resource-usage remarks), optionally filtered by a name substring.
usage: python tools/kres.py group-gan-gcn-gat_amd/csrc/pool.hip [filter]"""
import re
import subprocess
import sys

FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-munsafe-fp-atomics",
         "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/dev/null"]


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    # the build's per-source flags (e.g. lstm_mfma.hip's -amdgpu-mfma-vgpr-form), as kernel_resources.py does
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "group-gan-gcn-gat_amd"))
    from build_native import FILE_FLAGS
    extra = FILE_FLAGS.get(os.path.basename(src), [])
    r = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + extra + [src], capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    print("%-6s %-6s %-6s %-7s %-5s %-6s %s" % ("VGPR", "AGPR", "spill", "scratch", "occ", "LDS", "kernel"))
    for c in rows:
        n = subprocess.run(["c++filt"], input=c["name"], capture_output=True, text=True).stdout.strip()
        if filt not in n:
            continue
        print("%-6s %-6s %-6s %-7s %-5s %-6s %s" % (c.get("VGPRs"), c.get("AGPRs"), c.get("VGPRs Spill"), c.get("ScratchSize [bytes/lane]"),
                                              c.get("Occupancy [waves/SIMD]"), c.get("LDS Size [bytes/block]"),
                                              n[:110]))


if __name__ == "__main__":
    main()
