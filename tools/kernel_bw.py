"""Per-kernel HBM GB/s: PMC traffic per launch (profiles/r01_pool_traffic.json,
eager bench) / rocprofv3 average duration (kernel stats of the graphed bench).
usage: python tools/kernel_bw.py TRAFFIC_JSON KERNEL_STATS_CSV [N]"""
import csv
import json
import re
import sys

tab = json.load(open(sys.argv[1]))["kernels"]
rows = list(csv.DictReader(open(sys.argv[2])))
n = int(sys.argv[3]) if len(sys.argv) > 3 else 15


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(sgg::[A-Za-z_0-9:]+(<[^()]*>)?)\(", name)
    return m.group(1) if m else name[:50]


print("%-42s %9s %10s %9s %7s" % ("kernel", "avg us", "HBM MB", "GB/s", "% 8TB/s"))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    k = short(r["Name"])
    us = float(r["AverageNs"]) / 1e3
    t = tab.get(k)
    if t is None:
        print("%-42s %9.1f %10s" % (k[:42], us, "-"))
        continue
    gbs = t["hbm_bytes"] / (us * 1e-6) / 1e9
    print("%-42s %9.1f %10.2f %9.0f %6.1f%%" % (k[:42], us, t["hbm_bytes"] / 1e6, gbs, gbs / 80.0))
