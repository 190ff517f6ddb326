"""Average duration per (kernel, grid) from a rocprofv3 kernel trace CSV.
usage: python tools/ktrace_summary.py DIR [filter]"""
import collections
import csv
import os
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.search(r"((sgg|at::native)::[A-Za-z_0-9:]+(<[^()]{0,40})?)", n)
    return (m.group(1) if m else n)[:60]


rows = list(csv.DictReader(open(os.path.join(sys.argv[1], "run_kernel_trace.csv"))))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for r in rows:
    k = short(r["Kernel_Name"])
    if flt not in k:
        continue
    d[(k, r.get("Grid_Size_X") or r.get("Grid_Size"))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print("%-55s grid=%-8s n=%4d avg %7.1f us  total %8.1f" % (k, g, len(v), sum(v) / len(v), sum(v)))
