"""The kernels of one graph-replayed training iteration from a rocprofv3
kernel trace (bench.py's timed replays): the launches between two
consecutive starts of the best-of-k rollout, with durations and gaps.
usage: python tools/ktrace_iter.py TRACE_DIR [which replay, default: the middle one]"""
import csv
import os
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.search(r"((sgg|at::native)::[A-Za-z_0-9:]+(<[^()]{0,40})?)", n)
    return (m.group(1) if m else n)[:58]


rows = list(csv.DictReader(open(os.path.join(sys.argv[1], "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def grid(r):
    return int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)


# the rollout: the largest-grid launch of the rollout kernel (configurations
# whose decoder also runs lstm_fwd_mfma launch it with a smaller grid)
mark = [i for i, r in enumerate(rows) if "lstm_fwd_mfma" in r["Kernel_Name"]]
gmax = max(grid(rows[i]) for i in mark)
idx = [i for i in mark if grid(rows[i]) == gmax]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
busy, prev, cover, reach = 0, None, 0, t0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f %6.1f %6.1f  %-58s grid=%s q=%s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0,
                                                     short(r["Kernel_Name"]), r.get("Grid_Size_X") or r.get("Grid_Size"),
                                                     r.get("Queue_Id", r.get("Stream_Id", "?"))))
    busy += e - s
    prev = e
    cover += max(0, e - max(s, reach))   # union of the kernels' intervals (two streams may overlap)
    reach = max(reach, e)
print("%d kernels, %.1f us busy, %.1f us covered, %.1f us period" % (
    b - a, busy / 1e3, cover / 1e3, (int(rows[b]["Start_Timestamp"]) - t0) / 1e3))
