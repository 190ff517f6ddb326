"""Kernel sequence of one training iteration from a rocprofv3 kernel trace:
iterations are delimited by the G-step's fused-Adam launch (every second
FusedAdam).  Usage: python tools/iter_seq.py [prof_dir] [iteration_index]"""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
want = int(sys.argv[2]) if len(sys.argv) > 2 else -4
rows = sorted(csv.DictReader(open(d + "/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "FusedAdam" in r["Kernel_Name"]]
ends = adam[1::2]
i1 = ends[want]
i0 = ends[want - 1] + 1
seq = rows[i0:i1 + 1]
t0 = int(seq[0]["Start_Timestamp"])
prev_end = t0
tot_k = tot_gap = 0.0
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3
    dur = (e - s) / 1e3
    tot_k += dur
    tot_gap += max(gap, 0)
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "at::native" in name:
        name = "at::" + name.split("at::native::")[-1][:60]
    wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    print("%8.1f %6.1f %6.1f  wgs=%-5d %s" % ((s - t0) / 1e3, dur, gap, wg, name[:90]))
print("launches %d  kernel %.1f us  gaps %.1f us  span %.1f us" % (len(seq), tot_k, tot_gap,
      (int(seq[-1]["End_Timestamp"]) - t0) / 1e3))
