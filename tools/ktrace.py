"""Per-(kernel, grid) launch durations from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
pat = sys.argv[2] if len(sys.argv) > 2 else "sgg::"
rows = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
agg = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if pat in n:
        key = (n.split("(")[0][-48:], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), r["Workgroup_Size_X"],
               r["LDS_Block_Size"], r["VGPR_Count"])
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print("%-48s wgs=%-6d wg=%-5s lds=%-6s vgpr=%-4s n=%3d avg=%8.1f us tot=%8.1f" % (k[0], k[1], k[2], k[3], k[4],
          len(v), sum(v) / len(v), sum(v)))
