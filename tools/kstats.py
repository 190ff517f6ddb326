"""Summarise a rocprofv3 kernel_stats.csv / kernel_trace.csv pair."""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
rows = list(csv.DictReader(open(d + "/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print("total kernel ms %.3f over %d launches" % (tot / 1e6, calls))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print("%8.3f ms %6s calls %8.1f us avg %5.1f%%  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["Percentage"]), r["Name"][:100]))
