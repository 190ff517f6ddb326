"""Spans between consecutive launches of a marker kernel (one per training
iteration) in a rocprofv3 kernel trace, largest first, with the kernels
around the largest span's gap.  usage: python tools/ktrace_spans.py DIR [marker]"""
import csv
import os
import sys

rows = list(csv.DictReader(open(os.path.join(sys.argv[1], "run_kernel_trace.csv"))))
marker = sys.argv[2] if len(sys.argv) > 2 else "lstm_fwd_mfma_kernel"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
idx = [i for i, e in enumerate(ev) if marker in e[2]]
spans = sorted(((ev[b][0] - ev[a][0]) / 1e3, a, b) for a, b in zip(idx, idx[1:]))
print("%d spans; median %.1f us; largest:" % (len(spans), spans[len(spans) // 2][0]))
for s, a, b in spans[::-1][:6]:
    print("  %.1f us (kernels %d..%d)" % (s, a, b))
s, a, b = spans[-1]
gaps = sorted(((ev[i + 1][0] - ev[i][1]) / 1e3, i) for i in range(a, b))
for g, i in gaps[::-1][:4]:
    print("  gap %.1f us after %s -> %s" % (g, ev[i][2][:70], ev[i + 1][2][:70]))
