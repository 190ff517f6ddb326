"""Device timeline of steady-state training iterations from a rocprofv3
kernel trace: an iteration = the kernels from one launch of a marker kernel
(once per iteration) to the next; reports busy vs idle per iteration and the
largest gaps.  usage: python tools/ktrace_gaps.py DIR [marker]"""
import csv
import os
import re
import statistics
import sys

rows = list(csv.DictReader(open(os.path.join(sys.argv[1], "run_kernel_trace.csv"))))
marker = sys.argv[2] if len(sys.argv) > 2 else "lstm_fwd_mfma_kernel"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.search(r"((sgg|at::native)::[A-Za-z_0-9:]+(<[^()]{0,40})?)", n)
    return (m.group(1) if m else n)[:50]


idx = [i for i, e in enumerate(ev) if marker in e[2]]
its = []
for a, b in zip(idx, idx[1:]):
    span = ev[b][0] - ev[a][0]
    if span < 3e6:   # < 3 ms: back-to-back iterations
        its.append((a, b, span))
n_per = statistics.median([b - a for a, b, _ in its])
its = [t for t in its if t[1] - t[0] == n_per]
print("%d steady iterations of %d kernels; span median %.1f us" % (len(its), n_per,
                                                                  statistics.median(t[2] for t in its) / 1e3))
a, b, span = sorted(its, key=lambda t: t[2])[len(its) // 2]
seg = ev[a:b + 1]
busy = sum(e - s for s, e, _ in seg[:-1])
gaps = [(y[0] - x[1], short(x[2]), short(y[2])) for x, y in zip(seg, seg[1:])]
print("median iteration: span %.1f us, kernel time %.1f us, idle %.1f us; gaps > 0: %d (mean %.2f us)" % (
    span / 1e3, busy / 1e3, sum(max(g, 0) for g, _, _ in gaps) / 1e3, sum(g > 0 for g, _, _ in gaps),
    statistics.mean([g for g, _, _ in gaps if g > 0]) / 1e3))
for g, x, y in sorted(gaps, key=lambda t: -t[0])[:12]:
    print("%7.2f us  %s -> %s" % (g / 1e3, x, y))
if len(sys.argv) > 3:
    for (s, e, nm), (g, _, _) in zip(seg, gaps + [(0, 0, 0)]):
        print("%7.2f  +%5.2f  %s" % ((e - s) / 1e3, g / 1e3, short(nm)))
