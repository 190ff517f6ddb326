"""Where the host thread spends the slowest graphed real-data iterations:
rocprofv3 --sys-trace CSVs of tools/realdata_graph_probe.py (SGG_PROBE_MARKS
= the per-iteration CLOCK_MONOTONIC windows) -> for the slowest iterations,
the HIP API calls inside the window (longest first), the largest gaps between
consecutive calls of the main thread (time spent outside the HIP runtime:
Python, the allocator, the collector), and the kernels / copies in it.
usage: python tools/systrace_stall.py TRACE_DIR MARKS_JSON [n_slowest]"""
import csv
import glob
import json
import os
import sys


def load(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main():
    d, marks = sys.argv[1], json.load(open(sys.argv[2]))
    nslow = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    api = load(d, "*hip_api_trace.csv")
    kern = load(d, "*kernel_trace.csv")
    cpy = load(d, "*memory_copy_trace.csv")
    if not api:
        print("no hip_api_trace.csv under", d)
        return
    # the main thread: the one with most API calls
    by_tid = {}
    for r in api:
        by_tid.setdefault(r["Thread_Id"], []).append(r)
    main_tid = max(by_tid, key=lambda k: len(by_tid[k]))
    calls = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in by_tid[main_tid]))
    med = sorted(m["host_ms"] for m in marks)[len(marks) // 2]
    print("%d iterations, host median %.3f ms; threads with API calls: %s (main %s)"
          % (len(marks), med, {k: len(v) for k, v in by_tid.items()}, main_tid))
    for m in sorted(marks, key=lambda m: -m["host_ms"])[:nslow]:
        a, b = m["start_ns"], m["end_ns"]
        inside = [c for c in calls if c[1] > a and c[0] < b]
        print("\niteration %d: %.3f ms host, bucket %s, %s earlier replays; %d HIP calls"
              % (m["index"], m["host_ms"], m["bucket"], m["prior_replays"], len(inside)))
        tot = {}
        for s, e, f in inside:
            tot[f] = tot.get(f, 0) + (min(e, b) - max(s, a))
        for f, t in sorted(tot.items(), key=lambda x: -x[1])[:8]:
            print("   %-40s %8.3f ms total" % (f, t / 1e6))
        for s, e, f in sorted(inside, key=lambda c: c[0] - c[1])[:5]:
            print("   longest: %-32s %8.3f ms at +%.3f ms" % (f, (e - s) / 1e6, (s - a) / 1e6))
        pts = [a] + [x for c in inside for x in (c[0], c[1])] + [b]
        gaps = sorted(((pts[i + 1] - pts[i], pts[i]) for i in range(0, len(pts) - 1, 2)), reverse=True)[:4]
        for g, at in gaps:
            print("   host gap outside HIP %.3f ms at +%.3f ms" % (g / 1e6, (at - a) / 1e6))
        ks = [r for r in kern if int(r["Start_Timestamp"]) < b and int(r["End_Timestamp"]) > a]
        cs = [r for r in cpy if int(r["Start_Timestamp"]) < b and int(r["End_Timestamp"]) > a]
        print("   kernels in window %d, copies %d" % (len(ks), len(cs)))


if __name__ == "__main__":
    main()
