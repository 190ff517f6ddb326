# kernel trace + stats of graph-replayed real-data training (zara1, batch 64)
# usage: bash tools/gpu_realdata_trace.sh TAG [gran] [pad] [caps]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rd_$1
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/realdata_graph_probe.py 40 ${2:-256} ${3:-32} ${4:-48,64} > $O/probe.txt 2> $O/prof.err || { echo PROF_FAIL; tail -20 $O/prof.err; exit 1; }
cat $O/probe.txt
python3 $R/tools/ktrace_iter.py $O/prof > $O/iteration_trace.txt 2>&1
tail -60 $O/iteration_trace.txt
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
rm -rf $O/prof
python3 - $O/kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print("%-70s %6s %8.1f %6.1f%%" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, 100 * float(r["TotalDurationNs"]) / tot))
PY
