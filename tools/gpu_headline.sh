# default bench line (every leg, real data, CPU baseline) + a short kernel
# trace of the headline's iteration.  usage: bash tools/gpu_headline.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hl_$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline %.1f %s  ms/step %.4f  roofline %s %.3f  iteration %s" % (d["value"], d["unit"], d["ms_per_step"], d["roofline"].get("kernel"), d["roofline"]["frac"], d["roofline"].get("iteration")))
for l in d.get("legs", []):
    print("leg %-26s %10.1f  ms %.4f  %s %.3f" % (l["config"], l["value"], l["ms_per_step"], l["roofline"].get("kernel"), l["roofline"]["frac"]))
print("real_data", json.dumps(d.get("real_data"))[:600])
print("scaling_reference", json.dumps(d.get("scaling_reference"))[:300])
print("cpu_baseline", json.dumps(d.get("cpu_baseline"))[:300])
PY
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-real-data --no-scaling-reference --no-legs > $O/prof_bench.json 2> $O/prof.err || { echo PROF_FAIL; tail -20 $O/prof.err; exit 1; }
python3 $R/tools/ktrace_iter.py $O/prof > $O/iteration_trace.txt 2>&1
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
rm -rf $O/prof
tail -50 $O/iteration_trace.txt
