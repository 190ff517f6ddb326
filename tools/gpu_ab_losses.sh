set -o pipefail
mkdir -p gpurun_out
for v in 0 1 0 1; do
SGG_DEFER_LOSSES=$v SGG_BENCH_TABLE=gpurun_out/ab_$v.txt timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo BENCH_FAIL; tail -5 gpurun_out/ab_$v.err; exit 1; }
python - gpurun_out/ab_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("defer", sys.argv[2], "value %.1f ms %.4f" % (d["value"], d["ms_per_step"]), [ (r["kernel"][5:30], round(r["avg_us"],1)) for r in d["launch_table"] if "finish" in r["kernel"] or "bce" in r["kernel"] or "l2_" in r["kernel"]])
PY
done
