# A/B of one environment knob on the headline bench: bash tools/gpu_ab_env.sh VAR "v1 v2 ..." [kernel filter]
set -o pipefail
mkdir -p gpurun_out
var=$1; vals=$2; filt=${3:-lstm_mw_fwd_kernel<32}
for v in $vals; do
  env $var=$v timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > gpurun_out/abe_$v.json 2> gpurun_out/abe_$v.err || { echo BENCH_FAIL; tail -5 gpurun_out/abe_$v.err; exit 1; }
  python - gpurun_out/abe_$v.json "$var=$v" "$filt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value %.1f ms %.4f" % (d["value"], d["ms_per_step"]), [(r["kernel"][5:45], r["shape"][1], round(r["avg_us"], 2)) for r in d["launch_table"] if sys.argv[3] in r["kernel"]])
PY
done
