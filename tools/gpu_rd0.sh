# real-data leg: the first timed iteration's host time (2 runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-scaling-reference --no-legs > gpurun_out/rd0_$r.json 2> gpurun_out/rd0_$r.err || { echo BENCH_FAIL; tail -5 gpurun_out/rd0_$r.err; exit 1; }
  python - gpurun_out/rd0_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g = d["real_data"]["graphed_device_data_path"]
print("value", g["value"], "host max", g["host_ms_max"], "median", g["host_ms_median"], "slowest", g["slowest_iteration"]["index"], g["host_ms_per_iteration"][:4])
PY
done
