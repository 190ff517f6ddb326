# A/B of an environment toggle on one box: bench headline (+ real data) with
# and without the variable, alternating.  usage: bash tools/gpu_ab.sh TAG VAR=VALUE [extra bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
VAR=$2
shift 2
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --no-scaling-reference --steps 200 --warmup 20 "$@" > $O/base_$i.json 2> $O/base_$i.err || { echo BENCH_FAIL; tail -20 $O/base_$i.err; exit 1; }
  env $VAR timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --no-scaling-reference --steps 200 --warmup 20 "$@" > $O/var_$i.json 2> $O/var_$i.err || { echo BENCH_FAIL; tail -20 $O/var_$i.err; exit 1; }
done
python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f))
    rd = (d.get("real_data") or {}).get("graphed_device_data_path", {})
    print(os.path.basename(f), d["value"], d["ms_per_step"], rd.get("value"), rd.get("ms_per_iteration"))
PY
