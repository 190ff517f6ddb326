# iteration run: GPU tests (optionally a -k filter) + the headline bench line
# (no CPU baseline / scaling / real-data legs).  usage: bash tools/gpu_quick.sh TAG [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread "${K[@]}" > gpurun_out/q_${tag}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/q_${tag}_tests.log; exit 1; }
tail -2 gpurun_out/q_${tag}_tests.log
SGG_BENCH_TABLE=gpurun_out/q_${tag}_table.txt timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data > gpurun_out/q_${tag}_bench.json 2> gpurun_out/q_${tag}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/q_${tag}_bench.err; exit 1; }
python - gpurun_out/q_${tag}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.1f  ms/step %.3f  roofline %s %.4f" % (d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"]))
for r in d["launch_table"][:40]:
    print("%-48s %-28s %4.1f %7.2f %7.1f" % (r["kernel"][:48], str(r["shape"])[:28], r["per_iter"], r["avg_us"], r["us_per_iter"]))
PY
