# generator pooling at two pair groups per wave: pooling / train-step GPU
# tests, the headline + legs bench line, a short kernel trace
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05pt}
mkdir -p $O
cd $R
TAG=$(basename $O) timeout -k 10 600 bash tools/gpu_tests_k.sh "pool or train_step or bucket or gcn or gat" | tail -3 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 400 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("head value %.1f ms %.4f" % (d["value"], d["ms_per_step"]))
for l in d.get("legs", []): print(l["config"], l["value"], l["ms_per_step"])
PY
bash tools/gpu_trace_quick.sh $(basename $O) | tail -3
