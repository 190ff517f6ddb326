# GAT encoder backward: the saved state + dy loaded in one batched round trip
# (segs_from_global); phase probe, un-instrumented probe, GAT GPU tests, headline
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05gb}
mkdir -p $O
cd $R
echo "== gatenc_probe"; timeout -k 10 60 tools/bin/gatenc_probe 64 20 1 | grep -A16 "^bwd" || { echo PROBE_FAIL; exit 1; }
echo "== gatenc_probe_np"; timeout -k 10 60 tools/bin/gatenc_probe_np 64 20 1 | grep "us/launch" || { echo PROBE_FAIL; exit 1; }
TAG=$(basename $O) timeout -k 10 600 bash tools/gpu_tests_k.sh "gat or train_step or bucket" | tail -4 || { echo TESTS_FAIL; exit 1; }
SGG_BENCH_TABLE=$O/head_table.txt timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-legs --no-real-data > $O/head.json 2> $O/head.err || { echo BENCH_FAIL; tail -20 $O/head.err; exit 1; }
python - $O/head.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("head value %.1f ms %.4f" % (d["value"], d["ms_per_step"]))
PY
grep "gatenc" $O/head_table.txt
