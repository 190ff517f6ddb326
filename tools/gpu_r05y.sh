# all GPU tests, the LSTM backward microbench, the headline bench line
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05y}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" $O/tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo TESTS_CRASH $rc; tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 python tools/bench_kernels.py ${KMODE:-lbwd} 2>&1 | grep -v amdgpu.ids || { echo KB_FAIL; exit 1; }
SGG_BENCH_TABLE=$O/head_table.txt timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-legs --no-real-data > $O/head.json 2> $O/head.err || { echo BENCH_FAIL; tail -20 $O/head.err; exit 1; }
python - $O/head.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("head value %.1f ms %.4f roof %s %.4f" % (d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"]))
PY
grep "lstm" $O/head_table.txt
