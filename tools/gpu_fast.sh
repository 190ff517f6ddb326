# quick GPU loop: selected parity tests (-k expr in $1) + bench (no CPU baseline) + kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > gpurun_out/fast_tests.log 2>&1; rc=$?
  echo tests_rc=$rc >> gpurun_out/fast_tests.log
  [ $rc -eq 0 ] || { echo TESTS_FAIL; tail -30 gpurun_out/fast_tests.log; exit 1; }
fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/fast_bench.json 2> gpurun_out/fast_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/fast_bench.err; exit 1; }
cat gpurun_out/fast_bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err || { echo PROF_FAIL; exit 1; }
echo done
