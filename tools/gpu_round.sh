# round GPU loop: parity tests (all, or -k "$1"), kernel A/B micro-benchmarks,
# bench (100 steps), rocprofv3 kernel trace + stats of a short bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > gpurun_out/r_tests.log 2>&1; rc=$?
else
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r_tests.log 2>&1; rc=$?
fi
echo tests_rc=$rc >> gpurun_out/r_tests.log
[ $rc -eq 0 ] || { echo TESTS_FAIL; tail -40 gpurun_out/r_tests.log; exit 1; }
tail -3 gpurun_out/r_tests.log
timeout -k 10 300 python tools/bench_kernels.py ab > gpurun_out/r_kernels.txt 2>&1 || { echo KB_FAIL; tail -20 gpurun_out/r_kernels.txt; exit 1; }
cat gpurun_out/r_kernels.txt
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r_bench.json 2> gpurun_out/r_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r_bench.err; exit 1; }
cat gpurun_out/r_bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err || { echo PROF_FAIL; exit 1; }
echo done
