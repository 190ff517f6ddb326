set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "pool or generator or evaluate" > gpurun_out/gpu_pool_tests.log 2>&1; rc=$?; echo tests_rc=$rc >> gpurun_out/gpu_pool_tests.log
[ $rc -le 1 ] || { echo TESTS_CRASH; exit 1; }
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_pool.txt 2>&1 || { echo POOLBENCH_FAIL; exit 1; }
echo done
