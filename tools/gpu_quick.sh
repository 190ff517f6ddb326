set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -x tools/mfma_probe ]; then timeout -k 10 60 ./tools/mfma_probe > gpurun_out/mfma_probe.txt 2>&1 || { echo PROBE_FAIL; exit 1; }; fi
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo tests_rc=$rc >> gpurun_out/gpu_tests.log
[ $rc -le 1 ] || { echo TESTS_CRASH; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; exit 1; }
echo done
