set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "lstm or generator or discriminator" > gpurun_out/gpu_lstm_tests.log 2>&1; rc=$?; echo tests_rc=$rc >> gpurun_out/gpu_lstm_tests.log
[ $rc -le 1 ] || { echo TESTS_CRASH; exit 1; }
timeout -k 10 300 python tools/bench_kernels.py lstm > gpurun_out/bench_lstm.txt 2>&1 || { echo LSTMBENCH_FAIL; exit 1; }
echo done
