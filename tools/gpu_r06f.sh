set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06f/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r06f/tests.log; exit 1; }
tail -1 gpurun_out/r06f/tests.log
bash tools/gpu_ab_lib.sh "lstm_mw\|gatenc" 2 head f32
