set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06d/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r06d/tests.log; exit 1; }
tail -1 gpurun_out/r06d/tests.log
bash tools/gpu_ab_lib.sh lstm_mw_fwd 2 head f32
