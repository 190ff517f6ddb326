set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 400 python -u -m pytest tests/test_gpu_a_benched_path.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "lstm or benched or train_step or shared_prefix or encoder_projection or graphed or segments or paired" > gpurun_out/r06b/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r06b/tests.log; exit 1; }
tail -2 gpurun_out/r06b/tests.log
bash tools/gpu_ab_lib.sh lstm_mw_fwd 2 head f32
