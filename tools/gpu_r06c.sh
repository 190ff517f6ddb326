set -o pipefail
mkdir -p gpurun_out/r06c
bash tools/gpu_lstm_probe.sh x3 > gpurun_out/r06c/probe.txt 2>&1 || { echo PROBE_FAIL; cat gpurun_out/r06c/probe.txt; exit 1; }
grep -A6 "== x3 2560" gpurun_out/r06c/probe.txt | head -3; grep -A5 "sub-phases" gpurun_out/r06c/probe.txt | head -6
timeout -k 10 400 python -u -m pytest tests/test_gpu_a_benched_path.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "lstm or benched or train_step or shared_prefix or encoder_projection or graphed or segments or paired" > gpurun_out/r06c/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r06c/tests.log; exit 1; }
tail -1 gpurun_out/r06c/tests.log
bash tools/gpu_ab_lib.sh lstm_mw_fwd 2 head f32
