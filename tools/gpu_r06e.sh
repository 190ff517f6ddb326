set -o pipefail
mkdir -p gpurun_out/r06e
echo "== bwd probe"; timeout -k 10 60 tools/run/lstm_bwd_probe 2560 20 > gpurun_out/r06e/bwd_probe.txt || { echo PROBE_FAIL; exit 1; }
head -4 gpurun_out/r06e/bwd_probe.txt; tail -9 gpurun_out/r06e/bwd_probe.txt
for a in "2560 12 1 1" "2560 12 1 0"; do echo "== fwd probe $a"; timeout -k 10 60 tools/run/lstm_probe_x3 $a > gpurun_out/r06e/fwd_probe.txt || exit 1; grep -E "us/launch|step  [89] |end|wave" gpurun_out/r06e/fwd_probe.txt; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06e/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r06e/tests.log; exit 1; }
tail -1 gpurun_out/r06e/tests.log
bash tools/gpu_ab_lib.sh lstm 1 head
