# LSTM tests (every H, both directions, vs the oracle) + kernel trace of the probe
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
tag=${1:-a}
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "lstm or train_step" > gpurun_out/lstmq_tests_$tag.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/lstmq_tests_$tag.log; exit 1; }
tail -2 gpurun_out/lstmq_tests_$tag.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lstm_kt_$tag -o run -- python3 $R/tools/lstm_probe.py 20 > $R/gpurun_out/lstm_kt_$tag.log 2>&1 || { echo KT_FAIL; tail -20 $R/gpurun_out/lstm_kt_$tag.log; exit 1; }
echo done
