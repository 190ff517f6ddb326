# LSTM forward with the Wu prefetch spread over the steps: LSTM / pooling /
# train-step GPU tests, a short kernel trace of the graphed bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05lw}
mkdir -p $O
cd $R
TAG=$(basename $O) timeout -k 10 600 bash tools/gpu_tests_k.sh "lstm or pool or train_step or bucket or encoder" | tail -3 || { echo TESTS_FAIL; exit 1; }
bash tools/gpu_trace_quick.sh $(basename $O) | tail -34
