# discriminator head backward with its X operands hoisted: head / BCE /
# train-step GPU tests, a short kernel trace
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05hd}
mkdir -p $O
cd $R
TAG=$(basename $O) timeout -k 10 600 bash tools/gpu_tests_k.sh "head or bce or train_step or bucket or discriminator" | tail -3 || { echo TESTS_FAIL; exit 1; }
bash tools/gpu_trace_quick.sh $(basename $O) | tail -34
