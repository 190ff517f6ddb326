# GAT encoder backward, branch-free batched preload: phase probe, GAT GPU
# tests, a short kernel trace of the graphed bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05gc}
mkdir -p $O
cd $R
echo "== gatenc_probe"; timeout -k 10 60 tools/bin/gatenc_probe 64 20 1 || { echo PROBE_FAIL; exit 1; }
TAG=$(basename $O) timeout -k 10 600 bash tools/gpu_tests_k.sh "gat or train_step or bucket" | tail -3 || { echo TESTS_FAIL; exit 1; }
bash tools/gpu_trace_quick.sh $(basename $O) | tail -14
