# GAT encoder forward: per-lane group masks (A/B of the probes) + GAT GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_gat_ab.sh || exit 1
TAG=r05gm timeout -k 10 600 bash tools/gpu_tests_k.sh "gat or group or train_step or bucket or gcn" | tail -3 || { echo TESTS_FAIL; exit 1; }
