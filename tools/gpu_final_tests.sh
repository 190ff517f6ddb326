# every GPU test and smoke() at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/final/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/final/tests.log; exit 1; }
tail -1 gpurun_out/final/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
