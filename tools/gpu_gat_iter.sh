# GAT encoder iteration: phase probe + the GPU tests that touch the GAT encoder
# (then the whole -m gpu suite).  usage: bash tools/gpu_gat_iter.sh TAG [full]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 30 tools/permlane_probe > $O/permlane.txt 2>&1; cat $O/permlane.txt
timeout -k 10 60 tools/gatenc_probe_np 64 20 1 > $O/probe.txt 2>&1 || { echo PROBE_FAIL; cat $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "gat or generator or train or smoke" > $O/tests_gat.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests_gat.log | head -30; tail -30 $O/tests_gat.log; exit 1; }
tail -2 $O/tests_gat.log
if [ "$2" = full ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FULL_FAIL; tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
echo done
