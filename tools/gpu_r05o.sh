# bucketed real-data tests + stall probe with the scene-structure copy inside
# the graph; LSTM backward ablations (tools/ablib)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05o
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "bucket or padded or real" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in a L2HIT NOFBP NOACC; do
  SGG_LIB=$R/tools/ablib/libsgg_$v.so timeout -k 10 120 python tools/bench_kernels.py lbwd 2>&1 | grep -v amdgpu.ids | head -2 || { echo LBWD_FAIL; exit 1; }
done
for e in 1 2; do
  timeout -k 10 300 python tools/realdata_stall_probe.py 150 > $O/stall_$e.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/stall_$e.txt; exit 1; }
  head -24 $O/stall_$e.txt
done
