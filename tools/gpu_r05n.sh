# real-data stall probe (PaddedScenes.load split), new vs reused staging events;
# the LSTM backward+wgrad microbench over the ablation builds
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05n
mkdir -p $O
cd $R
for v in a NOHELP NOOWN; do
  SGG_LIB=$R/tools/ablib/libsgg_$v.so timeout -k 10 120 python tools/bench_kernels.py lbwd 2>&1 | grep -v amdgpu.ids || { echo LBWD_FAIL; exit 1; }
done
for e in 0 1 0 1; do
  PROBE_REUSE_EVENT=$e timeout -k 10 300 python tools/realdata_stall_probe.py 150 > $O/stall_$e.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/stall_$e.txt; exit 1; }
  head -30 $O/stall_$e.txt
done
