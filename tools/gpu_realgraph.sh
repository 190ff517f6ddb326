# graph-replayed real-data path: parameter sweep + kernel trace of the default
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
tag=${1:-a}
cd $R
for cfg in "256 32 48,64" "128 32 48,64" "128 16 48,64" "256 32 64" "128 16 64"; do
  timeout -k 10 120 python -u tools/realdata_graph_probe.py 40 $cfg >> gpurun_out/rg_$tag.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/rg_$tag.log; exit 1; }
done
cat gpurun_out/rg_$tag.log | grep gran
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rg_kt_$tag -o run -- python3 $R/tools/realdata_graph_probe.py 40 > $R/gpurun_out/rg_kt_$tag.log 2>&1 || { echo KT_FAIL; tail -20 $R/gpurun_out/rg_kt_$tag.log; exit 1; }
echo done
