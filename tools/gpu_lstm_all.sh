set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
tag=${1:-a}
cd /tmp
SGG_LSTM_MW=all timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lstm_all_$tag -o run -- python3 $R/tools/lstm_probe.py 20 > $R/gpurun_out/lstm_all_$tag.log 2>&1 || { echo KT_FAIL; tail -20 $R/gpurun_out/lstm_all_$tag.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/lstm_pa_$tag -o run -- python3 $R/tools/lstm_probe.py 5 > $R/gpurun_out/lstm_pa_$tag.log 2>&1 || { echo PA_FAIL; tail -20 $R/gpurun_out/lstm_pa_$tag.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $R/gpurun_out/lstm_pb_$tag -o run -- python3 $R/tools/lstm_probe.py 5 > $R/gpurun_out/lstm_pb_$tag.log 2>&1 || { echo PB_FAIL; tail -20 $R/gpurun_out/lstm_pb_$tag.log; exit 1; }
echo done
