# counter passes over the bf16 pooling forward (tools/pool_bf16_probe.py)
# usage: tools/gpu_pool_bf16_pmc.sh TAG BN S N
set -o pipefail
export TMPDIR=/tmp
tag=$1; bn=${2:-48}; S=${3:-128}; n=${4:-64}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 120 python3 $R/tools/pool_bf16_probe.py $bn $S $n 5 || exit 1
PREC=fp32 timeout -k 10 120 python3 $R/tools/pool_bf16_probe.py $bn $S $n 5 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pbf_pa_$tag -o run -- python3 $R/tools/pool_bf16_probe.py $bn $S $n 3 > $R/gpurun_out/pbf_pa_$tag.log 2>&1 || { echo PA_FAIL; tail -20 $R/gpurun_out/pbf_pa_$tag.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $R/gpurun_out/pbf_pb_$tag -o run -- python3 $R/tools/pool_bf16_probe.py $bn $S $n 3 > $R/gpurun_out/pbf_pb_$tag.log 2>&1 || { echo PB_FAIL; tail -20 $R/gpurun_out/pbf_pb_$tag.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pbf_pc_$tag -o run -- python3 $R/tools/pool_bf16_probe.py $bn $S $n 3 > $R/gpurun_out/pbf_pc_$tag.log 2>&1 || { echo PC_FAIL; tail -20 $R/gpurun_out/pbf_pc_$tag.log; exit 1; }
echo done
