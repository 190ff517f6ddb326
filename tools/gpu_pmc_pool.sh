# SQ counter passes (separate runs) over the roofline pool launch
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp_a -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -- python $R/tools/pool_one.py > $R/gpurun_out/pp_a.log 2>&1 || { echo PMC_A_FAIL; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp_b -o run --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE -- python $R/tools/pool_one.py > $R/gpurun_out/pp_b.log 2>&1 || { echo PMC_B_FAIL; exit 1; }
echo done
