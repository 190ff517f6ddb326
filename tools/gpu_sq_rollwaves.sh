# SQ counters of the best-of-k rollout kernel at one wave per SIMD (16,384
# sequences) and at 1,600 waves (25,600, the training shape): two --pmc passes
# of tools/bench_kernels.py roll2, summarised per launch grid by tools/sq_by_grid.py
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sqw
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $O/a -o run -- python $R/tools/bench_kernels.py roll2 > $O/a.log 2>&1 || { echo SQ_A_FAIL; tail -5 $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $O/b -o run -- python $R/tools/bench_kernels.py roll2 > $O/b.log 2>&1 || { echo SQ_B_FAIL; tail -5 $O/b.log; exit 1; }
python $R/tools/sq_by_grid.py $O lstm_fwd_mfma > $O/summary.json && cat $O/summary.json
