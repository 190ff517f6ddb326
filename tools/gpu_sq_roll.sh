# SQ counters of one kernel's launch, re-issued 20x by the eager bench (--pmc-target):
# usage: bash tools/gpu_sq_roll.sh "KERNEL NAME" [TAG]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $R/gpurun_out/sq_a$2 -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline --no-scaling-reference --no-real-data --pmc-target 20 --pmc-kernel "$1" > $R/gpurun_out/sq_a$2.json 2> $R/gpurun_out/sq_a$2.log || { echo SQ_A_FAIL; tail -5 $R/gpurun_out/sq_a$2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/sq_b$2 -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline --no-scaling-reference --no-real-data --pmc-target 20 --pmc-kernel "$1" > $R/gpurun_out/sq_b$2.json 2> $R/gpurun_out/sq_b$2.log || { echo SQ_B_FAIL; tail -5 $R/gpurun_out/sq_b$2.log; exit 1; }
echo done
