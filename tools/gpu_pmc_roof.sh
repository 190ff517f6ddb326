# the two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) of the eager bench
# re-issuing one kernel's main launch 20x.  usage: bash tools/gpu_pmc_roof.sh "KERNEL NAME"
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/p_$C -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline --no-scaling-reference --no-real-data --pmc-target 20 --pmc-kernel "$1" > $R/gpurun_out/p_$C.json 2> $R/gpurun_out/p_$C.log || { echo PMC_FAIL $C; tail -20 $R/gpurun_out/p_$C.log; exit 1; }
done
echo done
