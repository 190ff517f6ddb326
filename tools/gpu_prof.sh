# quick perf loop: bench (no CPU baseline) under rocprofv3 kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo BENCH_FAIL; exit 1; }
echo done
