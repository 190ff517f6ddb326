# quick bench line (headline only) + a kernel trace of the same command
# usage: bash tools/gpu_quickprof.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --no-scaling-reference --steps 100 --warmup 10 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-real-data --no-scaling-reference --no-legs > $O/prof_bench.json 2> $O/prof.err || { echo PROF_FAIL; tail -20 $O/prof.err; exit 1; }
echo done
