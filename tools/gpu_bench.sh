# bench evidence run: default bench line (CPU baseline, scaling reference),
# rocprofv3 kernel trace + stats of the same command, and two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs) targeting the dominant kernel.
# usage: tools/gpu_bench.sh TAG [STEPS]
set -o pipefail
export TMPDIR=/tmp
tag=$1
steps=${2:-50}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u bench.py --steps $steps --warmup 10 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$tag -o run -- python3 $R/bench.py --steps $steps --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data > $R/gpurun_out/prof_bench_$tag.json 2> $R/gpurun_out/prof_$tag.err || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_$tag.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_$tag -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-scaling-reference --no-real-data --pmc-target 20 > $R/gpurun_out/pmcf_bench_$tag.json 2> $R/gpurun_out/pmcf_$tag.err || { echo PMC_FETCH_FAIL; tail -20 $R/gpurun_out/pmcf_$tag.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_$tag -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-scaling-reference --no-real-data --pmc-target 20 > $R/gpurun_out/pmcw_bench_$tag.json 2> $R/gpurun_out/pmcw_$tag.err || { echo PMC_WRITE_FAIL; tail -20 $R/gpurun_out/pmcw_$tag.err; exit 1; }
echo done
