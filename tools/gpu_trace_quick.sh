# short rocprofv3 kernel trace of the graphed bench -> the iteration's launch list
# usage: bash tools/gpu_trace_quick.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tq_$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-real-data --no-scaling-reference --no-legs > $O/bench.json 2> $O/prof.err || { echo PROF_FAIL; tail -20 $O/prof.err; exit 1; }
python tools/ktrace_iter.py $O/prof > $O/iteration_trace.txt 2>&1
find $O/prof -name "*kernel_trace.csv" -delete
cat $O/iteration_trace.txt
