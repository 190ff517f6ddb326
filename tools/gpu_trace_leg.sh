# short rocprofv3 kernel trace of one graphed bench leg -> the iteration's launch list
# usage: bash tools/gpu_trace_leg.sh LEG TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tl_$2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --leg $1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/prof.err || { echo PROF_FAIL; tail -20 $O/prof.err; exit 1; }
python tools/ktrace_iter.py $O/prof > $O/iteration_trace.txt 2>&1
find $O/prof -name "*kernel_trace.csv" -delete
cat $O/iteration_trace.txt
