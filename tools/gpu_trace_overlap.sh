# kernel traces of the graphed bench with SGG_OVERLAP 0 and 1 -> iteration lists
# usage: bash tools/gpu_trace_overlap.sh TAG
set -o pipefail
export TMPDIR=/tmp
for v in 0 1; do
  O=gpurun_out/to_$1_$v
  mkdir -p $O
  SGG_OVERLAP=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-real-data --no-scaling-reference --no-legs > $O/bench.json 2> $O/prof.err || { echo PROF_FAIL; tail -20 $O/prof.err; exit 1; }
  python tools/ktrace_iter.py $O/prof > $O/iteration_trace.txt 2>&1
  find $O/prof -name "*kernel_trace.csv" -delete
  cat $O/iteration_trace.txt
done
