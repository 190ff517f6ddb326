# A/B of two builds of libsgg.so on the headline bench (tools/ab/libsgg_{a,b}.so), interleaved
# usage: bash tools/gpu_ab_lib.sh [kernel filter] [rounds]
set -o pipefail
mkdir -p gpurun_out
filt=${1:-lstm_mw_fwd}; n=${2:-2}
for r in $(seq 1 $n); do
  for v in a b; do
    SGG_LIB=$PWD/tools/ab/libsgg_$v.so timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err || { echo BENCH_FAIL; tail -5 gpurun_out/abl_$v.err; exit 1; }
    python - gpurun_out/abl_$v.json "$v" "$filt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value %.1f ms %.4f" % (d["value"], d["ms_per_step"]), [(r["kernel"][5:45], r["shape"][1], round(r["avg_us"], 2)) for r in d["launch_table"] if sys.argv[3] in r["kernel"]])
PY
  done
done
