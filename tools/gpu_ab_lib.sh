# A/B of builds of libsgg.so on the headline bench (tools/abx/libsgg_<v>.so,
# tools/build_ab.py), interleaved; prints each run's rate and the launches of
# the kernels matching the filter (from the bench's detail file)
# usage: bash tools/gpu_ab_lib.sh "kernel filter" rounds variant...
set -o pipefail
mkdir -p gpurun_out
filt=$1; n=$2; shift 2
for r in $(seq 1 $n); do
  for v in "$@"; do
    lib=$PWD/tools/abx/libsgg_$v.so; [ "$v" = head ] && lib=
    SGG_LIB=$lib SGG_BENCH_DETAIL=$PWD/gpurun_out/abl_$v.detail.json timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err || { echo BENCH_FAIL $v; tail -5 gpurun_out/abl_$v.err; exit 1; }
    python - gpurun_out/abl_$v.json "$v" "$filt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t = json.load(open(sys.argv[1].replace(".json", ".detail.json")))["launch_table"]
print(sys.argv[2], "value %.1f ms %.4f" % (d["value"], d["ms_per_step"]), [(r["kernel"][5:45], r["shape"][:2], round(r["avg_us"], 2)) for r in t if sys.argv[3] in r["kernel"]], flush=True)
PY
  done
done
