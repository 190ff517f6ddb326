# A/B of two builds of libsgg.so (tools/ab/libsgg_{a,b}.so) on the full bench
# line (headline, legs, real data; no CPU baseline / scaling reference)
# usage: bash tools/gpu_ab_lib_full.sh [kernel filter]
set -o pipefail
mkdir -p gpurun_out
filt=${1:-pool_bwd}
for v in a b; do
  SGG_LIB=$PWD/tools/ab/libsgg_$v.so timeout -k 10 400 python bench.py --steps 60 --no-cpu-baseline --no-scaling-reference > gpurun_out/abf_$v.json 2> gpurun_out/abf_$v.err || { echo BENCH_FAIL; tail -5 gpurun_out/abf_$v.err; exit 1; }
  python - gpurun_out/abf_$v.json "$v" "$filt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "headline %.1f ms %.4f" % (d["value"], d["ms_per_step"]), [(r["kernel"][5:45], r["shape"][1], round(r["avg_us"], 2)) for r in d["launch_table"] if sys.argv[3] in r["kernel"]])
for l in d.get("legs", []):
    print("   leg %-26s %10.1f  ms %.4f" % (l["config"], l["value"], l["ms_per_step"]))
rd = d.get("real_data") or {}
g = rd.get("graphed_device_data_path") or {}
print("   real_data", g.get("value"), g.get("ms_per_iteration"))
PY
done
