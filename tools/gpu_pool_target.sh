# pooling chunk-plan target (SGG_POOL_TARGET_CHUNKS) A/B on the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for t in 512 256 384; do
    SGG_POOL_TARGET_CHUNKS=$t timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > gpurun_out/pt_$t.json 2> gpurun_out/pt_$t.err || { echo BENCH_FAIL; tail -5 gpurun_out/pt_$t.err; exit 1; }
    python - gpurun_out/pt_$t.json "$t" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value %.1f ms %.4f" % (d["value"], d["ms_per_step"]), [(r["kernel"][5:40], r["shape"][1], round(r["avg_us"], 2)) for r in d["launch_table"] if "pool_fwd" in r["kernel"]])
PY
  done
done
