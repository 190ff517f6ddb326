# round 5: the rollout over batch sizes and its SQ counters; the real-data leg
# three times (host and device per-iteration spans)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
timeout -k 10 120 python tools/bench_kernels.py rollb > $O/rollb.txt 2>&1 || { echo ROLLB_FAIL; tail -20 $O/rollb.txt; exit 1; }
cat $O/rollb.txt
bash tools/gpu_sq_rollwaves.sh > $O/sqw.txt 2>&1 || { echo SQW_FAIL; tail -20 $O/sqw.txt; exit 1; }
tail -40 $O/sqw.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-legs --no-cpu-baseline --no-scaling-reference > $O/rd_$i.json 2> $O/rd_$i.err || { echo RD_FAIL; tail -20 $O/rd_$i.err; exit 1; }
  python - $O/rd_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["real_data"]["graphed_device_data_path"]
print("real graphed %.1f k  host med %.3f max %.3f  dev med %.3f max %.3f (idx %d) slowest host %s" % (
    r["value"] / 1e3, r["host_ms_median"], r["host_ms_max"], r["device_ms_median"], r["device_ms_max"],
    r["device_slowest_index"], r["slowest_iteration"]))
print("  host", r["host_ms_per_iteration"])
print("  dev ", r["device_ms_per_iteration"])
PY
done
