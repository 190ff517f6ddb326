# real-data leg x3 with host diagnostics (run-queue wait, cgroup throttling)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05g
mkdir -p $O
cd $R
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-legs --no-cpu-baseline --no-scaling-reference > $O/rd_$i.json 2> $O/rd_$i.err || { echo RD_FAIL; tail -20 $O/rd_$i.err; exit 1; }
  python - $O/rd_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["real_data"]["graphed_device_data_path"]
print("real graphed %.1f k  host med %.3f max %.3f  dev med %.3f max %.3f (idx %d) runq %.3f throttled %s slowest %s" % (
    r["value"] / 1e3, r["host_ms_median"], r["host_ms_max"], r["device_ms_median"], r["device_ms_max"],
    r["device_slowest_index"], r["runqueue_wait_ms_total"], r["cgroup_throttled_ms_total"], r["slowest_iteration"]))
print("  host", r["host_ms_per_iteration"])
PY
done
