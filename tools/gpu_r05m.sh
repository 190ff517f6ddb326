# A/B of two libsgg.so builds (tools/ablib/libsgg_{a,b}.so, interleaved) on the
# headline bench, then the real-data leg x4 with the per-phase host breakdown
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05m}
mkdir -p $O
cd $R
filt=${FILT:-lstm_mw_bwd}
for r in 1 2; do
  for v in a b; do
    SGG_LIB=$R/tools/ablib/libsgg_$v.so timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > $O/ab_$v$r.json 2> $O/ab_$v$r.err || { echo BENCH_FAIL; tail -5 $O/ab_$v$r.err; exit 1; }
    python - $O/ab_$v$r.json "$v" "$filt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value %.1f ms %.4f" % (d["value"], d["ms_per_step"]), [(r["kernel"][5:45], r["shape"][1], round(r["avg_us"], 2)) for r in d["launch_table"] if any(f in r["kernel"] for f in sys.argv[3].split(","))])
PY
  done
done
[ "${RD:-1}" = 1 ] || exit 0
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-legs --no-cpu-baseline --no-scaling-reference > $O/rd_$i.json 2> $O/rd_$i.err || { echo RD_FAIL; tail -20 $O/rd_$i.err; exit 1; }
  python - $O/rd_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["real_data"]["graphed_device_data_path"]
print("real graphed %.1f k  host med %.3f max %.3f  dev med %.3f max %.3f allocs %s slowest %s" % (
    r["value"] / 1e3, r["host_ms_median"], r["host_ms_max"], r["device_ms_median"], r["device_ms_max"],
    r.get("device_allocs_timed"), r["slowest_iteration"]))
PY
done
