# all GPU tests, the LSTM backward microbench, the headline bench line (launch
# table), the real-data leg x2
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05p}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python tools/bench_kernels.py lbwd 2>&1 | grep -v amdgpu.ids || { echo LBWD_FAIL; exit 1; }
SGG_BENCH_TABLE=$O/head_table.txt timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-legs > $O/head.json 2> $O/head.err || { echo BENCH_FAIL; tail -20 $O/head.err; exit 1; }
python - $O/head.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("head value %.1f ms %.4f roof %s %.4f" % (d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"]))
r = d["real_data"]["graphed_device_data_path"]
print("real graphed %.1f k  host med %.3f max %.3f  dev med %.3f max %.3f slowest %s" % (
    r["value"] / 1e3, r["host_ms_median"], r["host_ms_max"], r["device_ms_median"], r["device_ms_max"], r["slowest_iteration"]))
PY
head -14 $O/head_table.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-legs --no-cpu-baseline --no-scaling-reference > $O/rd_$i.json 2> $O/rd_$i.err || { echo RD_FAIL; tail -20 $O/rd_$i.err; exit 1; }
  python - $O/rd_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["real_data"]["graphed_device_data_path"]
print("real graphed %.1f k  host med %.3f max %.3f  dev med %.3f max %.3f slowest %s" % (
    r["value"] / 1e3, r["host_ms_median"], r["host_ms_max"], r["device_ms_median"], r["device_ms_max"], r["slowest_iteration"]))
print("  host", r["host_ms_per_iteration"])
PY
done
