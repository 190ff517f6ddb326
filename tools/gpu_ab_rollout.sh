# A/B: the best-of-k rollout on the batch-MFMA kernel (default) vs the
# four-wave family (SGG_LSTM_NO_MFMA=1); bench headline, rollout launch time
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export SGG_LSTM_NO_MFMA=1; else unset SGG_LSTM_NO_MFMA; fi
  SGG_BENCH_TABLE=gpurun_out/ro_$v.txt timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > gpurun_out/ro_$v.json 2> gpurun_out/ro_$v.err || { echo BENCH_FAIL; tail -5 gpurun_out/ro_$v.err; exit 1; }
  python - gpurun_out/ro_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("no_mfma", sys.argv[2], "value %.1f ms %.4f" % (d["value"], d["ms_per_step"]), [(r["kernel"][5:40], r["shape"], round(r["avg_us"], 1)) for r in d["launch_table"] if "25600" in str(r["shape"])])
PY
done
