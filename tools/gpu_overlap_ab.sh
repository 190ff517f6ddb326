# Overlapped plan: its GPU tests, then the headline bench with SGG_OVERLAP 0 / 1
# (twice each, interleaved).  usage: bash tools/gpu_overlap_ab.sh TAG
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "overlap or graphed_trainer or pipelined" > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAIL; tail -60 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for v in 0 1 0 1; do
  SGG_OVERLAP=$v timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > gpurun_out/${tag}_$v.json 2> gpurun_out/${tag}_$v.err || { echo BENCH_FAIL; tail -20 gpurun_out/${tag}_$v.err; exit 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/${tag}_$v.json').read().strip().splitlines()[-1]); print('SGG_OVERLAP=$v value %.1f ms %.4f' % (d['value'], d['ms_per_step']))"
done
