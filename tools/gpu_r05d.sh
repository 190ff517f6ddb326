# round 5: every GPU test, the headline (launch table), the configs[4] leg
# with its launch table, PMC traffic of its bf16 pooling forward
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=${1:-r05d}
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
grep -o "{'eager_dp.*}" $O/tests.log || true
SGG_BENCH_TABLE=$O/head_table.txt timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > $O/head.json 2> $O/head.err || { echo HEAD_FAIL; tail -20 $O/head.err; exit 1; }
python -c "
import json; d = json.loads(open('$O/head.json').read().strip().splitlines()[-1])
print('HEAD value %.1f ms %.3f roof %s %.4f traffic %s' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic']))"
head -12 $O/head_table.txt
SGG_BENCH_TABLE=$O/c4_table.txt timeout -k 10 300 python bench.py --leg configs4_sgangat_bf16 --steps 50 --warmup 5 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -20 $O/c4.err; exit 1; }
python -c "
import json; d = json.loads(open('$O/c4.json').read().strip().splitlines()[-1])
print('C4 value %.1f ms %.3f roof %s %.4f' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))"
head -16 $O/c4_table.txt
bash tools/gpu_leg_pmc.sh $tag configs4_sgangat_bf16 "sgg::pool_fwd_bf16_kernel<48, 4>" || exit 1
python -c "
import json; t = json.load(open('$O/pmc_traffic.json'))
for k, v in t.items():
    if '|' in k: print(k, {a: b for a, b in v.items() if a != 'note'})"
