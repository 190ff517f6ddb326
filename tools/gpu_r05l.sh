# bf16 pool tests + configs[4] leg (launch table)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05l
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "bf16 or pool" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SGG_BENCH_TABLE=$O/c4_table.txt timeout -k 10 300 python bench.py --leg configs4_sgangat_bf16 --steps 50 --warmup 5 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -20 $O/c4.err; exit 1; }
python -c "
import json; d = json.loads(open('$O/c4.json').read().strip().splitlines()[-1])
print('C4 value %.1f ms %.3f roof %s %.4f' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))"
grep pool_fwd_bf16 $O/c4_table.txt
