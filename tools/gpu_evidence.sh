# Round evidence at HEAD: every GPU test, smoke(), the default bench line (with
# the CPU baseline, the BASELINE legs and the real-data leg), a rocprofv3
# kernel trace + stats of the same bench, and the two PMC passes (FETCH_SIZE,
# WRITE_SIZE; separate runs, eager) re-issuing the dominant kernel's main launch
# of the headline and of every leg -> the traffic table.  Each GPU step has its
# own time limit; the script stops at the first failure.
# usage: [PMC=0] [LEGS="head ..."] bash tools/gpu_evidence.sh TAG   (PMC=0: no PMC passes)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
SGG_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 400 python bench.py --steps 100 --warmup 10 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-real-data --no-scaling-reference --no-legs > $O/prof_bench.json 2> $O/prof.err || { echo PROF_FAIL; tail -20 $O/prof.err; exit 1; }
[ "${PMC:-1}" = 1 ] && for leg in ${LEGS:-head configs3_shard512 configs2_gcn_fp32 configs2_gcn_bf16 configs4_sgangat_bf16}; do
  K=$(python -c "
import json; d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
legs = {l['config']: l for l in d.get('legs', [])}
print(d['roofline']['kernel'] if '$leg' == 'head' else legs['$leg']['roofline']['kernel'])")
  LA=""; [ "$leg" != head ] && LA="--leg $leg"
  for C in FETCH_SIZE WRITE_SIZE; do
    c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${leg}_$c -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs $LA --pmc-target 20 --pmc-kernel "$K" > $O/pmc_${leg}_$c.json 2> $O/pmc_${leg}_$c.log || { echo PMC_FAIL $leg $C; tail -20 $O/pmc_${leg}_$c.log; exit 1; }
  done
  python $R/tools/pmc_traffic.py $O/pmc_${leg}_fetch $O/pmc_${leg}_write $O/pmc_${leg}_fetch.json $O/pmc_traffic.json || { echo TRAFFIC_FAIL $leg; exit 1; }
done
# keep what is judged, drop the raw traces (gpurun copies back <= 64 MiB)
python $R/tools/ktrace_iter.py $O/prof > $O/iteration_trace.txt 2>&1 || true
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
rm -rf $O/prof $O/pmc_*_fetch $O/pmc_*_write
echo done
