# round-end evidence run: all GPU parity tests, smoke(), the default bench line
# (with the CPU baseline), rocprofv3 kernel trace + stats of the same bench, and
# two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) of an eager bench for
# the pool kernel's HBM traffic.  Every GPU step has its own time limit and the
# script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/f_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/f_tests.log; exit 1; }
tail -2 gpurun_out/f_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/f_smoke.log; exit 1; }
cat gpurun_out/f_smoke.log
timeout -k 10 400 python bench.py --steps 100 --warmup 10 > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/f_bench.err; exit 1; }
cat gpurun_out/f_bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/f_prof -o run -- python $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data > $R/gpurun_out/f_prof_bench.json 2> $R/gpurun_out/f_prof.err || { echo PROF_FAIL; tail -20 $R/gpurun_out/f_prof.err; exit 1; }
RK=$(python -c "import json; print(json.loads(open('$R/gpurun_out/f_bench.json').read().strip().splitlines()[-1])['roofline']['kernel'])")
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/f_pmc_fetch -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline --no-scaling-reference --no-real-data --pmc-target 20 --pmc-kernel "$RK" > $R/gpurun_out/f_pmc_fetch.json 2> $R/gpurun_out/f_pmc_fetch.log || { echo PMC_FETCH_FAIL; tail -20 $R/gpurun_out/f_pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/f_pmc_write -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline --no-scaling-reference --no-real-data --pmc-target 20 --pmc-kernel "$RK" > $R/gpurun_out/f_pmc_write.json 2> $R/gpurun_out/f_pmc_write.log || { echo PMC_WRITE_FAIL; tail -20 $R/gpurun_out/f_pmc_write.log; exit 1; }
echo done
