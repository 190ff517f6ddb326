# iteration GPU loop: parity tests (-k "$1"), bench without the CPU leg, rocprofv3
# kernel trace + stats, and the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v ${1:+-k "$1"} -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/i_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/i_tests.log; exit 1; }
tail -2 gpurun_out/i_tests.log
timeout -k 10 400 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/i_bench.json 2> gpurun_out/i_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/i_bench.err; exit 1; }
cat gpurun_out/i_bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/i_prof -o run -- python $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $R/gpurun_out/i_prof_bench.json 2> $R/gpurun_out/i_prof.err || { echo PROF_FAIL; tail -20 $R/gpurun_out/i_prof.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/i_pmc_fetch -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline > $R/gpurun_out/i_pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAIL; tail -20 $R/gpurun_out/i_pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/i_pmc_write -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline > $R/gpurun_out/i_pmc_write.log 2>&1 || { echo PMC_WRITE_FAIL; tail -20 $R/gpurun_out/i_pmc_write.log; exit 1; }
echo done
