# direct-RCCL captured all-reduce: the world-1 worker x6, then every GPU test
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R
for i in 1 2 3 4 5 6; do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + i)) RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 180 python tests/_nccl_world1_worker.py > $O/w_$i.log 2>&1 || { echo "RUN $i FAILED"; grep -v "^frame" $O/w_$i.log | tail -12; exit 1; }
  echo "run $i: $(grep -c 'rank 0 OK' $O/w_$i.log) ok, watchdog messages: $(grep -ci 'watchdog\|CapturedEvent' $O/w_$i.log)  $(grep allreduce $O/w_$i.log | cut -c1-200)"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
