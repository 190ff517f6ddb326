# the world-1 RCCL worker (captured collectives) 8 times; stops at the first failure
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05r
mkdir -p $O
cd $R
for i in 1 2 3 4 5 6 7 8; do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + i)) RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 180 python tests/_nccl_world1_worker.py > $O/w_$i.log 2>&1 || { echo "RUN $i FAILED"; tail -5 $O/w_$i.log; exit 1; }
  echo "run $i: $(grep -c 'rank 0 OK' $O/w_$i.log) ok, watchdog messages: $(grep -ci 'watchdog\|CapturedEvent' $O/w_$i.log)"
done
