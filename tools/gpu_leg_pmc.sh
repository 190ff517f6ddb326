# PMC traffic of one kernel's main launch in one bench configuration: the two
# counter passes (FETCH_SIZE, WRITE_SIZE; separate runs, eager) re-issuing it
# 20x (bench.py --pmc-target), merged into gpurun_out/TAG/pmc_traffic.json.
# usage: bash tools/gpu_leg_pmc.sh TAG LEG|head "KERNEL"
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1; leg=$2; K=$3
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp
LA=""; [ "$leg" != head ] && LA="--leg $leg"
for C in FETCH_SIZE WRITE_SIZE; do
  c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${leg}_$c -o run -- python $R/bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs $LA --pmc-target 20 --pmc-kernel "$K" > $O/pmc_${leg}_$c.json 2> $O/pmc_${leg}_$c.log || { echo PMC_FAIL $leg $C; tail -20 $O/pmc_${leg}_$c.log; exit 1; }
done
python $R/tools/pmc_traffic.py $O/pmc_${leg}_fetch $O/pmc_${leg}_write $O/pmc_${leg}_fetch.json $O/pmc_traffic.json || { echo TRAFFIC_FAIL; exit 1; }
rm -rf $O/pmc_${leg}_fetch $O/pmc_${leg}_write
echo pmc done $leg
