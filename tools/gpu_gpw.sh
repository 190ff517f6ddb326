set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 1 2 4 8; do
cd /tmp && SGG_POOL_MAX_GPW=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_g$g -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_g$g.json 2>&1 || { echo FAIL; exit 1; }
done
echo done
