set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dense -o run -- python $R/tools/bench_kernels.py dense > $R/gpurun_out/prof_dense.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo done
