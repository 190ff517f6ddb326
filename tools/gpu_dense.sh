set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_kernels.py dense > gpurun_out/bench_dense.txt 2>&1 || { echo DENSE_FAIL; exit 1; }
bash tools/gpu_check.sh
