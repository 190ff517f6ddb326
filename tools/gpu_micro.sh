set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/mfma_rate > gpurun_out/mfma_rate.txt 2>&1 || { echo RATE_FAIL; exit 1; }
echo done
