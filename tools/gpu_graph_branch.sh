set -o pipefail; mkdir -p gpurun_out; timeout -k 10 200 python -u tools/graph_branch_probe.py > gpurun_out/gb.txt 2>&1
