set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/launch_probe.py > gpurun_out/lp.txt 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python tools/launch_probe.py >> gpurun_out/lp.txt 2>&1 || exit 1
DEBUG_HIP_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python tools/launch_probe.py >> gpurun_out/lp.txt 2>&1 || exit 1
DEBUG_HIP_GRAPH_PACKET_CAPTURE=1 timeout -k 10 120 python tools/launch_probe.py >> gpurun_out/lp.txt 2>&1 || exit 1
AMD_SERIALIZE_KERNEL=0 HIP_LAUNCH_BLOCKING=0 timeout -k 10 120 python tools/launch_probe.py >> gpurun_out/lp.txt 2>&1 || exit 1
env | grep -E "^(HIP|GPU|AMD|HSA|ROC)" >> gpurun_out/lp.txt
