# Do forked graph branches overlap under the HIP runtime's graph knobs?
# tools/fork_probe.py under the default, DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 and
# DEBUG_HIP_FORCE_GRAPH_QUEUES=4; then the headline bench under the first
# knob (its cost on a one-stream graph).  usage: bash tools/gpu_fork_env.sh TAG
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
for E in SGG_NONE=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4"; do
  echo "== $E"
  env $E timeout -k 10 120 python tools/fork_probe.py > gpurun_out/${tag}_fork.txt 2>&1 || { echo PROBE_FAIL; tail -5 gpurun_out/${tag}_fork.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/${tag}_fork.txt | tail -12
done
env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-scaling-reference --no-real-data --no-legs > gpurun_out/${tag}_pc0.json 2> gpurun_out/${tag}_pc0.err || { echo BENCH_FAIL; tail -5 gpurun_out/${tag}_pc0.err; exit 1; }
python -c "
import json; d = json.loads(open('gpurun_out/${tag}_pc0.json').read().strip().splitlines()[-1]); print('packet capture off: value %.1f ms %.4f' % (d['value'], d['ms_per_step']))"
