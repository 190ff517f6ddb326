# GAT encoder diagnosis: the phase probe (workgroup 0's wall clock per phase,
# 64 x 20-ped scenes, 1 head; tools/gatenc_probe, built on the CPU beforehand)
# and the SQ counters of both directions of the fused kernel as the bench
# issues them (two --pmc passes each, tools/gpu_sq_roll.sh).
# usage: bash tools/gpu_gatenc_explain.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 60 $R/tools/gatenc_probe 64 20 1 > $O/probe.txt 2>&1 || { echo PROBE_FAIL; cat $O/probe.txt; exit 1; }
cat $O/probe.txt
for K in "sgg::gatenc_kernel<false>" "sgg::gatenc_kernel<true>"; do
  t=$(echo "$K" | tr -dc "a-z" | sed s/sgg//)
  bash $R/tools/gpu_sq_roll.sh "$K" _$1_$t || exit 1
done
echo done
