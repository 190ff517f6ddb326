# SQ counters of the bf16 pooling forward at configs[4]'s D shape (128 x 64-ped scenes)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_pool_bf16_pmc.sh r05 48 128 64 || exit 1
mkdir -p $R/gpurun_out/pbf_r05
for d in pa pb pc; do cp -r $R/gpurun_out/pbf_${d}_r05 $R/gpurun_out/pbf_r05/$d; done
python3 $R/tools/sq_by_grid.py $R/gpurun_out/pbf_r05 "pool_fwd_bf16_kernel<48, 4>" > $R/gpurun_out/pbf_r05/summary.json && cat $R/gpurun_out/pbf_r05/summary.json
