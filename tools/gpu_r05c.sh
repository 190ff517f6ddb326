# round 5: the nccl world-1 DP test + draw/lifetime tests, the configs[4] leg
# with its launch table, PMC traffic of its bf16 pooling forward
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "nccl_world1 or draw_source or decoder_init_rejects or in_a_cycle or native_loaded or bf16" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
grep -o "{'eager_dp.*}" $O/tests.log || true
SGG_BENCH_TABLE=$O/c4_table.txt timeout -k 10 300 python bench.py --leg configs4_sgangat_bf16 --steps 50 --warmup 5 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -20 $O/c4.err; exit 1; }
head -30 $O/c4_table.txt
bash tools/gpu_leg_pmc.sh r05c configs4_sgangat_bf16 "sgg::pool_fwd_bf16_kernel<48, 4>" || exit 1
python -c "
import json; t = json.load(open('$O/pmc_traffic.json'))
for k, v in t.items():
    if '|' in k: print(k, {a: b for a, b in v.items() if a != 'note'})"
