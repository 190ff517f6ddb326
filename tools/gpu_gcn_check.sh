# GCN-module tests, then the GCN legs and configs[4] with the current library
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gcn or configs or sgangat or 64ped or graph_module or family or evaluate" > gpurun_out/gcn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gcn_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gcn_tests.log | head -20; exit 1; }
for leg in configs2_gcn_fp32 configs2_gcn_bf16 configs4_sgangat_bf16; do
  timeout -k 10 300 python bench.py --leg $leg --steps 60 --no-cpu-baseline > gpurun_out/gl_$leg.json 2>/dev/null || { echo BENCH_FAIL $leg; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/gl_$leg.json').read().strip().splitlines()[-1]); print('$leg', d['value'], d['ms_per_step'], [(r['kernel'][5:30], round(r['avg_us'],1)) for r in d['launch_table'] if 'gcnmod' in r['kernel']])"
done
