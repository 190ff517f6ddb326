# GAT / sgangat / configs GPU tests, then the configs[4] leg with the current library
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gat or sgangat or graph_module or 64ped or configs" > gpurun_out/gat_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gat_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/gat_tests.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --leg configs4_sgangat_bf16 --steps 40 --no-cpu-baseline > gpurun_out/gc4.json 2> gpurun_out/gc4.err || { tail -20 gpurun_out/gc4.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/gc4.json').read().strip().splitlines()[-1]); print('configs4', d['value'], d['ms_per_step'])"
