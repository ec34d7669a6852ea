#!/bin/bash
# flattened pair scatter: pair/kernel GPU tests, pair probe and headline A/B (FA_PAIR_FLAT=1 default vs 0)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/fl_tests.log 2>&1
timeout -k 10 300 python benchmarks/pair_probe.py --config T10I4D100M --modes 0,1 > gpurun_out/fl_probe1.txt 2>/dev/null
FA_PAIR_FLAT=0 timeout -k 10 300 python benchmarks/pair_probe.py --config T10I4D100M --modes 0,1 > gpurun_out/fl_probe0.txt 2>/dev/null
for v in 1 0 1 0; do
  FA_PAIR_FLAT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/fl_T10_$v.json 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/fl_T10_$v.json').read().strip().splitlines()[-1]);print('flat=$v', d['ms_per_step'])" >> gpurun_out/fl_summary.txt
done
