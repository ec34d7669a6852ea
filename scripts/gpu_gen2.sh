#!/bin/bash
# gen chain grids: GPU kernel tests, T40I10D100M phase timing twice, headline
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gg_tests.log 2>&1
for i in 1 2; do
  FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/gg_T40_$i.json 2>/dev/null
done
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/gg_T40p.json 2>/dev/null
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/gg_T10.json 2>/dev/null
