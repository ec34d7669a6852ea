#!/bin/bash
# deep-k check: level-kernel GPU tests, then T40I10D100M plain and with per-phase timing
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/t40_tests.log 2>&1
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/T40.json 2> gpurun_out/T40.err
FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/lv_T40.json 2> gpurun_out/lv_T40.err
