#!/bin/bash
# compression tiers: GPU kernel tests, T40I10D100M per-phase timing, headline bench
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/cm_tests.log 2>&1
FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/cm_lv_T40.json 2> gpurun_out/cm_lv_T40.err
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/cm_T40.json 2> gpurun_out/cm_T40.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/cm_T10.json 2> gpurun_out/cm_T10.err
