#!/bin/bash
# deep-k A/B: GPU tests, then T40I10D100M default / fused compress for long rows / packed 16-bit accumulators
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/ab_tests.log 2>&1
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/ab_T40.json 2> gpurun_out/ab_T40.err
FA_FUSED_COMPRESS_MEAN_LEN=64 FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/ab_T40_fused.json 2> gpurun_out/ab_T40_fused.err
FA_ACC16=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/ab_T40_acc16.json 2> gpurun_out/ab_T40_acc16.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/ab_T10.json 2> gpurun_out/ab_T10.err
