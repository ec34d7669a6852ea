#!/bin/bash
# Gram pair kernel A/B: GPU tests, T40I10D100M with 256-tile (default) and 128-tile kernels, headline twice
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/gr_tests.log 2>&1
FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/gr_T40.json 2> gpurun_out/gr_T40.err
FA_GRAM_TILE=128 FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/gr_T40_128.json 2> gpurun_out/gr_T40_128.err
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/gr_T40p.json 2> gpurun_out/gr_T40p.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/gr_T10a.json 2> gpurun_out/gr_T10a.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/gr_T10b.json 2> gpurun_out/gr_T10b.err
