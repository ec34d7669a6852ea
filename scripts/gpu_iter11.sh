#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "gram or bitmaps" > gpurun_out/iter_tests.log 2>&1
export FA_PHASE_TIMING=1
timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it11_T40.json 2>/dev/null
FA_GRAM_KERNEL=popc timeout -k 10 400 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/it11_T40_10M_popc.json 2>/dev/null
timeout -k 10 400 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/it11_T40_10M.json 2>/dev/null
