#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "compress or parse or weighted or trim" --timeout 120 --timeout-method thread > gpurun_out/cmp_tests.log 2>&1
export FA_PHASE_TIMING=1
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/it33_T10.json 2>/dev/null
timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it33_T40.json 2>/dev/null
