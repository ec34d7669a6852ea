#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "pair or bitmaps_pairs or weighted" --timeout 120 --timeout-method thread > gpurun_out/pair_tests.log 2>&1
export FA_PHASE_TIMING=1
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/it24_T10.json 2>/dev/null
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/it24_12M.json 2>/dev/null
