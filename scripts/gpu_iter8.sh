#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "slab or bundled or bitmaps or trie" > gpurun_out/iter_tests.log 2>&1
export FA_PHASE_TIMING=1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it8_T10.json 2>/dev/null
unset FA_PHASE_TIMING
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it8_T10_nosync.json 2>/dev/null
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/it8_12M.json 2>/dev/null
timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it8_T40.json 2>/dev/null
