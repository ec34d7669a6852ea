#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "trie or bitmaps_pairs" > gpurun_out/iter_tests.log 2>&1
export FA_PHASE_TIMING=1
for r in 2 4 8; do
FA_TRIE_ROUNDS=$r timeout -k 10 200 python bench.py --steps 2 --warmup 1 > gpurun_out/sw_T10_r$r.json 2>/dev/null
done
FA_TRIE_ROUNDS=4 timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/sw_T40_r4.json 2>/dev/null
FA_TRIE_ROUNDS=2 timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/sw_T40_r2.json 2>/dev/null
FA_TRIE_ROUNDS=8 timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/sw_T40_r8.json 2>/dev/null
