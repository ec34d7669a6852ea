#!/bin/bash
# Iteration pass: targeted GPU tests, then the headline and deep-k benches.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "${FA_TEST_K:-trie or bitmaps_pairs}" > gpurun_out/iter_tests.log 2>&1
export FA_PHASE_TIMING=1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/iter_T10.json 2> gpurun_out/iter_T10.err
timeout -k 10 300 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/iter_T40.json 2> gpurun_out/iter_T40.err
