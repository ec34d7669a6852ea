#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/it3_12M.json 2>/dev/null
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it3_T10.json 2>/dev/null
timeout -k 10 300 python benchmarks/host_profile.py --n-txn 12500000 > gpurun_out/host_profile2.txt 2>&1
FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it3_T40_100M.json 2>/dev/null
