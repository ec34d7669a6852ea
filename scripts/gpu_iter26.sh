#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
for i in 1 2; do
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 20 --warmup 3 > gpurun_out/it26_12M_$i.json 2>/dev/null
FA_GEN_CHAIN=0 timeout -k 10 200 python bench.py --n-txn 12500000 --steps 20 --warmup 3 > gpurun_out/it26_12M_nochain_$i.json 2>/dev/null
done
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it26_T10.json 2>/dev/null
