#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it20_T10.json 2>/dev/null
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 20 --warmup 3 > gpurun_out/it20_12M.json 2>/dev/null
timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it20_T40.json 2>/dev/null
