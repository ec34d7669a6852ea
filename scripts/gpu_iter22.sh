#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "dfs or bundl or chain" --timeout 120 --timeout-method thread > gpurun_out/dfs_tests.log 2>&1
export FA_PHASE_TIMING=1
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/it22_dfs.json 2>/dev/null
FA_BUNDLE_DFS=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/it22_nodfs.json 2>/dev/null
unset FA_PHASE_TIMING
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it22_dfs_ns.json 2>/dev/null
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 20 --warmup 3 > gpurun_out/it22_12M.json 2>/dev/null
