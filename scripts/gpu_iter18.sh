#!/bin/bash
set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it18_T10.json 2>/dev/null
FA_SLAB_ONEPASS=1 timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it18_T10_op.json 2>/dev/null
unset FA_PHASE_TIMING
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it18_T10_ns.json 2>/dev/null
FA_SLAB_ONEPASS=1 timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it18_T10_op_ns.json 2>/dev/null
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/it18_12M.json 2>/dev/null
FA_SLAB_ONEPASS=1 timeout -k 10 200 python bench.py --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/it18_12M_op.json 2>/dev/null
