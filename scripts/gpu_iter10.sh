#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it10_T10.json 2>/dev/null
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/it10_12M.json 2>/dev/null
timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it10_T40.json 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof10_12M -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --n-txn 12500000 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof10_12M.log 2>&1
