#!/bin/bash
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 20 --warmup 3 > gpurun_out/it31_12M.json 2>/dev/null
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/it31_T10.json 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/gpurun_out/mk12g" -o run -- \
  python3 "$R/bench.py" --n-txn 12500000 --steps 2 --warmup 1 > "$R/gpurun_out/mk12g.log" 2>&1
