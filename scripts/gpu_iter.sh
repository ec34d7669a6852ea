#!/bin/bash
# Scratch pass of the current change: GPU tests of the touched paths (-k EXPR), then the
# 12.5M-row shard and headline bench lines.  Output under gpurun_out/iter/.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/iter
mkdir -p "$O"
cd "$R"
K=${1:-"f1_rank or end_to_end"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > "$O/tests.log" 2>&1
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off > "$O/shard.json" 2> "$O/shard.err"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --e2e off > "$O/head.json" 2> "$O/head.err"
