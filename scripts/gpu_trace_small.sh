#!/bin/bash
# Kernel trace of the headline at a 1/8 shard (what one rank of 8 runs): kernel busy vs gaps.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/kt_small" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --n-txn 12500000 --steps 2 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/kt_small.log" 2>&1
