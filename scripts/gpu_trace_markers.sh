#!/bin/bash
# 12.5M-row shard (the per-rank work at 8 GPUs): timed bench, then a kernel +
# roctx marker trace for benchmarks/gap_attrib.py (GPU idle time by host range)
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python "$R/bench.py" --n-txn 12500000 --steps 20 --warmup 3 --e2e off > "$R/gpurun_out/shard12.json" 2> "$R/gpurun_out/shard12.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/gpurun_out/mk12" -o run -- \
  python3 "$R/bench.py" --n-txn 12500000 --steps 2 --warmup 1 --e2e off > "$R/gpurun_out/mk12.log" 2>&1
