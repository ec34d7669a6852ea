#!/bin/bash
# kernel + roctx marker trace of the 12.5M-row shard (per-rank work at 8 GPUs)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/gpurun_out/mk12" -o run -- \
  python3 "$R/bench.py" --n-txn 12500000 --steps 2 --warmup 1 > "$R/gpurun_out/mk12.log" 2>&1
find "$R/gpurun_out/mk12" -name "*.csv" | head -20 > "$R/gpurun_out/mk12_files.txt"
