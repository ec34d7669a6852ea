#!/bin/bash
# headline kernel + roctx marker trace for benchmarks/gap_attrib.py (GPU idle time by host range)
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/gpurun_out/mkh" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --e2e off > "$R/gpurun_out/mkh.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/gpurun_out/mk12" -o run -- \
  python3 "$R/bench.py" --n-txn 12500000 --steps 2 --warmup 1 --e2e off > "$R/gpurun_out/mk12.log" 2>&1
