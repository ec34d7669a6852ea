#!/bin/bash
# 12.5M-row shard idle-time trace (scripts/gpu_trace_markers.sh) + T40I10D100M kernel stats
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash scripts/gpu_trace_markers.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_T40" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_T40.log" 2>&1
