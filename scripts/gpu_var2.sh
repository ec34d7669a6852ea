#!/bin/bash
# where the run-to-run spread lives: 3 processes under rocprofv3 kernel stats (bench line + per-kernel totals)
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kv_$i" -o run -- \
    python3 "$R/bench.py" --steps 10 --warmup 2 --e2e off > "$R/gpurun_out/kv_$i.json" 2> "$R/gpurun_out/kv_$i.err"
done
