#!/bin/bash
# kernel stats of the headline with and without the compress-written pair layout
set -e -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ktlr
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  FA_PAIR_LR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ktlr/lr$v" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --e2e off > "$R/gpurun_out/ktlr/lr$v.log" 2>&1
done
