#!/bin/bash
# rocprofv3 kernel stats of the headline and the deep-k config (1 timed step each)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_T10" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 > "$R/gpurun_out/kt_T10.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_T40" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 > "$R/gpurun_out/kt_T40.log" 2>&1
