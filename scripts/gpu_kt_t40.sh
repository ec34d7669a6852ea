#!/bin/bash
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_T40_10M -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config T40I10D10M --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_T40_10M.log 2>&1
