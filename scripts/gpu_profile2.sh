#!/bin/bash
# Profiles for docs/PERF.md: kernel stats of the headline (100M) and a 1/8 shard (12.5M) timeline.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_T10 -o run -- \
  python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof_T10.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_12M -o run -- \
  python3 $R/bench.py --n-txn 12500000 --steps 2 --warmup 1 > $R/gpurun_out/prof_12M.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_T40 -o run -- \
  python3 $R/bench.py --config T40I10D100M --steps 1 --warmup 1 > $R/gpurun_out/prof_T40.log 2>&1
