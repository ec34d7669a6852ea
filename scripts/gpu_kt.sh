#!/bin/bash
# rocprofv3 kernel trace + stats of the headline bench (1 timed step)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/kt_${TAG:-T10}" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/kt_${TAG:-T10}.log" 2>&1
