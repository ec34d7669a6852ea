#!/bin/bash
# build-measure cycle on one MI355X: every GPU test, then an A/B of an env toggle
# (default FA_DEVICE_LEVELS 1 vs 0) on the headline and the 12.5M-row shard, then a
# kernel + marker trace of the headline (benchmarks/gap_attrib.py, kernel tables)
# usage: bash scripts/gpu_cycle.sh [VAR A B]
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=${1:-FA_DEVICE_LEVELS}; A=${2:-1}; B=${3:-0}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cy_tests.log 2>&1
for i in 1 2; do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/cy_T10_${val}_$i.json 2>/dev/null
    env $V=$val timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > gpurun_out/cy_s12_${val}_$i.json 2>/dev/null
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/gpurun_out/cymkh" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --e2e off > "$R/gpurun_out/cymkh.log" 2>&1
