#!/bin/bash
# GPU tests, then T40I10D100M A/B of an env toggle (default FA_DFS_PAIR 1 vs 0), the
# headline once, and a kernel trace of the T40 default
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=${1:-FA_DFS_PAIR}; A=${2:-1}; B=${3:-0}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t4_tests.log 2>&1
for i in 1 2; do
  for val in $A $B; do
    env $V=$val timeout -k 10 400 python bench.py --config T40I10D100M --steps 5 --warmup 1 --e2e off > gpurun_out/t4_T40_${val}_$i.json 2>gpurun_out/t4_T40_${val}_$i.err
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/t4_T10_x_1.json 2>/dev/null
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/t4kt" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/t4kt.log" 2>&1
