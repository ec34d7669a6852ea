#!/bin/bash
# A/B of an env toggle on one MI355X: targeted GPU tests first (pytest -k EXPR), then
# alternating runs of the headline and the 12.5M-row shard with VAR=A and VAR=B.
# usage: bash scripts/gpu_ab_env.sh VAR A B [rounds] [pytest -k expression]
set -e -o pipefail
mkdir -p gpurun_out
V=$1; A=$2; B=$3; N=${4:-2}; K=${5:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/abe_tests.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abe_tests.log 2>&1
fi
for i in $(seq 1 $N); do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/abe_T10_${val}_$i.json 2>/dev/null
    env $V=$val timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > gpurun_out/abe_s12_${val}_$i.json 2>/dev/null
  done
done
