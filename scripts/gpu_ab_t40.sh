#!/bin/bash
# A/B of an env toggle on T40I10D100M (the deep-level config) on one MI355X: targeted
# GPU tests first (pytest -k EXPR), then alternating bench runs with VAR=A and VAR=B,
# and one headline T10I4D100M run per value.
# usage: bash scripts/gpu_ab_t40.sh VAR A B [rounds] [pytest -k expression]
set -e -o pipefail
mkdir -p gpurun_out/ab40
V=$1; A=$2; B=$3; N=${4:-2}; K=${5:-slab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab40/tests.log 2>&1
for i in $(seq 1 $N); do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > gpurun_out/ab40/T40_${val}_$i.json 2>/dev/null
  done
done
for val in $A $B; do
  env $V=$val timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/ab40/T10_${val}.json 2>/dev/null
done
