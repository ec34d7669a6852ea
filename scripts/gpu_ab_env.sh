#!/bin/bash
# Every GPU test, then an A/B of an env toggle: alternating runs of the headline and the
# 12.5M-row shard.  usage: bash scripts/gpu_ab_env.sh VAR VALUE_A VALUE_B [rounds]
set -e -o pipefail
mkdir -p gpurun_out/abe
V=$1; A=$2; B=$3; N=${4:-3}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/abe/tests.log 2>&1
for i in $(seq 1 $N); do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/abe/T10_${val}_$i.json 2>/dev/null
    env $V=$val timeout -k 10 300 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off > gpurun_out/abe/s12_${val}_$i.json 2>/dev/null
  done
done
