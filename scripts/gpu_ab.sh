#!/bin/bash
# A/B of an env toggle on the headline and the 12.5M shard: alternating runs, 20 timed steps each
# usage: bash scripts/gpu_ab.sh VAR VALUE_A VALUE_B
set -e -o pipefail
mkdir -p gpurun_out
V=$1; A=$2; B=$3
for i in 1 2 3; do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/ab_${val}_T10_$i.json 2>/dev/null
    env $V=$val timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > gpurun_out/ab_${val}_s12_$i.json 2>/dev/null
  done
done
