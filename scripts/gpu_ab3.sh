#!/bin/bash
# A/B/C of an env variable's values: alternating runs of the headline and the 12.5M shard.
# usage: bash scripts/gpu_ab3.sh VAR "V1 V2 V3" [rounds]
set -e -o pipefail
mkdir -p gpurun_out/ab3
V=$1; VALS=$2; N=${3:-3}
for i in $(seq 1 $N); do
  for val in $VALS; do
    env $V=$val timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/ab3/T10_${val}_$i.json 2>/dev/null
    env $V=$val timeout -k 10 300 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off > gpurun_out/ab3/s12_${val}_$i.json 2>/dev/null
  done
done
