#!/bin/bash
# flattened pairs per tile kind: pair probe under FA_PAIR_FLAT = 1 (all), 2 (off-diagonal), 3 (diagonal), 0 (none)
set -e -o pipefail
mkdir -p gpurun_out
for v in 1 2 3 0; do
  FA_PAIR_FLAT=$v timeout -k 10 300 python benchmarks/pair_probe.py --config T10I4D100M --modes 0 --reps 5 > gpurun_out/f2_probe_$v.txt 2>/dev/null
done
