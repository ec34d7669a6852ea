#!/bin/bash
set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
for d in 0 1 2 3; do
FA_PAIR_DEBUG=$d timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/pp_$d.json 2>/dev/null || true
done
