#!/bin/bash
# device-sized chain A/B on the deep-k config (phase times) and the headline
set -e -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  FA_GEN_DEVCHAIN=$v FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/dc_T40_$v.json 2> gpurun_out/dc_T40_$v.err
  FA_GEN_DEVCHAIN=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/dc_T10_$v.json 2> gpurun_out/dc_T10_$v.err
done
