#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out
for L in 48 24; do
FA_COMPRESS_WAVE_MEAN_LEN=$L FA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/t40_cmp_$L.json 2> gpurun_out/t40_cmp_$L.err
done
