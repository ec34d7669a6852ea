#!/bin/bash
# Per-level plans and phase timings (FA_PHASE_TIMING=1 syncs at phase edges) of the
# headline and the deep-k config, plus the plain 12.5M-row shard bench.
set -e -o pipefail
mkdir -p gpurun_out
FA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --e2e off > gpurun_out/lv_T10.json 2> gpurun_out/lv_T10.err
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 20 --warmup 3 --e2e off > gpurun_out/shard12.json 2> gpurun_out/shard12.err
FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/lv_T40.json 2> gpurun_out/lv_T40.err
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/T40.json 2> gpurun_out/T40.err
