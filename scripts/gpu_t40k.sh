#!/bin/bash
# deep-k level-kernel choice: T40I10D100M with per-phase timing, slab kernel forced vs the trie threshold
set -e -o pipefail
mkdir -p gpurun_out
FA_LEVEL_KERNEL=slab FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/lv_T40_slab.json 2> gpurun_out/lv_T40_slab.err
FA_LEVEL_KERNEL=slab timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/T40_slab.json 2> gpurun_out/T40_slab.err
