#!/bin/bash
# T40I10D100M: trie threshold sweep (per-level timings)
set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
timeout -k 10 300 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it25_T40.json 2>/dev/null
FA_TRIE_MIN_SAVING=0.6 timeout -k 10 300 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it25_T40_s60.json 2>/dev/null
FA_TRIE_MIN_SAVING=0.75 timeout -k 10 300 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it25_T40_s75.json 2>/dev/null
