#!/bin/bash
set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/it21_base.json 2>/dev/null
FA_BUNDLE=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/it21_nob.json 2>/dev/null
FA_BUNDLE=0 FA_LEVEL_KERNEL=trie timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/it21_nob_trie.json 2>/dev/null
