#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "trie or bitmaps_pairs or slab" > gpurun_out/iter_tests.log 2>&1
export FA_PHASE_TIMING=1
timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/it2_T40.json 2>/dev/null
FA_LEVEL_KERNEL=trie timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/it2_T40_trie.json 2>/dev/null
FA_LEVEL_KERNEL=trie FA_SLAB_SW=32 timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/it2_T40_trie32.json 2>/dev/null
FA_LEVEL_KERNEL=trie FA_SLAB_SW=16 timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/it2_T40_trie16.json 2>/dev/null
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/it2_T10.json 2>/dev/null
timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 > gpurun_out/it2_T40_100M.json 2>/dev/null
