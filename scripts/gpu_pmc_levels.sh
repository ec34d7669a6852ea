#!/bin/bash
# PMC counters of the level kernels (old slab vs trie) on T10I4D10M; one pass per counter set.
set -e
mkdir -p gpurun_out/pmc
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "trie or bitmaps_pairs" > gpurun_out/iter_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for K in slab trie; do
  export FA_LEVEL_KERNEL=$K
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex "k_count" --output-format csv -d $R/gpurun_out/pmc/$K -o run -- python3 $R/bench.py --config T10I4D10M --steps 1 --warmup 0 > $R/gpurun_out/pmc/$K.log 2>&1
done
unset FA_LEVEL_KERNEL
cd $R
export FA_PHASE_TIMING=1
timeout -k 10 200 python bench.py --steps 2 --warmup 1 > gpurun_out/sw2_T10.json 2>/dev/null
timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/sw2_T40.json 2>/dev/null
FA_LEVEL_KERNEL=slab timeout -k 10 200 python bench.py --config T40I10D10M --steps 2 --warmup 1 > gpurun_out/sw2_T40_slab.json 2>/dev/null
FA_LEVEL_KERNEL=slab timeout -k 10 200 python bench.py --steps 2 --warmup 1 > gpurun_out/sw2_T10_slab.json 2>/dev/null
