#!/bin/bash
# Every BASELINE config on one GPU (phase timing on), plus the CLI end-to-end job.
set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/cfg_T10I4D100M.json 2> gpurun_out/cfg_T10I4D100M.err
timeout -k 10 300 python bench.py --config webdocs --steps 5 --warmup 1 > gpurun_out/cfg_webdocs.json 2> gpurun_out/cfg_webdocs.err
timeout -k 10 300 python bench.py --config T10I4D100K --steps 10 --warmup 2 > gpurun_out/cfg_T10I4D100K.json 2> gpurun_out/cfg_T10I4D100K.err
timeout -k 10 300 python bench.py --config T10I4D1K --steps 10 --warmup 2 > gpurun_out/cfg_T10I4D1K.json 2> gpurun_out/cfg_T10I4D1K.err
timeout -k 10 500 python bench.py --config T40I10D100M --steps 2 --warmup 1 > gpurun_out/cfg_T40I10D100M.json 2> gpurun_out/cfg_T40I10D100M.err
unset FA_PHASE_TIMING
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/cfg_T10I4D100M_nosync.json 2>&1
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/cfg_T10_12M_nosync.json 2>&1
timeout -k 10 300 python bench.py --strategy candidate --n-txn 12500000 --steps 5 --warmup 1 > gpurun_out/cfg_T10_12M_cand.json 2>&1
timeout -k 10 500 python benchmarks/run_bench.py --config T10I4D10M --mode e2e > gpurun_out/cfg_e2e_T10I4D10M.json 2> gpurun_out/cfg_e2e.err
