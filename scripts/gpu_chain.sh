#!/bin/bash
# device-sized apriori-gen chain: GPU tests, headline and 12.5M-row shard benches (per-level chain A/B)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ch_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/ch_T10.json 2> gpurun_out/ch_T10.err
FA_GEN_DEVCHAIN=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/ch_T10_old.json 2> gpurun_out/ch_T10_old.err
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 20 --warmup 3 --e2e off > gpurun_out/ch_s12.json 2> gpurun_out/ch_s12.err
FA_GEN_DEVCHAIN=0 timeout -k 10 300 python bench.py --n-txn 12500000 --steps 20 --warmup 3 --e2e off > gpurun_out/ch_s12_old.json 2> gpurun_out/ch_s12_old.err
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 20 --warmup 3 --e2e off > gpurun_out/ch_s12b.json 2> gpurun_out/ch_s12b.err
