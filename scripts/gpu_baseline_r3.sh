#!/bin/bash
# round-3 start: GPU tests, the default bench line, the 12.5M-row shard
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_tests.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > gpurun_out/r3_s12.json 2> gpurun_out/r3_s12.err
