#!/bin/bash
# cooperative apriori-gen chain: kernel tests, headline + 12.5M shard benches
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "chain or bundl or gen" > gpurun_out/coop_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/bench_coop.json 2> gpurun_out/bench_coop.err
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 20 --warmup 3 --e2e off > gpurun_out/shard_coop.json 2> gpurun_out/shard_coop.err
