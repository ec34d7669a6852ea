#!/bin/bash
# k = 2 kernel check: pair-kernel GPU tests, then the pair probe (full / no
# scatter / no flush / neither) for each schedule on the headline config.
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/pair_tests.log 2>&1
timeout -k 10 300 python benchmarks/pair_probe.py --config T10I4D100M --kernels queue16 --modes 0,1,9,4 \
  > gpurun_out/pair_probe.json 2> gpurun_out/pair_probe.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/bench_pair.json 2> gpurun_out/bench_pair.err
