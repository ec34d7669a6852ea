#!/bin/bash
# pair kernel check: GPU kernel tests, the pair probe (full / no scatter), headline bench twice
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pr_tests.log 2>&1
timeout -k 10 300 python benchmarks/pair_probe.py --config T10I4D100M --modes 0,1 --reps 5 > gpurun_out/pr_probe.txt 2>/dev/null
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/pr_T10a.json 2>/dev/null
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/pr_T10b.json 2>/dev/null
