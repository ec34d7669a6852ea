#!/bin/bash
# pair kernel iteration: GPU kernel tests, pair probe (default vs FA_PAIR_FLAT=0), headline twice
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f3_tests.log 2>&1
for v in 2 0; do
  FA_PAIR_FLAT=$v timeout -k 10 300 python benchmarks/pair_probe.py --config T10I4D100M --modes 0,1 --reps 5 > gpurun_out/f3_probe_$v.txt 2>/dev/null
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/f3_T10a.json 2>/dev/null
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/f3_T10b.json 2>/dev/null
