#!/bin/bash
# Round check on one MI355X: GPU tests, the driver's bench command (with the e2e
# window), and the C++ CPU baseline of the headline config (vs_baseline).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
if [ "${FA_CPU_BASELINE:-0}" = "1" ]; then
  timeout -k 10 600 python benchmarks/run_bench.py --mode cpu --device cpu --config T10I4D100M --steps 1 \
    --warmup 0 > gpurun_out/cpu_T10I4D100M.json 2> gpurun_out/cpu_T10I4D100M.err
fi
