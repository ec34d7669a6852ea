#!/bin/bash
# Deep-k iteration: level-kernel GPU tests, then T40I10D100M per-phase and plain timing
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-t40}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --e2e off > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
FA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/t40p_$TAG.json 2> gpurun_out/t40p_$TAG.err
timeout -k 10 300 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/t40_$TAG.json 2> gpurun_out/t40_$TAG.err
