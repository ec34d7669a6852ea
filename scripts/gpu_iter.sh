#!/bin/bash
# Iteration check: GPU kernel + scale tests, the headline bench with phase timing,
# and the slab-kernel build/count split.  Every GPU step has its own time limit.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-it}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py tests/test_gpu_end_to_end.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --e2e off > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
FA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --e2e off > gpurun_out/phase_$TAG.json 2> gpurun_out/phase_$TAG.err
timeout -k 10 300 python benchmarks/slab_probe.py --config T10I4D100M > gpurun_out/slab_probe_$TAG.txt 2>&1
