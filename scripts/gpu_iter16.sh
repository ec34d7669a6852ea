#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parse_tests.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
timeout -k 10 400 python benchmarks/run_bench.py --config T10I4D10M --mode e2e --device cuda --steps 2 --warmup 1 > gpurun_out/e2e_T10I4D10M.json 2> gpurun_out/e2e_T10I4D10M.err
timeout -k 10 600 python benchmarks/run_bench.py --config T10I4D100M --mode e2e --device cuda --steps 2 --warmup 1 > gpurun_out/e2e_T10I4D100M.json 2> gpurun_out/e2e_T10I4D100M.err
