#!/bin/bash
# Quick GPU verification: kernel tests, smoke, headline bench, deep-k bench.
set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_T10I4D100M.json 2> gpurun_out/bench_T10I4D100M.err
timeout -k 10 500 python bench.py --config T40I10D100M --steps 2 --warmup 1 > gpurun_out/bench_T40I10D100M.json 2> gpurun_out/bench_T40I10D100M.err
