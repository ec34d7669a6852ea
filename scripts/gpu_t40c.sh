#!/bin/bash
# T40I10D100M: scale tests, per-phase timing, plain timing
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tc_tests.log 2>&1
FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/tc_lv_T40.json 2> gpurun_out/tc_lv_T40.err
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/tc_T40.json 2> gpurun_out/tc_T40.err
