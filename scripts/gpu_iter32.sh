#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_end_to_end.py -x -v --timeout 250 --timeout-method thread > gpurun_out/e2e_tests.log 2>&1
