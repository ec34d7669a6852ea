#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
timeout -k 10 300 python benchmarks/rules_probe.py --config T10I4D10M > gpurun_out/rules_T10.json 2>gpurun_out/rules_T10.err
timeout -k 10 500 python benchmarks/rules_probe.py --config T40I10D10M --reps 2 > gpurun_out/rules_T40.json 2>gpurun_out/rules_T40.err
