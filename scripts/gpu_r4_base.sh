#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r4b/T10.json 2> gpurun_out/r4b/T10.err
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/r4b/T40.json 2> gpurun_out/r4b/T40.err
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1
