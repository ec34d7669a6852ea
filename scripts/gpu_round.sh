#!/bin/bash
# the driver's round-end sequence on one GPU: every GPU test, smoke(), the default bench line
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/rd_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rd_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/rd_bench.json 2> gpurun_out/rd_bench.err
