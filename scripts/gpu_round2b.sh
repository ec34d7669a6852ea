#!/bin/bash
# GPU tests, headline bench, and the string-token webdocs end-to-end job
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/bench.json 2> gpurun_out/bench.err
FA_PARSE_TIMING=1 timeout -k 10 400 python benchmarks/run_bench.py --config webdocs --mode e2e --tokens str --steps 1 \
  --warmup 1 > gpurun_out/webdocs_str_e2e.json 2> gpurun_out/webdocs_str_e2e.err
