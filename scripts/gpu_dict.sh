#!/bin/bash
# device dictionary parser: parse tests, then the string-token webdocs end-to-end job
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parse.py tests/test_gpu_end_to_end.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/gpu_parse_tests.log 2>&1
timeout -k 10 400 python benchmarks/run_bench.py --config webdocs --mode e2e --tokens str --steps 2 \
  --warmup 1 > gpurun_out/webdocs_str_e2e.json 2> gpurun_out/webdocs_str_e2e.err
