#!/bin/bash
# iteration check: kernel tests, headline bench, kernel-time profile of the headline
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/iter_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e off > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_iter" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_iter.log" 2>&1
