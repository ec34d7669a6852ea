#!/bin/bash
# compression count kernel: GPU kernel tests, T40I10D100M phase timing, kernel stats
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/td_tests.log 2>&1
FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > gpurun_out/td_lv_T40.json 2> gpurun_out/td_lv_T40.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_T40d" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_T40d.log" 2>&1
