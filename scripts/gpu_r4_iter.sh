#!/bin/bash
# round 4 iteration pass: device-level tests, T40 bench runs
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/it
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_device_levels.py tests/test_gpu_scale.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_dl.log 2>&1
for i in 1 2; do
  timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > $O/T40_trim$i.json 2> $O/T40_trim$i.err
done
