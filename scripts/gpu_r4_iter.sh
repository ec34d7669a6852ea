#!/bin/bash
# round 4 iteration pass: compression tests, T40 A/B of the bitmap compression tier
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/it
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_device_levels.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_parse.log 2>&1
for v in 1 0 1 0; do
  FA_COMPRESS_BITMAP=$v timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > $O/T40_bm$v.json 2> $O/T40_bm$v.err
  tail -1 $O/T40_bm$v.json >> $O/T40_bm$v.all
done
