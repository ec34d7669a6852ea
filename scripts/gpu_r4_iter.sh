#!/bin/bash
# round 4 iteration pass: Gram tests, T40 A/B of the Gram register tile (KM = 2 vs 4)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/it
mkdir -p $O
export TMPDIR=/tmp
FA_GRAM_KM=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gram" -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_gram.log 2>&1
for v in 2 4 2 4; do
  FA_GRAM_KM=$v timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > $O/T40_km$v.json 2> $O/T40_km$v.err
  tail -1 $O/T40_km$v.json >> $O/T40_km$v.all
done
