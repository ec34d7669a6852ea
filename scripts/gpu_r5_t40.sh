#!/bin/bash
# round 5 T40I10D100M A/B pass: GPU tests (optional), then alternating bench runs of a tuning knob
#   bash scripts/gpu_r5_t40.sh NAME "pytest -k EXPR" KNOB V1 V2
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_$1
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" > $O/tests.log 2>&1
fi
K=$3; shift 3
for i in 1 2; do
  for v in "$@"; do
    FA_TUNE="$K=$v" timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > $O/T40_${v}_$i.json 2> $O/T40_${v}_$i.err
  done
done
