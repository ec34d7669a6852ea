#!/bin/bash
# round 5 A/B pass: GPU tests of the touched paths, then alternating bench runs of a
# tuning knob (FA_TUNE=KNOB=VALUE) on the 12.5M-row shard and the headline config, and
# one rocprofv3 kernel trace per value on the headline
#   bash scripts/gpu_r5_ab.sh NAME "pytest -k EXPR" KNOB V1 V2 [V3]
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
    FA_TUNE="$K=$v" timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > $O/s12_${v}_$i.json 2> $O/s12_${v}_$i.err
    FA_TUNE="$K=$v" timeout -k 10 400 python bench.py --steps 10 --warmup 2 --e2e off > $O/T10_${v}_$i.json 2> $O/T10_${v}_$i.err
  done
done
cd /tmp
for v in "$@"; do
  FA_TUNE="$K=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$v" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$O/kt_$v.log" 2>&1
done
