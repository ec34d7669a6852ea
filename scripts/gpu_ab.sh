#!/bin/bash
# A/B pass over FA_TUNE specs: GPU tests of the touched paths, then alternating bench
# runs of every spec on the 12.5M-row shard and the headline config, and one rocprofv3
# kernel trace per spec on the headline.  A spec is a full FA_TUNE value
# ("knob=v,knob=v"); "base" runs the defaults.
#   bash scripts/gpu_ab.sh NAME "pytest -k EXPR" SPEC1 SPEC2 ...
#   CFG=T40I10D100M bash scripts/gpu_ab.sh ...   (headline replaced by another config, no shard)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_$1
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" \
    > "$O/tests.log" 2>&1
fi
shift 2
CFG=${CFG:-T10I4D100M}
spec() { [ "$1" = base ] && echo "" || echo "$1"; }
tag() { echo "$1" | tr ',=' '_-'; }
for i in 1 2; do
  for s in "$@"; do
    t=$(tag "$s")
    if [ "$CFG" = T10I4D100M ]; then
      FA_TUNE=$(spec "$s") timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off \
        > "$O/s12_${t}_$i.json" 2> "$O/s12_${t}_$i.err"
      FA_TUNE=$(spec "$s") timeout -k 10 400 python bench.py --steps 10 --warmup 2 --e2e off \
        > "$O/T10_${t}_$i.json" 2> "$O/T10_${t}_$i.err"
    else
      FA_TUNE=$(spec "$s") timeout -k 10 500 python bench.py --config "$CFG" --steps 2 --warmup 1 --e2e off \
        > "$O/${CFG}_${t}_$i.json" 2> "$O/${CFG}_${t}_$i.err"
    fi
  done
done
[ -n "$NOKT" ] && exit 0          # NOKT=1: bench lines only, no kernel traces
cd /tmp
for s in "$@"; do
  t=$(tag "$s")
  FA_TUNE=$(spec "$s") timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$t" -o run -- \
    python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 1 --e2e off > "$O/kt_$t.log" 2>&1
done
