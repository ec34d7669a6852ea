#!/bin/bash
# Round-6 lane-deal pass: GPU tests of the touched paths, the T40 window log, lane-deal
# kernel stats on the 12.5M-row shard (deal forced on), shard A/B of the deal threshold,
# headline bench line.  Output under gpurun_out/ld/.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ld
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "lane_deal or window or t40_deep or la_qsum" > "$O/tests.log" 2>&1
timeout -k 10 400 python benchmarks/window_probe.py > "$O/window_log.txt" 2>&1
(cd /tmp && FA_TUNE=lane_deal_min_rows=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$O/kt" -o run -- python3 "$R/bench.py" --n-txn 12500000 --steps 3 --warmup 1 --e2e off > "$O/kt.log" 2>&1)
for i in 1 2; do
  for v in 33554432 0; do
    FA_TUNE=lane_deal_min_rows=$v timeout -k 10 200 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off \
      > "$O/shard_$v.$i.json" 2> /dev/null
  done
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --e2e off > "$O/head.json" 2> "$O/head.err"
