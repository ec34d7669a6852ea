#!/bin/bash
# Lane-deal timing pass: GPU tests of the deal, kernel stats of the 12.5M-row shard with
# the deal forced on, headline bench line.  Output under gpurun_out/ld2/.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ld2
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "lane_deal or device_levels or t40_deep" > "$O/tests.log" 2>&1
(cd /tmp && FA_TUNE=lane_deal_min_rows=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$O/kt" -o run -- python3 "$R/bench.py" --n-txn 12500000 --steps 3 --warmup 1 --e2e off > "$O/kt.log" 2>&1)
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --e2e off > "$O/head_$i.json" 2> /dev/null
done
