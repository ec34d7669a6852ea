#!/bin/bash
# round 5 scratch pass: GPU tests of the touched paths, the 12.5M-row shard (one rank of 8)
# bench line, the headline line and the shard's kernel trace
#   bash scripts/gpu_r5_iter.sh NAME [pytest -k EXPR]
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_${1:-base}
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$2" > $O/tests.log 2>&1
fi
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off > $O/shard12.json 2> $O/shard12.err
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --e2e off > $O/T10.json 2> $O/T10.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt12" -o run -- \
  python3 "$R/bench.py" --n-txn 12500000 --steps 1 --warmup 1 --e2e off > "$O/kt12.log" 2>&1
