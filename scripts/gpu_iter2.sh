#!/bin/bash
# Iteration check: every GPU test, then the headline and the 12.5M-row shard twice each, and a
# kernel + marker trace of the shard for benchmarks/gap_attrib.py.
set -e -o pipefail
mkdir -p gpurun_out/it
O=gpurun_out/it
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > $O/T10_$i.json 2> $O/T10_$i.err
  timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > $O/s12_$i.json 2> $O/s12_$i.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/$O/mk12" -o run -- \
  python3 "$R/bench.py" --n-txn 12500000 --steps 2 --warmup 1 --e2e off > "$R/$O/mk12.log" 2>&1
