#!/bin/bash
# targeted GPU tests, kernel tables of the headline under VAR=A / VAR=B, and a bench A/B
# usage: bash scripts/gpu_ab2.sh VAR A B "pytest -k expr" [rounds]
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=$1; A=$2; B=$3; K=$4; N=${5:-2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab2_tests.log 2>&1
for i in $(seq 1 $N); do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/ab2_T10_${val}_$i.json 2>/dev/null
    env $V=$val timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > gpurun_out/ab2_s12_${val}_$i.json 2>/dev/null
  done
done
cd /tmp
for val in $A $B; do
  export $V=$val
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt2_$val" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt2_$val.log" 2>&1
done
