#!/bin/bash
# Same-box A/B of one tuning knob: shard (12.5M rows) and headline bench lines,
# alternating FA_TUNE=KNOB=A / KNOB=B, REPS rounds.  Output under gpurun_out/ab2/.
#   bash scripts/gpu_ab2.sh KNOB A B [REPS] [EXTRA_FA_TUNE]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab2
mkdir -p "$O"
cd "$R"
V=$1; A=$2; B=$3; N=${4:-3}; X=${5:-}
for i in $(seq 1 "$N"); do
  for val in "$A" "$B"; do
    env "FA_TUNE=$V=$val${X:+,$X}" timeout -k 10 200 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off \
      --no-digest-check > "$O/shard_${val}_$i.json" 2> "$O/shard_${val}_$i.err"
  done
done
for i in $(seq 1 "$N"); do
  for val in "$A" "$B"; do
    env "FA_TUNE=$V=$val${X:+,$X}" timeout -k 10 300 python bench.py --steps 15 --warmup 3 --e2e off \
      > "$O/head_${val}_$i.json" 2> "$O/head_${val}_$i.err"
  done
done
