#!/bin/bash
# Alternating bench runs of several FA_TUNE settings on one box: REPS rounds over the
# settings.   bash scripts/gpu_ab_multi.sh CONFIG REPS "spec1" "spec2" ...
# Output: gpurun_out/abm/<i>_<n>.json (setting i, round n).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abm
mkdir -p "$O"
cd "$R"
CFG=$1; N=$2; shift 2
for n in $(seq 1 "$N"); do
  i=0
  for spec in "$@"; do
    env "FA_TUNE=$spec" timeout -k 10 300 python bench.py --config "$CFG" --steps 8 --warmup 1 --e2e off \
      > "$O/${i}_$n.json" 2> /dev/null
    i=$((i + 1))
  done
done
