#!/bin/bash
# kernel-stat runs of libfa_hip timing variants (FA_HIP_LIB=scripts/microbench/var/libfa_hip_NAME.so;
# "base" = the tree's build) on one config: bash scripts/gpu_var.sh NAME CFG base v1 v2 ...
# (CFG: a bench.py config, or shard12 for the 12.5M-row T10I4 shard)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/var_$1
CFG=$2
shift 2
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
if [ "$CFG" = shard12 ]; then ARGS="--n-txn 12500000 --steps 5 --warmup 1"; else ARGS="--config $CFG --steps 1 --warmup 1"; fi
ARGS="$ARGS --no-digest-check"
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L="$R/scripts/microbench/var/libfa_hip_$v.so"; fi
  FA_HIP_LIB="$L" timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_${CFG}_$v" -o run -- \
    python3 "$R/bench.py" $ARGS --e2e off > "$O/kt_${CFG}_$v.log" 2>&1
done
