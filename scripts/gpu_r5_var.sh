#!/bin/bash
# kernel-stat runs of libfa_hip variants (scripts/microbench/build_variants.py) on the
# 12.5M-row shard: bash scripts/gpu_r5_var.sh NAME base v1 v2 ...
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_$1
shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L="$R/scripts/microbench/var/libfa_hip_$v.so"; fi
  FA_HIP_LIB="$L" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$v" -o run -- \
    python3 "$R/bench.py" --n-txn 12500000 --steps 5 --warmup 1 --e2e off > "$O/kt_$v.log" 2>&1
done
