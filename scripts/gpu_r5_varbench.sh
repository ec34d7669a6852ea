#!/bin/bash
# bench.py (no profiler) of libfa_hip variants, alternating: shard and headline
#   bash scripts/gpu_r5_varbench.sh NAME base v1 ...
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_$1
shift
mkdir -p $O
cd $R
for i in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L="$R/scripts/microbench/var/libfa_hip_$v.so"; fi
    FA_HIP_LIB="$L" timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > $O/s12_${v}_$i.json 2> $O/s12_${v}_$i.err
    FA_HIP_LIB="$L" timeout -k 10 400 python bench.py --steps 10 --warmup 2 --e2e off > $O/T10_${v}_$i.json 2> $O/T10_${v}_$i.err
  done
done
