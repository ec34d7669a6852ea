#!/bin/bash
# A/B of two kernel-library builds without the test pass: the tree's libfa_hip.so ("new")
# against ablib/libfa_hip_base.so ("base", FA_HIP_LIB), alternating runs of the headline
# and the 12.5M-row shard.  usage: bash scripts/gpu_ab_lib_quick.sh [rounds]
set -e -o pipefail
mkdir -p gpurun_out/abq
N=${1:-3}
for i in $(seq 1 $N); do
  for v in new base; do
    L=""; [ $v = base ] && L=ablib/libfa_hip_base.so
    FA_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/abq/T10_${v}_$i.json 2>/dev/null
    FA_HIP_LIB=$L timeout -k 10 300 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off > gpurun_out/abq/s12_${v}_$i.json 2>/dev/null
  done
done
