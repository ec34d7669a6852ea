#!/bin/bash
# A/B of two builds of the kernel library on one MI355X: the tree's libfa_hip.so
# ("new") against ablib/libfa_hip_base.so ("base", FA_HIP_LIB), alternating runs of
# the headline and the 12.5M-row shard, after the GPU tests.
# usage: bash scripts/gpu_ab_lib.sh [rounds] [extra bench args for a third config]
set -e -o pipefail
mkdir -p gpurun_out
N=${1:-2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
for i in $(seq 1 $N); do
  for v in new base; do
    L=""; [ $v = base ] && L=ablib/libfa_hip_base.so
    FA_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/ab_T10_${v}_$i.json 2>/dev/null
    FA_HIP_LIB=$L timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > gpurun_out/ab_s12_${v}_$i.json 2>/dev/null
    if [ -n "$2" ]; then
      FA_HIP_LIB=$L timeout -k 10 400 python bench.py ${@:2} --e2e off > gpurun_out/ab_X_${v}_$i.json 2>/dev/null
    fi
  done
done
