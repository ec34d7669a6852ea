#!/bin/bash
# A/B of two kernel-library builds on the headline and on T40I10D100M: the tree's
# libfa_hip.so ("new") against ablib/libfa_hip_base.so ("base", FA_HIP_LIB), after the
# GPU tests matching -k EXPR; then T40 with the new library and FA_SLAB_CLS=0.
# usage: bash scripts/gpu_ab_lib_t40.sh [rounds] [pytest -k expression]
set -e -o pipefail
O=gpurun_out/abl; mkdir -p $O
N=${1:-2}; K=${2:-slab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $O/tests.log 2>&1
for i in $(seq 1 $N); do
  for v in new base; do
    L=""; [ $v = base ] && L=ablib/libfa_hip_base.so
    FA_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > $O/T10_${v}_$i.json 2>/dev/null
    FA_HIP_LIB=$L timeout -k 10 300 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > $O/T40_${v}_$i.json 2>/dev/null
  done
  FA_SLAB_CLS=0 timeout -k 10 300 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > $O/T40_nocls_$i.json 2>/dev/null
done
