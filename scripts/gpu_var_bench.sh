#!/bin/bash
# Alternating bench lines of libfa_hip variants (FA_HIP_LIB=scripts/microbench/var/libfa_hip_NAME.so;
# "base" = the tree's build): bash scripts/gpu_var_bench.sh NAME "CFG1 CFG2" base v1 v2 ...
# (a CFG is a bench.py config, or shard12 for the 12.5M-row T10I4 shard)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/vb_$1
CFGS=$2
shift 2
mkdir -p "$O"
cd "$R"
for i in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L="$R/scripts/microbench/var/libfa_hip_$v.so"; fi
    for c in $CFGS; do
      case $c in
        shard12) A="--n-txn 12500000 --steps 30 --warmup 3" ;;
        T10I4D100M) A="--steps 10 --warmup 2" ;;
        *) A="--config $c --steps 2 --warmup 1" ;;
      esac
      FA_HIP_LIB="$L" timeout -k 10 500 python bench.py $A --e2e off > "$O/${c}_${v}_$i.json" 2> "$O/${c}_${v}_$i.err"
    done
  done
done
