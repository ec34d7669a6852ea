#!/bin/bash
# PMC of the slab kernels under an env toggle (VAR=A vs VAR=B) on one config: two
# counter passes per value, every dispatch kept (benchmarks/pmc_dispatch.py aligns them).
# usage: bash scripts/gpu_pmc_ab.sh VAR A B [bench args...]
set -e -o pipefail
V=$1; A=$2; B=$3; shift 3
O=gpurun_out/pmcab; mkdir -p $O
for val in $A $B; do
  export $V=$val
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS \
    --kernel-include-regex "k_count_slab_rec" --output-format csv -d "$O/${val}_a" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --e2e off "$@" > "$O/${val}_a.log" 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_count_slab_rec" --output-format csv -d "$O/${val}_b" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --e2e off "$@" > "$O/${val}_b.log" 2>&1
done
