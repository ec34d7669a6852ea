#!/bin/bash
# round 5 PMC pass of one kernel regex on one config (two SQ counter sets)
#   bash scripts/gpu_r5_pmc.sh NAME REGEX CONFIG
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_pmc_$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS \
  --kernel-include-regex "$2" --output-format csv -d "$O/a" -o run -- \
  python3 "$R/bench.py" --config "$3" --steps 1 --warmup 0 --e2e off > "$O/a.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --kernel-include-regex "$2" --output-format csv -d "$O/b" -o run -- \
  python3 "$R/bench.py" --config "$3" --steps 1 --warmup 0 --e2e off > "$O/b.log" 2>&1
