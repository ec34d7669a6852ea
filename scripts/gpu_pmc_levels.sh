#!/bin/bash
# PMC counters of the level kernels (k_count_*) on T40I10D10M and T10I4D10M:
# one rocprofv3 pass per counter set (no trace domains with --pmc).
set -e -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for C in T40I10D10M T10I4D10M; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex "k_count" --output-format csv -d $R/gpurun_out/pmc/${C}_a -o run -- python3 $R/bench.py --config $C --steps 1 --warmup 0 --e2e off > $R/gpurun_out/pmc/${C}_a.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "k_count" --output-format csv -d $R/gpurun_out/pmc/${C}_b -o run -- python3 $R/bench.py --config $C --steps 1 --warmup 0 --e2e off > $R/gpurun_out/pmc/${C}_b.log 2>&1
done
