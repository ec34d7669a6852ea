#!/bin/bash
# PMC counters of the pair kernel and the level kernels on T10I4D10M (one pass)
set -e
mkdir -p gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex "k_pair_rows16|k_count_slab" --output-format csv -d $R/gpurun_out/pmc2/a -o run -- python3 $R/bench.py --config T10I4D10M --steps 1 --warmup 0 > $R/gpurun_out/pmc2/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --kernel-include-regex "k_pair_rows16|k_count_slab" --output-format csv -d $R/gpurun_out/pmc2/b -o run -- python3 $R/bench.py --config T10I4D10M --steps 1 --warmup 0 > $R/gpurun_out/pmc2/b.log 2>&1
