#!/bin/bash
# Headline (T10I4D100M) hot-kernel evidence: phase-timed bench with the level plans,
# kernel-trace stats, and PMC passes (LDS instructions, bank conflicts, VALU, waits)
# of the pair kernel and the level kernels.  One rocprofv3 pass per counter set.
set -e -o pipefail
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-head}
FA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --e2e off > gpurun_out/phase_$TAG.json 2> gpurun_out/phase_$TAG.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --e2e off > "$R/gpurun_out/kt_$TAG.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS \
  --kernel-include-regex "k_pair_queue16|k_count_slab|k_count_trie" --output-format csv -d "$R/gpurun_out/pmc/${TAG}_a" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --e2e off > "$R/gpurun_out/pmc/${TAG}_a.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_pair_queue16|k_count_slab|k_count_trie" --output-format csv -d "$R/gpurun_out/pmc/${TAG}_b" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --e2e off > "$R/gpurun_out/pmc/${TAG}_b.log" 2>&1
