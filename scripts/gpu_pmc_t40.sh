#!/bin/bash
# Deep-k evidence: PMC of the level kernels on T40I10D10M (one pass per counter
# set), then the slab-kernel build/count split of the headline levels.
set -e -o pipefail
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-t40}
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS \
  --kernel-include-regex "k_count_slab|k_count_trie" --output-format csv -d "$R/gpurun_out/pmc/${TAG}_a" -o run -- \
  python3 "$R/bench.py" --config T40I10D10M --steps 1 --warmup 0 --e2e off > "$R/gpurun_out/pmc/${TAG}_a.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_count_slab|k_count_trie" --output-format csv -d "$R/gpurun_out/pmc/${TAG}_b" -o run -- \
  python3 "$R/bench.py" --config T40I10D10M --steps 1 --warmup 0 --e2e off > "$R/gpurun_out/pmc/${TAG}_b.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_${TAG}10M" -o run -- \
  python3 "$R/bench.py" --config T40I10D10M --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_${TAG}10M.log" 2>&1
cd "$R"
timeout -k 10 300 python benchmarks/slab_probe.py --config T10I4D100M > gpurun_out/slab_probe_T10.txt 2>&1
