#!/bin/bash
# headline evidence: PMC passes of the hot kernels (scripts/gpu_pmc_hot.sh) and the
# slab-kernel build/count split of every level call (benchmarks/slab_probe.py)
set -e -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_pmc_hot.sh ${1:-r2b}
timeout -k 10 300 python benchmarks/slab_probe.py --config T10I4D100M > gpurun_out/slab_probe_T10.txt 2> gpurun_out/slab_probe_T10.err
