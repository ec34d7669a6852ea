#!/bin/bash
# Round-6 evidence pass at HEAD: bench lines of every config (+ T40I10D10M with its CPU
# digest), kernel stats of T10I4D100M and T40I10D100M, four PMC passes of T40's hot
# kernels.  Output under gpurun_out/{bench,kernels,pmc}/.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash scripts/gpu_pass.sh bench
timeout -k 10 300 python bench.py --config T40I10D10M --steps 5 --warmup 2 --e2e off > gpurun_out/bench/T40I10D10M.json 2> gpurun_out/bench/T40I10D10M.err
bash scripts/gpu_pass.sh kernels
bash scripts/gpu_pass.sh pmc "k_count_slab|k_win_|k_pair_gram|k_trim_emit|k_compress_staged|k_build_bitmaps" T40I10D100M
