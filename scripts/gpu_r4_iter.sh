#!/bin/bash
# round 4 evidence pass at HEAD: kernel stats of both configs, then the headline's PMC passes
set -e -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"
bash scripts/gpu_pass.sh kernels
bash scripts/gpu_pass.sh pmc "k_pair_queue16|k_count_slab|k_cmp_emit|k_cmp_agg|k_histogram" T10I4D100M
