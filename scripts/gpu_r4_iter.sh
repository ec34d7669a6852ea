#!/bin/bash
# round 4 iteration pass: changed-path GPU tests, headline A/B (fused pair layout),
# then the PMC passes of the headline's hot kernels and of T40's slab dispatches
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/it
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_end_to_end.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_parse.log 2>&1
for v in 1 0 1; do
  FA_FUSED_LAYOUT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --e2e off > $O/T10_fused$v.json 2> $O/T10_fused$v.err
done
timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 --job > $O/probe.json 2> $O/probe.err
bash scripts/gpu_pass.sh pmc "k_pair_queue16|k_count_slab|k_cmp_emit|k_cmp_agg|k_histogram" T10I4D100M
mv gpurun_out/pmc gpurun_out/pmc_T10
bash scripts/gpu_pass.sh pmc "k_count_slab|k_pair_gram" T40I10D100M
mv gpurun_out/pmc gpurun_out/pmc_T40
