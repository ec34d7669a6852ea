#!/bin/bash
# round 4 iteration pass: changed-path GPU tests, headline A/B (fused pair layout),
# T40 A/B (device class layout / device multi-pass / host loop), e2e probes (ring size)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/it
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_device_levels.py tests/test_gpu_parse.py tests/test_log_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_parse.log 2>&1
for v in 1 0; do
  FA_FUSED_LAYOUT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --e2e off > $O/T10_fused$v.json 2> $O/T10_fused$v.err
done
for v in 5 0; do
  FA_DL_CLS_MIN_M=$v timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > $O/T40_cls$v.json 2> $O/T40_cls$v.err
done
FA_DL_MULTI=0 timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > $O/T40_multi0.json 2> $O/T40_multi0.err
timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 --job > $O/probe.json 2> $O/probe.err
FA_RING_SLOTS=8 timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 > $O/probe8.json 2> $O/probe8.err
