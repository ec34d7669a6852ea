#!/bin/bash
# round 4 iteration pass: changed-path GPU tests, then T10 / T40 bench lines and the e2e probe
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/it
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_device_levels.py tests/test_gpu_end_to_end.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_parse.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --e2e off > $O/T10.json 2> $O/T10.err
timeout -k 10 400 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > $O/T40.json 2> $O/T40.err
FA_BITMAP_WAVE=0 FA_FREQ_WV=0 timeout -k 10 400 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > $O/T40_old.json 2> $O/T40_old.err
timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 --job > $O/probe.json 2> $O/probe.err
