#!/bin/bash
# round 4 iteration pass: parser + changed-path tests, e2e breakdown, kernel stats of the
# read path, T40 device multi-pass A/B and its marker trace (host gaps)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/it
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parse.py tests/test_log_parity.py tests/test_gpu_kernels.py tests/test_gpu_device_levels.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_parse.log 2>&1
for v in 1 0; do
  FA_FUSED_LAYOUT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --e2e off > $O/T10_fused$v.json 2> $O/T10_fused$v.err
done
timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 --job > $O/probe.json 2> $O/probe.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
  python3 "$R/benchmarks/e2e_probe.py" --reps 1 > "$O/kt.log" 2>&1
cd $R
for val in 1 0; do
  FA_DL_MULTI=$val timeout -k 10 400 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > $O/T40_multi$val.json 2> $O/T40_multi$val.err
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/k40" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 0 --e2e off > "$O/k40.log" 2>&1
