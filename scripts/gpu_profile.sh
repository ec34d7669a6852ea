#!/bin/bash
# One-GPU measurement pass for the docs: GPU tests, every BASELINE config's bench,
# the 12.5M-row shard (per-rank work at 8 GPUs), and rocprofv3 kernel stats of the
# headline and deep-k configs.  Every GPU step has its own time limit.
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_T10I4D100M.json 2> gpurun_out/bench_T10I4D100M.err
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 20 --warmup 3 --e2e off > gpurun_out/bench_shard12.json 2> gpurun_out/bench_shard12.err
timeout -k 10 300 python bench.py --config T10I4D100K --steps 20 --warmup 3 > gpurun_out/bench_T10I4D100K.json 2> gpurun_out/bench_T10I4D100K.err
timeout -k 10 300 python bench.py --config T10I4D1K --steps 20 --warmup 3 > gpurun_out/bench_T10I4D1K.json 2> gpurun_out/bench_T10I4D1K.err
timeout -k 10 300 python bench.py --config webdocs --steps 5 --warmup 1 > gpurun_out/bench_webdocs.json 2> gpurun_out/bench_webdocs.err
FA_PHASE_TIMING=1 timeout -k 10 500 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > gpurun_out/bench_T40I10D100M.json 2> gpurun_out/bench_T40I10D100M.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_T10" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_T10.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_T40" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_T40.log" 2>&1
