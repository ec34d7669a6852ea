#!/bin/bash
# One-GPU measurement pass: GPU tests, benches of every BASELINE config, and a
# rocprofv3 kernel trace of the headline config.  Every GPU step has its own
# time limit; the chain stops at the first failure.
set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_T10I4D100M.json 2> gpurun_out/bench_T10I4D100M.err
timeout -k 10 300 python bench.py --config webdocs --steps 5 --warmup 1 > gpurun_out/bench_webdocs.json 2> gpurun_out/bench_webdocs.err
timeout -k 10 300 python bench.py --config T10I4D100K --steps 10 --warmup 2 > gpurun_out/bench_T10I4D100K.json 2> gpurun_out/bench_T10I4D100K.err
timeout -k 10 300 python bench.py --config T10I4D1K --steps 10 --warmup 2 > gpurun_out/bench_T10I4D1K.json 2> gpurun_out/bench_T10I4D1K.err
timeout -k 10 500 python bench.py --config T40I10D100M --steps 2 --warmup 1 > gpurun_out/bench_T40I10D100M.json 2> gpurun_out/bench_T40I10D100M.err
unset FA_PHASE_TIMING
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/kt_T10I4D100M" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/kt_T10I4D100M.log" 2>&1
