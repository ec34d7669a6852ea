set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
FA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_T10I4D100M.json 2> gpurun_out/bench_T10I4D100M.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/kt_T10I4D100M" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/kt_T10I4D100M.log" 2>&1
