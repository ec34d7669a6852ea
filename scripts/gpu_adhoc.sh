set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --config webdocs --steps 3 --warmup 1 > gpurun_out/bench_webdocs.json 2> gpurun_out/bench_webdocs.err
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_T10I4D100M.json 2> gpurun_out/bench_T10I4D100M.err
