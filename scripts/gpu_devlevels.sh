#!/bin/bash
# device-resident level bundles: new tests, the GPU suite, A/B bench (FA_DEVICE_LEVELS 1 vs 0)
# on the headline and the 12.5M-row shard, and a marker trace of the shard for gap_attrib.py
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_levels.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dl_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dl_all.log 2>&1
for i in 1 2; do
  for v in 1 0; do
    FA_DEVICE_LEVELS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/dl_T10_${v}_$i.json 2>/dev/null
    FA_DEVICE_LEVELS=$v timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > gpurun_out/dl_s12_${v}_$i.json 2>/dev/null
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/gpurun_out/dlmk12" -o run -- \
  python3 "$R/bench.py" --n-txn 12500000 --steps 2 --warmup 1 --e2e off > "$R/gpurun_out/dlmk12.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$R/gpurun_out/dlmkh" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --e2e off > "$R/gpurun_out/dlmkh.log" 2>&1
cd "$R"
timeout -k 10 900 python benchmarks/run_bench.py --mode cpu --device cpu --config T10I4D100M --steps 1 --warmup 0 > gpurun_out/cpu_T10I4D100M.json 2> gpurun_out/cpu_T10I4D100M.err
