#!/bin/bash
# The C++ CPU path of the same miner on the box's host CPU share (16 threads), for
# bench.py's vs_baseline (benchmarks/cpu_baselines.json).  No GPU work.
set -e -o pipefail
mkdir -p gpurun_out/cpu
for c in T10I4D1K T10I4D100K; do
  timeout -k 10 300 python benchmarks/run_bench.py --config $c --mode cpu --device cpu --steps 3 --warmup 1 > gpurun_out/cpu/$c.json 2> gpurun_out/cpu/$c.err
done
timeout -k 10 600 python benchmarks/run_bench.py --config T10I4D100M --mode cpu --device cpu --steps 1 --warmup 0 > gpurun_out/cpu/T10I4D100M.json 2> gpurun_out/cpu/T10I4D100M.err
