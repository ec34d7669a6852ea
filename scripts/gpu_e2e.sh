#!/bin/bash
# End-to-end CLI job (file write -> parse -> mine -> rules -> write) on the GPU,
# and the CPU (C++ path) mining baseline, each under its own time limit.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python benchmarks/run_bench.py --config T10I4D10M --mode e2e --device cuda --steps 2 --warmup 1 > gpurun_out/e2e_T10I4D10M.json 2> gpurun_out/e2e_T10I4D10M.err
timeout -k 10 600 python benchmarks/run_bench.py --config T10I4D100M --mode e2e --device cuda --steps 1 --warmup 1 > gpurun_out/e2e_T10I4D100M.json 2> gpurun_out/e2e_T10I4D100M.err
timeout -k 10 600 python benchmarks/run_bench.py --config T10I4D10M --mode cpu --steps 1 --warmup 0 > gpurun_out/cpu_T10I4D10M.json 2> gpurun_out/cpu_T10I4D10M.err
