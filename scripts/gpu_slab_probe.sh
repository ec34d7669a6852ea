#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/slab_probe.py --config T10I4D100M > gpurun_out/slab_probe_T10.log 2>&1
