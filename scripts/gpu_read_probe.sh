#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -c "from fastapriori_amd.utils.io import write_quest_file; write_quest_file('/tmp/D100M.dat', 100_000_000, 10.0, 4.0, 2000, 1000, seed=1)"
free -g > gpurun_out/read_probe.txt
timeout -k 10 300 python benchmarks/read_probe.py /tmp/D100M.dat >> gpurun_out/read_probe.txt 2>&1
rm -f /tmp/D100M.dat
