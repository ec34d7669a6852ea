#!/bin/bash
# T40I10D100M evidence on one MI355X: the bench line and rocprofv3 kernel stats
# (gpurun_out/t40ev; copy summaries into profiles/).
set -e -o pipefail
O=gpurun_out/t40ev; mkdir -p $O
timeout -k 10 300 python bench.py --config T40I10D100M --steps 3 --warmup 1 > $O/bench_T40I10D100M.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py --config T40I10D100M --steps 1 --warmup 1 --e2e off > $O/kt.log 2>&1
