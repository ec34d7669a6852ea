#!/bin/bash
# round 4 iteration pass: parser/e2e tests, then the e2e probe with 1 / 2 H2D copy streams
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/it
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parse.py tests/test_gpu_end_to_end.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_parse.log 2>&1
for v in 2 1 2 1; do
  FA_COPY_STREAMS=$v timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 > $O/probe_cs$v.json 2> $O/probe_cs$v.err
  grep -v "^====" $O/probe_cs$v.json | tail -1 >> $O/probe_cs$v.all
done
