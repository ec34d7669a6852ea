#!/bin/bash
# round 4: the tile parser (streamed), its tests, the e2e window breakdown and kernel stats
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/parse
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parse.py tests/test_build_provenance.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 --job > $O/probe.json 2> $O/probe.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
  python3 "$R/benchmarks/e2e_probe.py" --reps 1 > "$O/kt.log" 2>&1
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/all_tests.log 2>&1
