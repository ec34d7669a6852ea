#!/bin/bash
# round 4: changed-path GPU tests, the e2e window breakdown, kernel stats of the read path
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/e2e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_log_parity.py tests/test_gpu_end_to_end.py tests/test_gpu_device_levels.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 --job > $O/probe.json 2> $O/probe.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
  python3 "$R/benchmarks/e2e_probe.py" --reps 1 > "$O/kt.log" 2>&1
