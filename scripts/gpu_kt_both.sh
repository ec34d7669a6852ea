#!/bin/bash
# rocprofv3 kernel stats of the headline and the deep-k config (1 warmup + 1 timed
# mining run each; the e2e window is off so only mining kernels are traced)
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_T10" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_T10.log" 2>&1
if [ "${FA_KT_T40:-1}" = "1" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_T40" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_T40.log" 2>&1
fi
