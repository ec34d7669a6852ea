#!/bin/bash
# Kernel tables (rocprofv3 --kernel-trace --stats) of the headline under two settings
# of an env toggle, plus a bench A/B of a second toggle.
# usage: bash scripts/gpu_kt_ab.sh VAR A B [VAR2 A2 B2]
set -e -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=$1; A=$2; B=$3
cd /tmp
for val in $A $B; do
  export $V=$val
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_${V}_$val" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/kt_${V}_$val.log" 2>&1
done
unset $V
cd "$R"
if [ -n "$4" ]; then
  for i in 1 2; do
    for val in $5 $6; do
      env $4=$val timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/abf_T10_${val}_$i.json 2>/dev/null
    done
  done
fi
