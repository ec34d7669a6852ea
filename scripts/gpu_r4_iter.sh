#!/bin/bash
# round 4 scratch pass: lane-split slab counting (FA_SLAB_LANES)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lanes
mkdir -p $O
export TMPDIR=/tmp
FA_SLAB_LANES=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_device_levels.py tests/test_oracle_deep.py tests/test_gpu_kernels.py -m gpu > $O/tests.log 2>&1
run() {   # name, env..., then bench args after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 400 python bench.py "$@" --e2e off > $O/$name.json 2> $O/$name.err
  tail -1 $O/$name.json >> $O/all.jsonl
  echo "$name" >> $O/names.txt
}
for i in 1 2; do
  run T10_lanes FA_SLAB_LANES=1 -- --steps 10 --warmup 2
  run T10_base FA_SLAB_LANES=0 -- --steps 10 --warmup 2
done
for i in 1 2; do
  run T40_lanes FA_SLAB_LANES=1 -- --config T40I10D100M --steps 2 --warmup 1
  run T40_base FA_SLAB_LANES=0 -- --config T40I10D100M --steps 2 --warmup 1
done
