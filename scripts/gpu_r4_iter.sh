#!/bin/bash
# round 4 scratch pass: fewest-pass slab width for window-by-window levels (FA_DL_MP_MINPASS)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/minpass
mkdir -p $O
export TMPDIR=/tmp
FA_DL_MP_MINPASS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_device_levels.py -m gpu > $O/tests.log 2>&1
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
  run T40_base FA_X=0 -- --config T40I10D100M --steps 2 --warmup 1
  run T40_minpass FA_DL_MP_MINPASS=1 -- --config T40I10D100M --steps 2 --warmup 1
done
