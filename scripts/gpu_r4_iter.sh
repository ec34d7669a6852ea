#!/bin/bash
# round 4 scratch pass: packed u16 accumulators in one-pass device bundles (FA_DL_ACC16)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/acc16b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
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
  run T10_acc16 FA_DL_ACC16=1 -- --steps 10 --warmup 2
  run T10_acc32 FA_DL_ACC16=0 -- --steps 10 --warmup 2
done
for i in 1 2; do
  run T40_acc16 FA_DL_ACC16=1 -- --config T40I10D100M --steps 2 --warmup 1
  run T40_acc32 FA_DL_ACC16=0 -- --config T40I10D100M --steps 2 --warmup 1
done
run T10K_acc16 FA_DL_ACC16=1 -- --config T10I4D100K --steps 20 --warmup 3
run T10K_acc32 FA_DL_ACC16=0 -- --config T10I4D100K --steps 20 --warmup 3
