#!/bin/bash
# round 4 parameter sweep: headline bundle growth / dense test, T40 slab width order
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sweep
mkdir -p $O
export TMPDIR=/tmp
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
  run T10_base FA_X=0 -- --steps 10 --warmup 2
  run T10_g1 FA_BUNDLE_GROWTH=1.0 -- --steps 10 --warmup 2
  run T10_g3 FA_BUNDLE_GROWTH=3.0 -- --steps 10 --warmup 2
  run T10_dense FA_DENSE_MIN_ROWS=0.4 -- --steps 10 --warmup 2
done
for i in 1 2; do
  run T40_base FA_X=0 -- --config T40I10D100M --steps 2 --warmup 1
  run T40_sw32 FA_DL_SW_ORDER=32,16,8,4 -- --config T40I10D100M --steps 2 --warmup 1
done
