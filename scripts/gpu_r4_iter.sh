#!/bin/bash
# round 4 scratch pass: Gram launch size (FA_GRAM_WGS)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wgs
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k gram > $O/tests.log 2>&1
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
  run T40_w4096 FA_GRAM_WGS=4096 -- --config T40I10D100M --steps 1 --warmup 1
  run T40_w2048 FA_GRAM_WGS=2048 -- --config T40I10D100M --steps 1 --warmup 1
  run T40_w1024 FA_GRAM_WGS=1024 -- --config T40I10D100M --steps 1 --warmup 1
  run T40_w8192 FA_GRAM_WGS=8192 -- --config T40I10D100M --steps 1 --warmup 1
done
