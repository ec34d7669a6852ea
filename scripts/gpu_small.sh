#!/bin/bash
# small-config A/B (launch-bound): T10I4D100K under FA_GEN_DEVCHAIN=1/0 and FA_PAIR_FLAT=2/0
set -e -o pipefail
mkdir -p gpurun_out
for e in "FA_GEN_DEVCHAIN=1" "FA_GEN_DEVCHAIN=0" "FA_PAIR_FLAT=0" "FA_GEN_DEVCHAIN=1"; do
  env $e timeout -k 10 300 python bench.py --config T10I4D100K --steps 20 --warmup 3 > gpurun_out/sm_$e.json 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/sm_$e.json').read().strip().splitlines()[-1]);print('$e', d['ms_per_step'])" >> gpurun_out/sm_summary.txt
done
FA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --config T10I4D100K --steps 5 --warmup 3 > gpurun_out/sm_phase.json 2>/dev/null
