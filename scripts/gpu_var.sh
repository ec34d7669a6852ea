#!/bin/bash
# run-to-run spread of the headline on one box (5 separate processes, 20 timed steps each)
set -e -o pipefail
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > gpurun_out/var_$i.json 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/var_$i.json').read().strip().splitlines()[-1]);print($i, d['ms_per_step'])" >> gpurun_out/var_summary.txt
done
