#!/bin/bash
# same-box A/B: 12.5M-row shard with and without a (world-1) RCCL process group
set -e
mkdir -p gpurun_out
: > gpurun_out/ab_pg.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --n-txn 12500000 --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; print('plain', json.loads(sys.stdin.read())['ms_per_step'])" >> gpurun_out/ab_pg.txt
  FA_FORCE_PG=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2954$i bench.py --n-txn 12500000 --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; print('rccl1', json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])" >> gpurun_out/ab_pg.txt
done
