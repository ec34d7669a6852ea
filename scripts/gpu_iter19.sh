#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_end_to_end.py -x -v --timeout 200 --timeout-method thread > gpurun_out/e2e_tests.log 2>&1
FA_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 > gpurun_out/it19_T10_rccl1.json 2> gpurun_out/it19_T10_rccl1.err
FA_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/it19_12M_rccl1.json 2> gpurun_out/it19_12M_rccl1.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 1 --steps 5 --warmup 1 > gpurun_out/it19_T10_trun.json 2> gpurun_out/it19_T10_trun.err
