#!/bin/bash
# Lane-pair slab kernel (k_count_slab_pl): its GPU tests, level plans of the headline and
# T40I10D100M, and alternating A/B runs against the padded record kernel.
set -e -o pipefail
mkdir -p gpurun_out/pl
O=gpurun_out/pl
timeout -k 10 500 python -u -m pytest tests/test_gpu_slab_pl.py tests/test_gpu_device_levels.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
FA_DEVICE_LEVELS=0 FA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --e2e off > $O/lv_T10.json 2> $O/lv_T10.err
for i in 1 2; do
  for v in 0 8192; do
    FA_SLAB_PL_MIN_CAP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e off > $O/T10_${v}_$i.json 2> $O/T10_${v}_$i.err
    FA_SLAB_PL_MIN_CAP=$v timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > $O/s12_${v}_$i.json 2> $O/s12_${v}_$i.err
  done
done
for v in 0 8192 4096; do
  FA_SLAB_PL_MIN_CAP=$v FA_PHASE_TIMING=1 timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > $O/T40_${v}.json 2> $O/T40_${v}.err
done
