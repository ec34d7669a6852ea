set -e
mkdir -p gpurun_out
export FA_PHASE_TIMING=1
for n in 12500000 25000000 50000000; do
timeout -k 10 200 python bench.py --n-txn $n --steps 5 --warmup 1 > gpurun_out/scale_$n.json 2> gpurun_out/scale_$n.err
done
unset FA_PHASE_TIMING
timeout -k 10 200 python bench.py --n-txn 12500000 --steps 10 --warmup 2 > gpurun_out/scale_nosync_12500000.json 2>&1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/nosync_100M.json 2>&1
