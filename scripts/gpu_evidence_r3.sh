#!/bin/bash
# Round-3 evidence on one MI355X: every BASELINE config's bench line, the 12.5M-row
# shard, a T40 A/B of the trie threshold, kernel tables of T10 / T40, PMC of the hot
# kernels (fresh counters, one counter set per rocprofv3 pass).
set -e -o pipefail
mkdir -p gpurun_out/ev gpurun_out/pmc
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/ev/bench_T10I4D100M.json 2> gpurun_out/ev/bench_T10I4D100M.err
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 30 --warmup 3 --e2e off > gpurun_out/ev/bench_shard12.json 2> gpurun_out/ev/bench_shard12.err
timeout -k 10 300 python bench.py --config T10I4D100K --steps 30 --warmup 5 > gpurun_out/ev/bench_T10I4D100K.json 2> gpurun_out/ev/bench_T10I4D100K.err
timeout -k 10 300 python bench.py --config T10I4D1K --steps 30 --warmup 5 > gpurun_out/ev/bench_T10I4D1K.json 2> gpurun_out/ev/bench_T10I4D1K.err
timeout -k 10 300 python bench.py --config webdocs --steps 5 --warmup 1 > gpurun_out/ev/bench_webdocs.json 2> gpurun_out/ev/bench_webdocs.err
for v in 0.3 0.5; do
  FA_TRIE_MIN_SAVING=$v timeout -k 10 400 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > gpurun_out/ev/t40_trie_$v.json 2> gpurun_out/ev/t40_trie_$v.err
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ev/kt_T10" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/ev/kt_T10.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ev/kt_T40" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$R/gpurun_out/ev/kt_T40.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU \
  --kernel-include-regex "k_pair_queue16|k_count_slab" --output-format csv -d "$R/gpurun_out/pmc/r3_a" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --e2e off > "$R/gpurun_out/pmc/r3_a.log" 2>&1
