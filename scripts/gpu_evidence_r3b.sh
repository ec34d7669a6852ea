#!/bin/bash
# Round-3 evidence on one MI355X for the tree as committed: every BASELINE config's bench
# line, the 12.5M-row shard, kernel tables of T10I4D100M and T40I10D100M, PMC of the hot
# kernels (one counter set per rocprofv3 pass), kernel + marker traces (GPU idle by host
# range) of the headline and the shard.
set -e -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ev
mkdir -p $O $O/pmc
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_T10I4D100M.json 2> $O/bench_T10I4D100M.err
timeout -k 10 300 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off > $O/bench_shard12.json 2> $O/bench_shard12.err
timeout -k 10 300 python bench.py --config T10I4D100K --steps 30 --warmup 5 > $O/bench_T10I4D100K.json 2> $O/bench_T10I4D100K.err
timeout -k 10 300 python bench.py --config T10I4D1K --steps 30 --warmup 5 > $O/bench_T10I4D1K.json 2> $O/bench_T10I4D1K.err
timeout -k 10 300 python bench.py --config webdocs --steps 5 --warmup 1 > $O/bench_webdocs.json 2> $O/bench_webdocs.err
timeout -k 10 400 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > $O/bench_T40I10D100M.json 2> $O/bench_T40I10D100M.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_T10" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$O/kt_T10.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_T40" -o run -- \
  python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$O/kt_T40.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS \
  --kernel-include-regex "k_pair_queue16|k_count_slab" --output-format csv -d "$O/pmc/a" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --e2e off > "$O/pmc/a.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_pair_queue16|k_count_slab" --output-format csv -d "$O/pmc/b" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --e2e off > "$O/pmc/b.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$O/mkh" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --e2e off > "$O/mkh.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$O/mk12" -o run -- \
  python3 "$R/bench.py" --n-txn 12500000 --steps 2 --warmup 1 --e2e off > "$O/mk12.log" 2>&1
