#!/bin/bash
# GPU measurement passes on one MI355X (run through gpurun).  Every GPU step runs under
# its own timeout and the steps are chained by `set -e`; output lands under
# gpurun_out/<pass>/ and the summaries worth keeping are copied into profiles/.
#
#   bash scripts/gpu_pass.sh round              the driver's round-end sequence: GPU tests, smoke(), bench line
#   bash scripts/gpu_pass.sh tests [-k EXPR]    GPU tests (optionally a subset)
#   bash scripts/gpu_pass.sh bench              the bench line of every BASELINE config + the 12.5M-row shard
#   bash scripts/gpu_pass.sh kernels            rocprofv3 kernel stats of T10I4D100M and T40I10D100M
#   bash scripts/gpu_pass.sh pmc [REGEX] [CFG]  four PMC passes (SQ sets, FETCH_SIZE, WRITE_SIZE) of the matching kernels
#   bash scripts/gpu_pass.sh trace [CFG]        kernel + roctx marker trace (benchmarks/gap_attrib.py: GPU idle by host range)
#   bash scripts/gpu_pass.sh e2e                the reference window's breakdown (benchmarks/e2e_probe.py) + its kernel stats
#   bash scripts/gpu_pass.sh multirank          8 gloo ranks sharing the GPU: collectives per run (benchmarks/multirank_probe.py)
#   bash scripts/gpu_pass.sh ab KNOB A B [CFG]  alternating bench runs with FA_TUNE=KNOB=A / KNOB=B (fastapriori_amd/tuning.py)
#   bash scripts/gpu_pass.sh head             tests + multirank + e2e + kernel stats of T10 and T40 (one HEAD's evidence)
#   bash scripts/gpu_pass.sh cpu                the C++ CPU comparator of vs_baseline (no GPU work)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
MODE=${1:-round}
shift || true
O=$R/gpurun_out/$MODE
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"

pytest_gpu() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@"
}

case "$MODE" in
  round)
    pytest_gpu > "$O/tests.log" 2>&1
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
    timeout -k 10 500 python bench.py > "$O/bench.json" 2> "$O/bench.err"
    ;;
  tests)
    if [ "$1" = "-k" ]; then pytest_gpu -k "$2" > "$O/tests.log" 2>&1; else pytest_gpu > "$O/tests.log" 2>&1; fi
    ;;
  bench)
    timeout -k 10 500 python bench.py --steps 20 --warmup 5 > "$O/T10I4D100M.json" 2> "$O/T10I4D100M.err"
    timeout -k 10 300 python bench.py --n-txn 12500000 --steps 40 --warmup 3 --e2e off > "$O/shard12.json" 2> "$O/shard12.err"
    timeout -k 10 300 python bench.py --config T10I4D100K --steps 30 --warmup 5 > "$O/T10I4D100K.json" 2> "$O/T10I4D100K.err"
    timeout -k 10 300 python bench.py --config T10I4D1K --steps 30 --warmup 5 > "$O/T10I4D1K.json" 2> "$O/T10I4D1K.err"
    timeout -k 10 300 python bench.py --config webdocs --steps 5 --warmup 1 > "$O/webdocs.json" 2> "$O/webdocs.err"
    timeout -k 10 500 python bench.py --config T40I10D100M --steps 3 --warmup 1 --e2e off > "$O/T40I10D100M.json" 2> "$O/T40I10D100M.err"
    ;;
  kernels)
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/T10" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$O/T10.log" 2>&1
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/T40" -o run -- \
      python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$O/T40.log" 2>&1
    ;;
  pmc)
    RX=${1:-"k_pair_queue16|k_count_slab"}
    CFG=${2:-T10I4D100M}
    cd /tmp
    timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS \
      --kernel-include-regex "$RX" --output-format csv -d "$O/a" -o run -- \
      python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --e2e off > "$O/a.log" 2>&1
    timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
      --kernel-include-regex "$RX" --output-format csv -d "$O/b" -o run -- \
      python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --e2e off > "$O/b.log" 2>&1
    # HBM bytes (FETCH_SIZE takes 3 of the 4 TCC counters, WRITE_SIZE 2: one pass each)
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE SQ_WAVES GRBM_GUI_ACTIVE \
      --kernel-include-regex "$RX" --output-format csv -d "$O/c" -o run -- \
      python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --e2e off > "$O/c.log" 2>&1
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE SQ_WAVES GRBM_GUI_ACTIVE \
      --kernel-include-regex "$RX" --output-format csv -d "$O/d" -o run -- \
      python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 0 --e2e off > "$O/d.log" 2>&1
    ;;
  trace)
    CFG=${1:-T10I4D100M}
    cd /tmp
    timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$O/$CFG" -o run -- \
      python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 1 --e2e off > "$O/$CFG.log" 2>&1
    ;;
  e2e)
    timeout -k 10 500 python benchmarks/e2e_probe.py --reps 3 --job > "$O/probe.json" 2> "$O/probe.err"
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
      python3 "$R/benchmarks/e2e_probe.py" --reps 1 > "$O/kt.log" 2>&1
    ;;
  multirank)
    timeout -k 10 600 python benchmarks/multirank_probe.py --world 8 --n-txn 4000000 > "$O/multirank.json" 2> "$O/multirank.err"
    ;;
  ab)
    V=$1; A=$2; B=$3; CFG=${4:-T10I4D100M}
    for i in 1 2; do
      for val in "$A" "$B"; do
        env "FA_TUNE=$V=$val" timeout -k 10 500 python bench.py --config "$CFG" --steps 10 --warmup 2 --e2e off \
          > "$O/${CFG}_${V}_${val}_$i.json" 2> /dev/null
      done
    done
    ;;
  head)
    # the evidence set of one HEAD: GPU tests, kernel stats of both configs, the 8-rank
    # rehearsal, the e2e breakdown
    pytest_gpu > "$O/tests.log" 2>&1
    timeout -k 10 600 python benchmarks/multirank_probe.py --world 8 --n-txn 4000000 > "$O/multirank.json" 2> "$O/multirank.err"
    timeout -k 10 400 python benchmarks/e2e_probe.py --reps 3 --job > "$O/probe.json" 2> "$O/probe.err"
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/T10" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 1 --e2e off > "$O/T10.log" 2>&1
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/T40" -o run -- \
      python3 "$R/bench.py" --config T40I10D100M --steps 1 --warmup 1 --e2e off > "$O/T40.log" 2>&1
    ;;
  cpu)
    for c in T10I4D1K T10I4D100K; do
      timeout -k 10 300 python benchmarks/run_bench.py --config $c --mode cpu --device cpu --steps 3 --warmup 1 > "$O/$c.json" 2> "$O/$c.err"
    done
    timeout -k 10 600 python benchmarks/run_bench.py --config T10I4D100M --mode cpu --device cpu --steps 1 --warmup 0 > "$O/T10I4D100M.json" 2> "$O/T10I4D100M.err"
    ;;
  *)
    echo "unknown pass $MODE" >&2
    exit 2
    ;;
esac
