set -e -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5_gram; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gram" > $O/tests.log 2>&1
timeout -k 10 400 python bench.py --config T40I10D100M --steps 2 --warmup 1 --e2e off > $O/T40.json 2> $O/T40.err
