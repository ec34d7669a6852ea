"""Time decomposition of the k = 2 pair kernel on a real mining run.

Mines a config once, recording the arguments of the ops.pair_counts_horizontal
call, then replays it under FA_PAIR_DEBUG = 0 (full), 1 (no scatter), 2 (no
flush), 3 (neither), 4 (layout kernels only) and each FA_PAIR_FLAT setting given,
and prints the times (CUDA events, median of --reps) plus a check that every full
variant returns identical counts.

    python benchmarks/pair_probe.py --config T10I4D100M --flat 2,1
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from fastapriori_amd import ops  # noqa: E402
from fastapriori_amd.models import apriori  # noqa: E402
from fastapriori_amd.models.apriori import FastApriori, MinerConfig  # noqa: E402
from fastapriori_amd.parallel.comm import Comm  # noqa: E402
from fastapriori_amd.utils.io import generate_shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="T10I4D100M")
    ap.add_argument("--n-txn", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="0,1,2,3,4")
    ap.add_argument("--flat", default="", help="comma list of FA_PAIR_FLAT values")
    a = ap.parse_args()
    n, L, I, P, N, ms = bench.CONFIGS[a.config]
    n = a.n_txn or n
    shard = generate_shard(n, Comm(), "cuda", L, I, P, N, 1)
    calls = []
    real = ops.pair_counts_horizontal

    def rec(*args, **kw):
        calls.append((args, kw))
        return real(*args, **kw)

    apriori.ops.pair_counts_horizontal = rec
    FastApriori(ms, config=MinerConfig(min_support=ms, pair_strategy="horizontal")).run(shard)
    apriori.ops.pair_counts_horizontal = real
    args, kw = calls[0]
    lens = (args[0][1:] - args[0][:-1]).to(torch.int64)
    print(json.dumps({"rows": int(lens.numel()), "nnz": int(lens.sum()),
                      "pair_increments": int((lens * (lens - 1) // 2).sum())}), flush=True)
    ref = None
    for kern in (a.flat.split(",") if a.flat else [""]):
        if kern:
            os.environ["FA_PAIR_FLAT"] = kern
        row = {"kernel": kern or "default"}
        for mode in a.modes.split(","):
            os.environ["FA_PAIR_DEBUG"] = mode
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out = real(*args, **kw)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            row[f"mode{mode}_ms"] = round(sorted(ts)[len(ts) // 2], 3)
            if mode == "0":
                if ref is None:
                    ref = out
                row["matches_first"] = bool(torch.equal(out, ref))
        os.environ["FA_PAIR_DEBUG"] = "0"
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
