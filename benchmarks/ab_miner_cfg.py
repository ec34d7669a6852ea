"""A/B of a MinerConfig field on one bench config (same shard, alternating runs):
    python benchmarks/ab_miner_cfg.py --config T40I10D100M --field trim --values 1 0 --reps 2"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from fastapriori_amd.models.apriori import FastApriori, MinerConfig  # noqa: E402
from fastapriori_amd.parallel.comm import Comm  # noqa: E402
from fastapriori_amd.utils.io import generate_shard  # noqa: E402
from fastapriori_amd.utils.metrics import Logger  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="T40I10D100M")
    ap.add_argument("--n-txn", type=int, default=0)
    ap.add_argument("--field", required=True)
    ap.add_argument("--values", nargs="+", required=True)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    n, L, I, P, N, ms = bench.CONFIGS[a.config]
    n = a.n_txn or n
    shard = generate_shard(n, Comm(), "cuda", L, I, P, N, 1)
    typ = type(getattr(MinerConfig(min_support=ms), a.field))
    vals = [(typ(int(v)) if typ is bool else typ(v)) for v in a.values]
    out = {str(v): [] for v in vals}
    for r in range(a.reps + 1):
        for v in vals:
            miner = FastApriori(ms, Comm(), MinerConfig(min_support=ms, **{a.field: v}), Logger(0, enabled=False))
            torch.cuda.synchronize()
            t = time.perf_counter()
            res = miner.run(shard)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) * 1e3
            if r:                                   # rep 0 warms both arms
                out[str(v)].append(round(dt, 2))
            print(json.dumps({"field": a.field, "value": str(v), "ms": round(dt, 2), "rep": r,
                              "itemsets": int(sum(len(x) for x in res.levels))}), flush=True)
    print(json.dumps({"summary": out}))


if __name__ == "__main__":
    main()
