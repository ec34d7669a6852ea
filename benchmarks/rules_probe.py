"""Rule building on the host (C++) vs the device (HIP) for a mined result.

    python benchmarks/rules_probe.py [--config T10I4D10M]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import bench
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.models.rules import AssociationRules
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="T10I4D10M")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    n, L, I, P, N, ms = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    sh = generate_shard(n, Comm(device=dev), dev, L, I, P, N, 1)
    res = FastApriori(ms, config=MinerConfig(min_support=ms), logger=Logger(enabled=False)).run(sh)
    del sh
    out = {"config": a.config, "n_itemsets": res.n_itemsets}
    for name, d in (("host", None), ("device", dev)):
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rt = AssociationRules(res, logger=Logger(enabled=False), device=d).rules()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        out[name + "_ms"] = round(best * 1e3, 2)
        out[name + "_rules"] = rt.n_rules
        out[name + "_sig"] = int(np.asarray(rt.cons, dtype=np.int64).sum() + rt.ante.astype(np.int64).sum())
    users = generate_shard(max(n // 100, 1000), Comm(device=dev), dev, L, I, P, N, 1, users=True)
    ar = AssociationRules(res, logger=Logger(enabled=False), device=dev)
    ar.rules()
    recs = {}
    for name, idx in (("recommend_indexed", True), ("recommend_scan", False)):
        ar.use_index = idx
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = ar.recommend_shard(users)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        out[name + "_ms"] = round(best * 1e3, 2)
        recs[name] = r.cpu()
    out["users"] = users.n_lines
    out["recommend_agree"] = bool(torch.equal(recs["recommend_indexed"], recs["recommend_scan"]))
    out["users_with_rec"] = int((recs["recommend_indexed"] >= 0).sum())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
