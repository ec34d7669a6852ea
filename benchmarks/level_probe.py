"""Per-bundle plan records of one mining run and the used-item row lengths behind them.

    python benchmarks/level_probe.py [--config T10I4D100M] [--n-txn N]

Prints the per-level metric records of the device loop (slab width, used items,
candidates, rows counted, device ms) and, for every level k >= 3, the share of the
compressed rows with fewer than k items among the items of F_{k-1}: rows that no
k-candidate can be contained in (what transaction trimming could drop).
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="T10I4D100M")
    ap.add_argument("--n-txn", type=int, default=0)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger
    n, avg_len, avg_pat, n_pat, n_items, ms = bench.CONFIGS[a.config]
    n = a.n_txn or n
    dev = torch.device("cuda", 0)
    comm = Comm(device=dev)
    shard = generate_shard(n, comm, dev, avg_len, avg_pat, n_pat, n_items, 1)
    mp = os.path.join(tempfile.mkdtemp(), "m.jsonl")
    miner = FastApriori(ms, comm, MinerConfig(min_support=ms), Logger(0, enabled=False))
    keep = {}
    orig = miner._compress

    def grab(*aa, **kw):
        db = orig(*aa, **kw)
        keep["roff"], keep["ranks"], keep["F1"] = db["roff"].clone(), db["ranks"].clone(), db["F1"]
        return db
    miner._compress = grab
    miner.run(shard)
    miner.log = Logger(0, enabled=False, metrics_path=mp)
    res = miner.run(shard)
    torch.cuda.synchronize()
    for line in open(mp):
        r = json.loads(line)
        if r.get("phase") in ("level", "compress", "pairs"):
            print(json.dumps({k: v for k, v in r.items() if not k.startswith("_")}))
    db = keep
    roff = db["roff"].cpu().numpy()
    ranks = db["ranks"].cpu().numpy()
    lens = np.diff(roff)
    print("rows", lens.size, "mean len", round(float(lens.mean()), 2), "F1", db["F1"])
    row_of = np.repeat(np.arange(lens.size), lens)
    for k in range(3, len(res.levels) + 1):
        prev = res.levels[k - 2]
        used = np.zeros(db["F1"], bool)
        used[np.unique(prev)] = True
        cnt = np.bincount(row_of[used[ranks]], minlength=lens.size)
        print(f"k={k} used={int(used.sum())} rows>= k: {float((cnt >= k).mean()):.3f} "
              f"used-nnz share {float(cnt[cnt >= k].sum() / max(1, ranks.size)):.3f}")


if __name__ == "__main__":
    main()
