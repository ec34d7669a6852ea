"""Per-window record of the window-by-window levels of one mining run (FastApriori
stats["window_log"]: level, items, candidates, the compaction gate `keep`, the binomial
estimate and the rows kept, as shares of the level's rows).

    python benchmarks/window_probe.py [--config T40I10D100M] [--n-txn N]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="T40I10D100M")
    ap.add_argument("--n-txn", type=int, default=0)
    a = ap.parse_args()
    import torch
    import bench
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger
    n, al, ap_, npat, ni, ms = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    shard = generate_shard(a.n_txn or n, Comm(device=dev), dev, al, ap_, npat, ni, 1)
    m = FastApriori(ms, Comm(device=dev), MinerConfig(min_support=ms, timing="events"), Logger(0, enabled=False))
    m.run(shard)
    m.stats.pop("window_log", None)
    m.run(shard)
    for r in m.stats.get("window_log", []):
        print(json.dumps(r))
    print(json.dumps({k: round(v, 2) for k, v in m.stats.get("gpu_phase_ms", {}).items() if k.startswith("level")}))


if __name__ == "__main__":
    main()
