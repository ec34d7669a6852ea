"""cProfile of the host side of bench.py steps (which Python/C++ calls the level loop spends
its time in).  python benchmarks/host_profile.py --n-txn 12500000 [--config T10I4D100M]"""
import argparse
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from fastapriori_amd.models.apriori import FastApriori, MinerConfig  # noqa: E402
from fastapriori_amd.parallel.comm import Comm  # noqa: E402
from fastapriori_amd.utils.io import generate_shard  # noqa: E402
from fastapriori_amd.utils.metrics import Logger  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="T10I4D100M")
    ap.add_argument("--n-txn", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    n, L, I, P, N, ms = bench.CONFIGS[a.config]
    n = a.n_txn or n
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    shard = generate_shard(n, Comm(), dev, L, I, P, N, 1)
    miner = FastApriori(ms, Comm(), MinerConfig(min_support=ms), Logger(0, enabled=False))
    miner.run(shard)
    if dev == "cuda":
        torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        miner.run(shard)
    if dev == "cuda":
        torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
