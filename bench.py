"""Headline benchmark: frequent-itemset mining throughput on T10I4D100M, min_sup 0.1%.

BASELINE.json metric: "mining wall-clock + itemsets/sec, T10I4D100M min_sup=0.1%
at 1/2/4/8 GPU".  One step = one complete mining run over the fixed synthetic
database (F1 histogram + all-reduce, compression, vertical bitmaps, every
level's candidate generation + counting + all-reduce, results replicated on
every rank).  The database (100M Quest transactions, |T|=10, |I|=4, |L|=2000,
N=1000 items) is generated deterministically per rank and kept resident in HBM
before timing; parsing text is not part of the step (the CLI path parses with
the native mmap parser, measured separately by benchmarks/run_bench.py).
The total work is fixed as N grows, so scaling is "strong".

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config T10I4D100M]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (n_txn, avg_len, avg_pat_len, n_patterns, n_items, min_support)
    "T10I4D100M": (100_000_000, 10.0, 4.0, 2000, 1000, 0.001),
    "T10I4D10M": (10_000_000, 10.0, 4.0, 2000, 1000, 0.001),
    "T10I4D100K": (100_000, 10.0, 4.0, 2000, 1000, 0.005),
    "T10I4D1K": (1_000, 10.0, 4.0, 200, 50, 0.1),
    "T40I10D100M": (100_000_000, 40.0, 10.0, 2000, 1000, 0.005),
    "T40I10D10M": (10_000_000, 40.0, 10.0, 2000, 1000, 0.005),
    # wide vocabulary (Zipf-Mandelbrot words + topics, utils/io.generate_zipf_shard):
    # avg_len is the mean document length, avg_pat_len unused, n_patterns = topics
    "webdocs": (1_700_000, 177.0, 0.0, 2000, 5_267_656, 0.05),
    "webdocs100K": (100_000, 177.0, 0.0, 2000, 5_267_656, 0.05),
}
HEADLINE = "T10I4D100M"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=HEADLINE, choices=sorted(CONFIGS))
    ap.add_argument("--n-txn", type=int, default=0, help="override the number of transactions")
    ap.add_argument("--min-support", type=float, default=0.0)
    ap.add_argument("--pair-strategy", default="auto")
    ap.add_argument("--dedup", default="auto")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--strategy", choices=["count", "candidate"], default="count",
                    help="count: each rank generates its row shard; candidate: every rank holds all rows")
    args = ap.parse_args()

    import torch
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm, init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_shard, generate_zipf_shard
    from fastapriori_amd.utils.metrics import Logger

    dev = args.device if (args.device != "cuda" or torch.cuda.is_available()) else "cpu"
    comm = init_comm(dev)
    n_txn, avg_len, avg_pat, n_pat, n_items, ms = CONFIGS[args.config]
    n_txn = args.n_txn or n_txn
    min_sup = args.min_support or ms
    world = comm.world_size

    t_gen = time.perf_counter()
    data_comm = comm if args.strategy == "count" else Comm(device=comm.device)
    if args.config.startswith("webdocs"):
        shard = generate_zipf_shard(n_txn, data_comm, comm.device, mean_len=avg_len, n_items=n_items,
                                    n_topics=n_pat, seed=args.seed)
    else:
        shard = generate_shard(n_txn, data_comm, comm.device, avg_len, avg_pat, n_pat, n_items, args.seed)
    if comm.device.type == "cuda":
        torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen

    cfg = MinerConfig(min_support=min_sup, dedup=args.dedup, pair_strategy=args.pair_strategy,
                      parallelism=args.strategy)
    quiet = Logger(comm.rank, enabled=False)

    def sync():
        comm.barrier()
        if comm.device.type == "cuda":
            torch.cuda.synchronize()

    miner = FastApriori(min_sup, comm, cfg, quiet)
    res = None
    for _ in range(args.warmup):
        res = miner.run(shard)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = miner.run(shard)
    sync()
    elapsed = time.perf_counter() - t0
    ms_step = comm.allreduce_float_max(elapsed * 1e3 / max(args.steps, 1))
    n_sets = res.n_itemsets
    value = n_sets / (ms_step / 1e3)
    if comm.is_root:
        line = {
            "metric": f"itemsets/sec (mining wall-clock), {args.config} min_sup={min_sup:g}",
            "value": round(value, 2),
            "unit": "itemsets/s",
            "n_gpus": world if comm.device.type == "cuda" else 0,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32/uint64-bitmap (exact integer counts)",
            "data": (f"synthetic {'Zipf-topic' if args.config.startswith('webdocs') else 'Quest'} {args.config} "
                     f"(n={n_txn}, seed={args.seed}), generated in-process"),
            "config": {"model": args.config, "global_batch": n_txn, "seq_len": avg_len,
                       "parallelism": f"{'dp' if args.strategy == 'count' else 'cp'}{world}",
                       "min_support": min_sup,
                       "n_itemsets": n_sets, "levels": [len(c) for c in res.counts],
                       "pair_strategy": miner.stats.get("pair_strategy"),
                       "min_count": res.min_count, "gen_s": round(t_gen, 2),
                       **({"phase_ms": miner.stats["phase_ms"]} if "phase_ms" in miner.stats else {}),
                       **({"level_info": miner.stats["level_info"]} if "level_info" in miner.stats else {})},
        }
        print(json.dumps(line), flush=True)
    shutdown_comm(comm)
    return 0


if __name__ == "__main__":
    sys.exit(main())
