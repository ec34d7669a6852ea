"""Time decomposition of the k >= 3 slab kernel on a real mining run.

Mines a config once, recording the arguments of every ops.count_level call
(slab kernel, bundles included), then replays each call under FA_SLAB_DEBUG = 0 (full), 1 (no slab build),
2 (no counting), 3 (neither: launch + prefetch + final atomics) and prints the
per-level times (CUDA events, median of --reps).

    python benchmarks/slab_probe.py --config T10I4D100M
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="0,1,2,3")
    a = ap.parse_args()
    n, L, I, P, N, ms = bench.CONFIGS[a.config]
    shard = generate_shard(n, Comm(), "cuda", L, I, P, N, 1)
    calls = []
    real = ops.count_level

    def rec(*args, **kw):
        calls.append((real, args, kw))
        return real(*args, **kw)

    apriori.ops.count_level = rec
    FastApriori(ms, config=MinerConfig(min_support=ms)).run(shard)
    apriori.ops.count_level = real
    out = []
    for i, (fn, args, kw) in enumerate(calls):
        row = {"call": i, "fn": fn.__name__}
        for mode in a.modes.split(","):
            os.environ["FA_SLAB_DEBUG"] = mode
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(*args, **kw)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            row[f"mode{mode}_ms"] = round(sorted(ts)[len(ts) // 2], 3)
        row.update(ops.primitives.LAST_LEVEL_PLAN)
        out.append(row)
        print(json.dumps(row), flush=True)
    os.environ["FA_SLAB_DEBUG"] = "0"


if __name__ == "__main__":
    main()
