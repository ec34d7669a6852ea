"""End-to-end and CPU-baseline benchmarks.

The reference publishes no numbers, so two baselines are measured here on the
same synthetic configs as bench.py:

* ``--mode e2e``: the full CLI job (``python -m fastapriori_amd in/ out/``):
  write D.dat/U.dat once (Quest generator), then time read+parse, mining,
  freqItemset write, rules + recommendations + write, on the chosen device.
  This is the reference's "mining wall-clock including read+parse+save"
  (Main.scala:28-32) and "get recommends" (Main.scala:34-37).
* ``--mode cpu``: mining only, on the multi-threaded C++ CPU path (CPU
  tensors through the same miner), i.e. our own non-GPU baseline.

Each run prints one JSON line.
    python benchmarks/run_bench.py --config T10I4D10M --mode e2e
    python benchmarks/run_bench.py --config T10I4D10M --mode cpu
"""
import argparse
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def _e2e(a, cfg):
    from fastapriori_amd.config import JobConfig
    from fastapriori_amd.pipeline import run_job
    from fastapriori_amd.utils.io import write_quest_file, write_zipf_file
    n, L, I, P, N, ms = cfg
    n = a.n_txn or n
    ms = a.min_support or ms
    d = os.path.join(a.workdir, f"{a.config}_{n}_{a.tokens}") + "/"
    os.makedirs(d, exist_ok=True)
    t0 = time.time()
    if not os.path.exists(d + "D.dat"):
        if a.config.startswith("webdocs"):
            # wide vocabulary: numeric ids or letter-string tokens (dictionary path)
            write_zipf_file(d + "D.dat", n, mean_len=L, n_items=N, n_topics=P, seed=1,
                            string_tokens=a.tokens == "str")
            write_zipf_file(d + "U.dat", max(n // 100, 1000), mean_len=L / 4, n_items=N, n_topics=P, seed=2,
                            string_tokens=a.tokens == "str")
        else:
            write_quest_file(d + "D.dat", n, L, I, P, N, seed=1)
            write_quest_file(d + "U.dat", max(n // 100, 1000), L, I, P, N, seed=1, users=True)
    gen_s = time.time() - t0
    out = os.path.join(a.workdir, "out") + "/"
    runs = []
    for _ in range(a.warmup + a.steps):
        job = JobConfig(input=d, output=out, temp="", min_support=ms, device=a.device, overwrite=True,
                        checkpoint=False)
        t, c = time.time(), time.process_time()
        s = run_job(job)
        s["total_ms"] = round((time.time() - t) * 1000, 1)
        s["host_cpu_s"] = time.process_time() - c      # host CPU time of this process (all threads)
        runs.append(s)
    best = min(runs[a.warmup:], key=lambda r: r["total_ms"])
    shutil.rmtree(out.rstrip("/") + "freqItemset", ignore_errors=True)
    return {"metric": f"end-to-end CLI job ms, {a.config} min_sup={ms}", "device": a.device, "n_txn": n,
            "tokens": a.tokens, "host_cpu_s": round(best.get("host_cpu_s", 0.0), 2),
            "D_bytes": os.path.getsize(d + "D.dat"), "gen_s": round(gen_s, 1),
            **{k: best[k] for k in ("total_ms", "read_ms", "mine_ms", "write_ms", "recommend_ms", "n_itemsets",
                                   "n_rules") if k in best},
            "mine_only_ms": round(best.get("miner", {}).get("mine_ms", 0.0), 1)}


def _cpu(a, cfg):
    import torch
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils.env import num_threads
    from fastapriori_amd.utils.io import generate_shard
    n, L, I, P, N, ms = cfg
    n = a.n_txn or n
    ms = a.min_support or ms
    shard = generate_shard(n, Comm(), "cpu", L, I, P, N, 1)
    times, res = [], None
    for _ in range(a.warmup + a.steps):
        t = time.time()
        res = FastApriori(ms, config=MinerConfig(min_support=ms)).run(shard)
        times.append((time.time() - t) * 1000)
    t_ms = min(times[a.warmup:])
    return {"metric": f"CPU mining ms (C++ path, {num_threads()} threads), {a.config} min_sup={ms}",
            "n_txn": n, "min_support": ms, "threads": num_threads(), "ms": round(t_ms, 1),
            "runs_ms": [round(t, 1) for t in times], "n_itemsets": res.n_itemsets,
            "itemsets_per_s": round(res.n_itemsets / (t_ms / 1e3), 1), "torch_threads": torch.get_num_threads(),
            "digest": res.digest()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="T10I4D10M", choices=sorted(bench.CONFIGS))
    ap.add_argument("--mode", default="e2e", choices=["e2e", "cpu"])
    ap.add_argument("--device", default="auto")
    ap.add_argument("--n-txn", type=int, default=0)
    ap.add_argument("--min-support", type=float, default=0.0)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workdir", default=os.environ.get("TMPDIR", "/tmp") + "/fa_bench")
    ap.add_argument("--tokens", choices=["num", "str"], default="num",
                    help="webdocs e2e: numeric ids or letter-string tokens (dictionary path)")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    if a.config.startswith("webdocs") and a.mode == "cpu":
        raise SystemExit("webdocs CPU baseline: not supported (bench.py generates it in-process)")
    line = _e2e(a, cfg) if a.mode == "e2e" else _cpu(a, cfg)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
