"""Breakdown of the reference's timing window (Main.scala:28-32: read + parse D.dat,
mine, write freqItemset) on one GPU, each step synchronised:

  bytes    pread into the pinned ring + H2D copies (io._file_to_device)
  parse    the device parser over the bytes already in HBM
  read     io.read_shard as the job calls it (bytes + parse, overlapped when streamed)
  mine     FastApriori.run on the parsed shard
  write    rank 0's freqItemset writer
  job      the CLI pipeline's own window (run_job's "Total time for get freqItemsets")

    python benchmarks/e2e_probe.py [--n-txn N] [--config T10I4D100M] [--reps R]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-txn", type=int, default=100_000_000)
    ap.add_argument("--min-support", type=float, default=0.001)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--workdir", default=os.environ.get("TMPDIR") or "/tmp")
    ap.add_argument("--job", action="store_true", help="also time the CLI job (run_job) with a temp path")
    args = ap.parse_args()

    import torch
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils import io
    from fastapriori_amd.utils.metrics import Logger

    d = os.path.join(args.workdir, f"fa_e2e_probe_{args.n_txn}")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "D.dat")
    if not os.path.exists(path):
        io.write_quest_file(path + ".tmp", args.n_txn, 10.0, 4.0, 2000, 1000, seed=1)
        os.replace(path + ".tmp", path)
    if args.job and not os.path.exists(os.path.join(d, "U.dat")):
        io.write_quest_file(os.path.join(d, "U.dat"), 100_000, 10.0, 4.0, 2000, 1000, seed=1, users=True)
    dev = torch.device("cuda", 0)
    comm = Comm(device=dev)
    size = os.path.getsize(path)
    quiet = Logger(0, enabled=False)
    cfg = MinerConfig(min_support=args.min_support)
    out = {"D_bytes": size, "rows": []}

    def t(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return r, (time.perf_counter() - t0) * 1e3

    for rep in range(args.reps):
        row = {}
        fd = os.open(path, os.O_RDONLY)
        try:
            buf, row["bytes_ms"] = t(lambda: io._file_to_device(fd, 0, size, dev))
        finally:
            os.close(fd)
        from fastapriori_amd.ops import primitives as prim
        got, row["parse_ms"] = t(lambda: prim.parse_numeric_device(buf, size, True))
        del buf, got
        shard, row["read_ms"] = t(lambda: io.read_shard(path, comm, dev))
        res, row["mine_ms"] = t(lambda: FastApriori(args.min_support, comm, cfg, quiet).run(shard))
        o = os.path.join(d, "out", "freqItemset")
        _, row["write_ms"] = t(lambda: io.write_freq_itemsets(res, o, overwrite=True))
        row["window_ms"] = row["read_ms"] + row["mine_ms"] + row["write_ms"]
        row["n_itemsets"] = res.n_itemsets
        del shard, res
        if args.job:
            from fastapriori_amd.config import JobConfig
            from fastapriori_amd.pipeline import run_job
            tmp = os.path.join(d, "tmp")
            shutil.rmtree(tmp, ignore_errors=True)
            os.makedirs(tmp)
            jc = JobConfig(input=d + "/", output=os.path.join(d, "job_"), temp=tmp, min_support=args.min_support,
                           device="cuda", overwrite=True)
            s, row["job_ms"] = t(lambda: run_job(jc, comm))
            row["job_mine_window_ms"] = s.get("mine_ms")
            row["job_read_ms"] = s.get("read_ms")
            row["job_device_bundles"] = s.get("miner", {}).get("device_bundles")
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
