"""Headline benchmark: frequent-itemset mining throughput on T10I4D100M, min_sup 0.1%.

BASELINE.json metric: "mining wall-clock + itemsets/sec, T10I4D100M min_sup=0.1%
at 1/2/4/8 GPU".  One step = one complete mining run over the fixed synthetic
database (F1 histogram + all-reduce, compression, vertical bitmaps, every
level's candidate generation + counting + all-reduce, results replicated on
every rank).  The database (100M Quest transactions, |T|=10, |I|=4, |L|=2000,
N=1000 items) is generated deterministically per rank and kept resident in HBM
before timing.  The total work is fixed as N grows, so scaling is "strong".

After the timed steps the reference's own timing window (Main.scala:28-32:
read + parse D.dat, mine, write freqItemset) is measured on the same database
written to a D.dat file: once with the file's pages dropped from the page cache
(posix_fadvise DONTNEED after fsync) and then warm.  Those numbers go into the
JSON line's "e2e" record (``--e2e off`` skips them).

``vs_baseline`` = this run's itemsets/s over the multi-threaded C++ CPU path of
the same miner on the same config (BASELINE.md:27: the reference publishes no
numbers; benchmarks/cpu_baselines.json, measured on the GPU box's 16 host threads
by scripts/gpu_cpu_baselines.sh).  That CPU path compresses rows, counts pairs per
row and counts every level with a column-tiled prefix-shared AND+popcount (its
"what" field is copied into the JSON line).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config T10I4D100M]

``--gpus N`` > 1 without a torchrun environment re-launches this script under
``torch.distributed.run`` with N ranks (one per GPU, RCCL); under torchrun the
world size must equal N or the run fails.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import shutil
import subprocess
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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="number of ranks (one per GPU)")
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
    ap.add_argument("--e2e", choices=["auto", "on", "off"], default="auto",
                    help="also time the reference window (read+parse+mine+write) on a D.dat file "
                         "(auto: on for file-backed configs)")
    ap.add_argument("--e2e-runs", type=int, default=2, help="warm-cache e2e runs after the cold one")
    ap.add_argument("--workdir", default="", help="where the e2e D.dat is written (default $TMPDIR)")
    ap.add_argument("--no-digest-check", action="store_true",
                    help="report the result digest without failing on a mismatch (timing-only kernel variants)")
    return ap.parse_args(argv)


def _relaunch(args) -> int:
    """--gpus N from a plain `python bench.py`: start N ranks under torch.distributed.run.

    This parent never touches the GPU; the children pick their device from LOCAL_RANK."""
    from fastapriori_amd.parallel.launch import free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


BASELINES = os.path.join(ROOT, "benchmarks", "cpu_baselines.json")


def cpu_baseline(config: str, min_sup: float, n_txn: int):
    """itemsets/s of the C++ CPU path on the same config (benchmarks/cpu_baselines.json,
    written from benchmarks/run_bench.py --mode cpu runs), or None."""
    if not os.path.exists(BASELINES):
        return None
    with open(BASELINES) as f:
        rec = json.load(f).get(config)
    if not rec or rec.get("n_txn") != n_txn or abs(rec.get("min_support", min_sup) - min_sup) > 1e-12:
        return None
    return rec


def _pread_floor(path: str) -> float:
    """ms to pread the whole file into the pinned ring by the same host threads as the
    device reader (no H2D copy, no parse): the storage / page-cache floor of the window."""
    from concurrent.futures import ThreadPoolExecutor
    from fastapriori_amd.utils import io
    from fastapriori_amd.utils.env import num_threads
    n = os.path.getsize(path)
    import torch
    from fastapriori_amd.tuning import TUNING
    NS = max(1, int(TUNING.ring_slots))
    ring = io._ring[:NS] if len(io._ring) >= NS else [torch.empty(io._RING_SLOT, dtype=torch.uint8,
                                                  pin_memory=torch.cuda.is_available())
                                      for _ in range(NS)]
    fd = os.open(path, os.O_RDONLY)
    t0 = time.perf_counter()
    try:
        def rd(c):
            off, m = c * io._RING_SLOT, min(io._RING_SLOT, n - c * io._RING_SLOT)
            mv = memoryview(ring[c % NS].numpy())
            got = 0
            while got < m:
                got += os.preadv(fd, [mv[got:m]], off + got)
        with ThreadPoolExecutor(min(num_threads(), NS)) as ex:
            list(ex.map(rd, range((n + io._RING_SLOT - 1) // io._RING_SLOT)))
    finally:
        os.close(fd)
    return (time.perf_counter() - t0) * 1e3


def _drop_cache(path: str) -> bool:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        return True
    except OSError:
        return False
    finally:
        os.close(fd)


def _e2e_window(args, comm, n_txn, min_sup, cfgv, miner_cfg, sync):
    """The reference's "Total time for get freqItemsets" window (Main.scala:28-32) on a
    real D.dat, through the CLI's own code path: pipeline.mine_window with a temp path
    (the three-argument `input output temp` form, per-level checkpoints on): read +
    parse, mine, write freqItemset, checkpoint.  Cold (page cache dropped) and warm,
    each next to the pread-only floor of the same file measured in the same run."""
    import torch
    from fastapriori_amd.config import JobConfig
    from fastapriori_amd.pipeline import make_checkpointer, mine_window
    from fastapriori_amd.utils import io
    from fastapriori_amd.utils.metrics import Logger
    _, avg_len, avg_pat, n_pat, n_items, _ = cfgv
    base = args.workdir or os.environ.get("TMPDIR") or "/tmp"
    d = os.path.join(base, f"fa_bench_{args.config}_{n_txn}_{args.seed}")
    path = os.path.join(d, "D.dat")
    out = os.path.join(d, f"out_{os.getpid() if comm.is_root else 0}_")
    tmp = os.path.join(d, f"tmp_{os.getpid() if comm.is_root else 0}")
    t_w = time.perf_counter()
    err = ""
    if comm.is_root:
        try:
            os.makedirs(d, exist_ok=True)
            if not os.path.exists(path):
                tmpf = path + ".tmp"
                io.write_quest_file(tmpf, n_txn, avg_len, avg_pat, n_pat, n_items, seed=args.seed)
                os.replace(tmpf, path)
        except OSError as e:           # e.g. no room for the file: skip the window, keep the bench
            err = f"{type(e).__name__}: {e}"
            shutil.rmtree(d, ignore_errors=True)
    if comm.allreduce_int(1 if err else 0, "max"):
        return {"window": "skipped", "error": err or "the D.dat file could not be written"}, None
    write_s = time.perf_counter() - t_w
    quiet = Logger(comm.rank, enabled=False)
    jc = JobConfig(input=d + "/", output=out, temp=tmp, min_support=min_sup, device=str(comm.device.type),
                   dedup=miner_cfg.dedup, pair_strategy=miner_cfg.pair_strategy, overwrite=True)

    def one_run():
        if comm.is_root:
            shutil.rmtree(tmp, ignore_errors=True)
        sync()
        ck = make_checkpointer(jc, comm)
        t0 = time.perf_counter()
        summ: dict = {}
        res = mine_window(jc, comm, quiet, ck, summ)
        sync()
        ms = (time.perf_counter() - t0) * 1e3
        t1 = time.perf_counter()
        if ck is not None:
            ck.wait()                    # (as run_job: the checkpoint completes after the window)
        summ["ckpt_wait_ms"] = (time.perf_counter() - t1) * 1e3
        return comm.allreduce_float_max(ms), res, summ

    # cold: the file's pages dropped from the page cache (every rank's local view)
    dropped = _drop_cache(path) if comm.is_root else False
    comm.barrier()
    cold_ms, res, summ = one_run()
    dropped_floor = _drop_cache(path) if comm.is_root else False
    floor_cold = _pread_floor(path) if comm.is_root else 0.0
    warm, bundles = [], summ.get("device_bundles", 0)
    for _ in range(max(args.e2e_runs, 1)):
        ms, _, summ = one_run()
        warm.append(ms)
    floor_warm = _pread_floor(path) if comm.is_root else 0.0
    warm_ms = min(warm)
    rec = _recommend_window(args, comm, d, jc, res, cfgv, sync)
    if comm.is_root:
        shutil.rmtree(out + "freqItemset", ignore_errors=True)
        shutil.rmtree(out + "recommends", ignore_errors=True)
        shutil.rmtree(tmp, ignore_errors=True)
    if comm.device.type == "cuda":
        torch.cuda.empty_cache()
    return {
        "window": "read+parse D.dat, mine, write freqItemset (Main.scala:28-32), through pipeline.mine_window "
                  "with a temp path (the CLI's `input output temp` form): the checkpoint's level files are "
                  "written by a background thread during the window, and the wait for its completion "
                  "(ckpt_wait_ms_last) is outside it, as in run_job",
        "ckpt_wait_ms_last": round(summ.get("ckpt_wait_ms", 0.0), 1),
        "D_bytes": os.path.getsize(path), "file_write_s": round(write_s, 1),
        "cold_ms": round(cold_ms, 1), "cold_cache_dropped": dropped,
        "pread_floor_cold_ms": round(floor_cold, 1), "pread_floor_cold_dropped": dropped_floor,
        "warm_ms": round(warm_ms, 1), "warm_runs": [round(x, 1) for x in warm],
        "pread_floor_warm_ms": round(floor_warm, 1),
        "read_ms_last": summ.get("read_ms"), "device_bundles": bundles,
        "itemsets_per_s_cold": round(res.n_itemsets / (cold_ms / 1e3), 1),
        "itemsets_per_s_warm": round(res.n_itemsets / (warm_ms / 1e3), 1),
        "n_itemsets": res.n_itemsets,
        "recommend": rec,
    }, path


U_LINES = 1_000_000


def _recommend_window(args, comm, d, jc, res, cfgv, sync) -> dict:
    """The reference's "Total time for get recommends" window (Main.scala:34-37) through
    the CLI's own function (pipeline.recommend_window): read + parse a U.dat of U_LINES
    user baskets (Quest transactions of the same config), build the rules from the mined
    itemsets (generation, cut, sort), recommend, write recommends.  The first run and
    the best of the warm runs."""
    from fastapriori_amd.pipeline import recommend_window
    from fastapriori_amd.utils import io
    from fastapriori_amd.utils.metrics import Logger
    _, avg_len, avg_pat, n_pat, n_items, _ = cfgv
    upath = os.path.join(d, "U.dat")
    err = ""
    if comm.is_root and not os.path.exists(upath):
        try:
            io.write_quest_file(upath + ".tmp", U_LINES, avg_len, avg_pat, n_pat, n_items, seed=args.seed + 1,
                                users=True)
            os.replace(upath + ".tmp", upath)
        except OSError as e:
            err = f"{type(e).__name__}: {e}"
    if comm.allreduce_int(1 if err else 0, "max"):
        return {"window": "skipped", "error": err or "U.dat could not be written"}
    quiet = Logger(comm.rank, enabled=False)
    runs, summ, steps = [], {}, []
    for _ in range(1 + max(args.e2e_runs, 1)):
        sync()
        t0 = time.perf_counter()
        summ = {}
        recommend_window(jc, comm, quiet, res, summ)
        sync()
        runs.append(comm.allreduce_float_max((time.perf_counter() - t0) * 1e3))
        steps.append(summ.get("recommend_steps_ms"))
    return {"window": "read+parse U.dat, rules (generation, cut, sort), recommend, write recommends "
                      "(Main.scala:34-37), through pipeline.recommend_window",
            "U_lines": U_LINES, "U_bytes": os.path.getsize(upath), "first_ms": round(runs[0], 1),
            "warm_ms": round(min(runs[1:]), 1), "runs_ms": [round(x, 1) for x in runs],
            "n_rules": summ.get("n_rules"), "n_users": summ.get("n_users"),
            "n_recommended": summ.get("n_recommended"), "steps_ms_first": steps[0], "steps_ms_last": steps[-1]}


def _cpu_ranges(cpus: list) -> str:
    """[0, 1, 2, 5] -> "0-2,5" (sysfs cpulist form)."""
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def _per_rank(args, comm, miner, shard, own_ms, comm_ms, comm_calls, sync) -> list | None:
    """Per-rank diagnostics of the timed steps, gathered to rank 0: the rank's own
    ms per step, host ms held inside collectives (Comm._timed) and collectives per
    step; then ONE extra, untimed run with hipEvent phase timers (MinerConfig.timing):
    device time of the top-level phases (F1, compression, pairs, each level or
    bundle; gaps inside a phase count as busy) and the rest of that run's wall time
    as host-bound time.  A bad scaling curve then shows which rank and which part
    (kernels, collectives, host steps) is slow."""
    import re
    if args.steps <= 0:
        return None
    from fastapriori_amd.parallel.affinity import PLACEMENT
    from fastapriori_amd.utils.env import num_threads
    rec = {"rank": comm.rank, "ms_per_step": round(own_ms, 3), "comm_ms_per_step": round(comm_ms, 3),
           "collectives_per_step": round(comm_calls, 1),
           # the rank's host placement (parallel.affinity: its GPU's NUMA-local CPU share)
           "numa_node": PLACEMENT.get("node"), "cpus": _cpu_ranges(sorted(os.sched_getaffinity(0))),
           "host_threads": num_threads()}
    if comm.device.type == "cuda":
        timing, miner.cfg.timing = miner.cfg.timing, "events"
        try:
            sync()
            t0 = time.perf_counter()
            miner.run(shard)
            sync()
            run_ms = (time.perf_counter() - t0) * 1e3
        finally:
            miner.cfg.timing = timing
        ph = miner.stats.get("gpu_phase_ms", {})
        top = {k: v for k, v in ph.items() if re.fullmatch(r"f1|compress|pairs|level\d+", k)}
        gpu = sum(top.values())
        rec.update(diag_run_ms=round(run_ms, 3), gpu_phase_ms=round(gpu, 3),
                   host_bound_ms=round(max(run_ms - gpu, 0.0), 3),
                   phases={k: round(v, 3) for k, v in top.items()})
    return comm.all_gather_object(rec)


def main() -> int:
    args = parse_args()
    in_torchrun = "WORLD_SIZE" in os.environ and "RANK" in os.environ
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if args.gpus > 1 and not in_torchrun:
        return _relaunch(args)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks",
              file=sys.stderr)
        return 2

    import torch
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm, init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_shard, generate_zipf_shard
    from fastapriori_amd.utils.metrics import Logger

    dev = args.device if (args.device != "cuda" or torch.cuda.is_available()) else "cpu"
    comm = init_comm(dev)
    if comm.world_size != args.gpus:
        print(f"bench.py: process group has {comm.world_size} ranks, --gpus {args.gpus}", file=sys.stderr)
        return 2
    n_txn, avg_len, avg_pat, n_pat, n_items, ms = CONFIGS[args.config]
    n_txn = args.n_txn or n_txn
    min_sup = args.min_support or ms
    world = comm.world_size

    t_gen = time.perf_counter()
    data_comm = comm if args.strategy == "count" else Comm(device=comm.device)
    webdocs = args.config.startswith("webdocs")
    if webdocs:
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
    # long-lived objects (the shard, the miner, torch/numpy state) out of the cyclic GC's
    # scans: collections between the timed runs then stay cheap
    gc.collect()
    gc.freeze()
    sync()
    c_ms0, c_n0 = comm.comm_ms, comm.comm_calls
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = miner.run(shard)
    sync()
    elapsed = time.perf_counter() - t0
    own_ms = elapsed * 1e3 / max(args.steps, 1)
    comm_ms = (comm.comm_ms - c_ms0) / max(args.steps, 1)
    comm_calls = (comm.comm_calls - c_n0) / max(args.steps, 1)
    ms_step = comm.allreduce_float_max(own_ms)
    n_sets = res.n_itemsets
    value = n_sets / (ms_step / 1e3)
    stats = dict(miner.stats)
    per_rank = _per_rank(args, comm, miner, shard, own_ms, comm_ms, comm_calls, sync)

    e2e = None
    want_e2e = args.e2e == "on" or (args.e2e == "auto" and not webdocs and args.strategy == "count")
    if want_e2e and args.steps > 0:
        del shard
        e2e, _ = _e2e_window(args, comm, n_txn, min_sup, CONFIGS[args.config], cfg, sync)
        if "n_itemsets" in e2e and e2e["n_itemsets"] != n_sets:
            print(f"bench.py: e2e run found {e2e['n_itemsets']} itemsets, in-memory run {n_sets}",
                  file=sys.stderr)
            return 3

    base = cpu_baseline(args.config, min_sup, n_txn)
    # correctness at benchmark scale (outside the timed region): the result's digest
    # (MiningResult.digest: the set of (itemset, count) in token space) against the C++
    # CPU path's on the same data, when benchmarks/cpu_baselines.json holds one
    digest = res.digest() if res is not None else None
    want = base.get("digest") if base else None
    digest_ok = None if (want is None or digest is None) else digest == want
    if comm.is_root:
        line = {
            "metric": f"itemsets/sec (mining wall-clock), {args.config} min_sup={min_sup:g}",
            "value": round(value, 2),
            "unit": "itemsets/s",
            "n_gpus": world if comm.device.type == "cuda" else 0,
            "world_size": world,
            "backend": comm.backend,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / base["itemsets_per_s"], 2) if base else None,
            "baseline": ({"what": base.get("what", "C++ CPU path of the same miner, same config (BASELINE.md:27)"),
                          "itemsets_per_s": base["itemsets_per_s"], "ms": base["ms"],
                          "threads": base.get("threads"), "source": "benchmarks/cpu_baselines.json"}
                         if base else None),
            "digest": digest,
            "digest_ok": digest_ok,
            "dtype": "int32/uint64-bitmap (exact integer counts)",
            "data": (f"synthetic {'Zipf-topic' if webdocs else 'Quest'} {args.config} "
                     f"(n={n_txn}, seed={args.seed}), generated in-process"),
            "config": {"model": args.config, "global_batch": n_txn, "seq_len": avg_len,
                       "parallelism": f"{'dp' if args.strategy == 'count' else 'cp'}{world}",
                       "min_support": min_sup,
                       "n_itemsets": n_sets, "levels": [len(c) for c in res.counts],
                       "pair_strategy": stats.get("pair_strategy"),
                       "min_count": res.min_count, "gen_s": round(t_gen, 2),
                       **({"phase_ms": stats["phase_ms"]} if "phase_ms" in stats else {}),
                       **({"level_info": stats["level_info"]} if "level_info" in stats else {})},
            "e2e": e2e,
            "per_rank": per_rank,
            "rank_spread_ms": (round(max(r["ms_per_step"] for r in per_rank) - min(r["ms_per_step"] for r in per_rank),
                                     3) if per_rank else None),
        }
        print(json.dumps(line), flush=True)
    shutdown_comm(comm)
    if digest_ok is False and not args.no_digest_check:
        print(f"bench.py: result digest {digest} differs from the CPU path's {want}", file=sys.stderr)
        return 4
    return 0


if __name__ == "__main__":
    sys.exit(main())
