"""The end-to-end job: Main.main of the reference (Main.scala:16-38).

    read D.dat/U.dat shards -> mine -> write freqItemset -> rules -> recommend
    -> write recommends

One process per GPU (torchrun); rank 0 writes the outputs.  Phase timings are
printed as the reference does ("==== Total time for get freqItemsets ..."); the
mining window includes reading and parsing D.dat, like the reference's lazy
RDD read makes it do.
"""
from __future__ import annotations

import json
import os
import time

from .config import JobConfig
from .models.apriori import FastApriori, MinerConfig
from .models.rules import AssociationRules
from .parallel.comm import Comm, init_comm, shutdown_comm
from .utils import io
from .utils.checkpoint import Checkpointer, input_fingerprint
from .utils.metrics import Logger


def _load_checkpoint(ckpt: Checkpointer, comm, require_complete: bool = False):
    """Rank 0 reads the checkpoint and sends it to every rank, so all ranks resume
    from the same level (a per-rank read could race rank 0's rewrite of meta.json,
    or miss a temp dir that is not shared, and then the ranks' collectives diverge)."""
    res, err = None, None
    if comm.is_root:
        try:
            res = ckpt.load(require_complete=require_complete)
        except (OSError, ValueError, KeyError) as e:
            err = f"{type(e).__name__}: {e}"
    res, err = comm.broadcast_object((res, err))
    if err:
        raise ValueError(f"checkpoint load failed on rank 0: {err}")
    return res


def _load_saved(cfg: JobConfig, comm):
    """Rank 0 rebuilds the mined result from the saved ``freqItems`` / ``ItemsToRank``
    files (io.load_saved_results, the reference's Utils.getAll) and sends it to every
    rank; None when the files are missing."""
    freq, rank = cfg.output + "freqItems", cfg.output + "ItemsToRank"
    res, err = None, None
    if comm.is_root and os.path.exists(rank) and os.path.exists(freq):
        try:
            res = io.load_saved_results(freq, rank)
        except (OSError, ValueError, KeyError) as e:
            err = f"{type(e).__name__}: {e}"
    res, err = comm.broadcast_object((res, err))
    if err:
        raise ValueError(f"loading {freq} failed on rank 0: {err}")
    return res


def mine_window(cfg: JobConfig, comm, log: Logger, ckpt: Checkpointer | None, summary: dict):
    """The reference's timed mining window (Main.scala:28-32): read + parse D.dat,
    mine, write freqItemset (and, with a temp path, the per-level checkpoint).
    bench.py times this same function for its e2e record."""
    d_path, out_freq = cfg.input + "D.dat", cfg.output + "freqItemset"
    resume = _load_checkpoint(ckpt, comm) if (ckpt is not None and cfg.resume) else None
    # candidate distribution: every rank holds the whole DB
    t_read = time.time()
    shard = io.read_shard(d_path, comm if cfg.strategy == "count" else Comm(device=comm.device))
    summary["read_ms"] = round((time.time() - t_read) * 1000, 1)
    # --profile: hipEvent phase times per level and a Chrome trace of the phases
    mcfg = MinerConfig(min_support=cfg.min_support, dedup=cfg.dedup, pair_strategy=cfg.pair_strategy,
                       max_level=cfg.max_level, parallelism=cfg.strategy, tiebreak=cfg.tiebreak,
                       timing="events" if cfg.profile else "off", trace=cfg.profile)
    miner = FastApriori(cfg.min_support, comm, mcfg, log, ckpt)
    result = miner.run(shard, resume=resume)
    summary["miner"] = dict(miner.stats)
    summary["device_bundles"] = int(miner.stats.get("device_bundles", 0))
    trace = summary["miner"].pop("trace", None)
    if cfg.profile and trace is not None and comm.is_root:
        # Chrome trace of the mining phases (host spans + hipEvent device spans)
        tpath = os.path.join(cfg.temp or ".", "fastapriori_trace.json")
        with open(tpath, "w") as f:
            json.dump({"traceEvents": trace, "displayTimeUnit": "ms"}, f)
        summary["trace_path"] = tpath
    del shard
    t_write = time.time()
    if comm.is_root:
        io.write_freq_itemsets(result, out_freq, overwrite=cfg.overwrite)
        if cfg.with_counts:
            io.write_freq_itemsets(result, cfg.output + "freqItems", with_counts=True, overwrite=cfg.overwrite)
            io.write_items_to_rank(result, cfg.output + "ItemsToRank")
            io.write_freq_items(result, cfg.output + "FreqItems")
    if ckpt is not None:
        # the completion follows the level files the device loop queued on the checkpoint
        # thread; the job joins it at its end (run_job), not inside this window
        ckpt.mark_complete(result, background=True)
    comm.barrier()
    summary["write_ms"] = round((time.time() - t_write) * 1000, 1)
    return result


def recommend_window(cfg: JobConfig, comm, log: Logger, result, summary: dict) -> list:
    """The reference's second timed window (Main.scala:34-37): read + parse U.dat,
    rules (generation, cut, sort), one recommendation per user line, write
    recommends.  bench.py times this same function for its e2e record."""
    t0 = time.perf_counter()
    users = io.read_shard(cfg.input + "U.dat", comm)
    t1 = time.perf_counter()
    ar = AssociationRules(result, comm, log)
    ar.rules()
    t2 = time.perf_counter()
    recs = ar.run(users)
    t3 = time.perf_counter()
    if comm.is_root:
        io.write_lines(recs, cfg.output + "recommends", overwrite=cfg.overwrite)
    comm.barrier()
    t4 = time.perf_counter()
    # host wall time of each step (a step's device work ends inside the next host readback)
    summary["recommend_steps_ms"] = {k: round(v * 1e3, 1) for k, v in
                                     (("read_U", t1 - t0), ("rules", t2 - t1), ("recommend", t3 - t2),
                                      ("write", t4 - t3))}
    summary["n_rules"] = ar.rules().n_rules
    if recs is not None:                   # rank 0 holds every user's recommendation
        summary.update(n_users=len(recs), n_recommended=sum(1 for r in recs if r != "0"))
    return recs


def make_checkpointer(cfg: JobConfig, comm) -> Checkpointer | None:
    if cfg.temp and (cfg.checkpoint or cfg.rules_only):
        # rules-only needs no D.dat: it reloads the mined itemsets (Utils.getAll's use case)
        fp = None if cfg.rules_only else input_fingerprint(cfg.input + "D.dat", cfg.min_support)
        return Checkpointer(cfg.temp, comm.rank, fp)
    return None


def run_job(cfg: JobConfig, comm=None) -> dict:
    own_comm = comm is None
    if comm is None:
        dev = None if cfg.device == "auto" else cfg.device
        comm = init_comm(dev)
    if cfg.world_size and comm.world_size != cfg.world_size:
        if own_comm:
            shutdown_comm(comm)
        raise RuntimeError(f"--world-size {cfg.world_size} but the process group has {comm.world_size} ranks")
    log = Logger(comm.rank, metrics_path=cfg.metrics_path)
    summary: dict = {}
    ckpt = None
    try:
        ckpt = make_checkpointer(cfg, comm)
        comm.barrier()

        t1 = time.time()
        if cfg.rules_only:
            # the complete checkpoint under temp, else the saved result files of a
            # --with-counts run (freqItems + ItemsToRank: Utils.getAll, Utils.scala:65-81)
            result = _load_checkpoint(ckpt, comm, require_complete=True) if ckpt is not None else None
            if result is None:
                result = _load_saved(cfg, comm)
            if result is None:
                where = f"under {ckpt.dir} " if ckpt is not None else ""
                raise FileNotFoundError(f"--rules-only: no complete checkpoint {where}and no "
                                        f"{cfg.output}freqItems + {cfg.output}ItemsToRank (written by --with-counts)")
            comm.barrier()
        else:
            result = mine_window(cfg, comm, log, ckpt, summary)
        t_mine = int((time.time() - t1) * 1000)
        log.line(f"Total time for get freqItemsets {t_mine}")

        t2 = time.time()
        recommend_window(cfg, comm, log, result, summary)
        t_rec = int((time.time() - t2) * 1000)
        log.line(f"Total time for get recommends {t_rec}")
        summary.update(mine_ms=t_mine, recommend_ms=t_rec, n_itemsets=result.n_itemsets,
                       world_size=comm.world_size)
        log.metric(phase="job", **{k: v for k, v in summary.items() if not isinstance(v, dict)})
        return summary
    except BaseException as e:
        # the job's own failure wins: a background checkpoint error is only attached to it
        if ckpt is not None:
            try:
                ckpt.wait()
            except BaseException as ck_err:   # noqa: BLE001 (logged; the original error propagates)
                import sys
                print(f"fastapriori: checkpoint thread also failed: {type(ck_err).__name__}: {ck_err}",
                      file=sys.stderr)
                log.metric(phase="checkpoint_error", error=f"{type(ck_err).__name__}: {ck_err}")
            ckpt = None
        raise e
    finally:
        if ckpt is not None:
            ckpt.wait()                  # the checkpoint is complete before the job returns
        if own_comm:
            shutdown_comm(comm)


def _relaunch(cfg: JobConfig, argv) -> int:
    """``--world-size N`` from a plain ``python -m fastapriori_amd``: start N ranks (one per
    GPU) under torch.distributed.run.  This parent process never touches the GPU."""
    import subprocess
    import sys

    from .parallel.launch import free_port
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={cfg.world_size}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", "-m", "fastapriori_amd", *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main(argv=None) -> int:
    from .config import parse_args
    cfg = parse_args(argv)
    if cfg.world_size > 1 and "WORLD_SIZE" not in os.environ:
        return _relaunch(cfg, argv)
    if cfg.profile and not cfg.metrics_path:
        # --profile: JSON-lines metrics (per-level device times, bytes reduced, HBM bytes
        # estimates) and a Chrome trace of the phases (mine_window), both under the temp path
        cfg.metrics_path = os.path.join(cfg.temp or ".", "fastapriori_metrics.jsonl")
    run_job(cfg)
    return 0
