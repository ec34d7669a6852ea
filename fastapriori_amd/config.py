"""Job configuration: CLI > environment (FA_*) > defaults.

The environment can set the product settings a batch scheduler typically fixes per
job: FA_MIN_SUPPORT, FA_DEVICE, FA_STRATEGY, FA_PROFILE and FA_METRICS; everything
else is a command-line flag.  Internal tuning knobs are not here: see tuning.py
(one FA_TUNE variable for experiments) and docs/ARCHITECTURE.md ("Configuration").

Positional arguments keep the reference's semantics (Main.scala:24-25,
Utils.scala:21-23,39,48): ``input`` and ``output`` are string PREFIXES —
``input + "D.dat"``, ``output + "freqItemset"`` — so directories need a
trailing slash; ``temp`` is the checkpoint location (ignored by the reference).
"""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass, field


def _env(name: str, default):
    v = os.environ.get(name)
    if v is None:
        return default
    if isinstance(default, bool):
        return v.lower() in ("1", "true", "yes", "on")
    return type(default)(v)


# every FA_* variable the package reads (config / tuning / env / checkpoint / comm / build)
KNOWN_ENV = frozenset({"FA_MIN_SUPPORT", "FA_DEVICE", "FA_STRATEGY", "FA_PROFILE", "FA_METRICS", "FA_TUNE",
                       "FA_NUM_THREADS", "FA_DIST_BACKEND", "FA_FORCE_PG", "FA_FAULT_AT_LEVEL", "FA_FAULT_RANK",
                       "FA_HIP_LIB"})
# variables of earlier versions that are no longer read, with what replaced them (ADVICE r5:
# a job script still setting one would otherwise run with the default, silently)
RETIRED_ENV = {"FA_DEDUP": "--dedup", "FA_MAX_LEVEL": "--max-level", "FA_RESUME": "--resume",
               "FA_WITH_COUNTS": "--with-counts", "FA_WORLD_SIZE": "--world-size",
               "FA_DL_MULTI": "FA_TUNE=dl_multi=0|1", "FA_BUCKET_MB": "FA_TUNE=bucket_mb=<MiB>",
               "FA_FUSED_LAYOUT": "FA_TUNE=fused_layout=0|1"}
_WARNED = False


def unread_env(environ=None) -> list[str]:
    """Warnings for FA_* variables set in the environment that nothing reads."""
    environ = os.environ if environ is None else environ
    out = []
    for k in sorted(environ):
        if not k.startswith("FA_") or k in KNOWN_ENV:
            continue
        hint = RETIRED_ENV.get(k)
        out.append(f"{k} is no longer read" + (f": use {hint}" if hint else " (unknown FA_* variable)"))
    return out


def warn_unread_env() -> None:
    """Print unread_env()'s warnings once per process (stderr)."""
    global _WARNED
    if _WARNED:
        return
    _WARNED = True
    import sys
    for w in unread_env():
        print(f"fastapriori: warning: {w}", file=sys.stderr)


@dataclass
class JobConfig:
    input: str = ""
    output: str = ""
    temp: str = ""
    min_support: float = 0.092                  # Main.scala:23
    device: str = "auto"                        # auto | cuda | cpu
    dedup: str = "auto"
    pair_strategy: str = "auto"
    with_counts: bool = False                   # also write <out>freqItems ("a b[cnt]", Utils.scala:51-63)
    resume: bool = False
    rules_only: bool = False
    checkpoint: bool = True
    overwrite: bool = False
    profile: bool = False
    metrics_path: str | None = None
    max_level: int = 0
    strategy: str = "count"                     # count | candidate distribution
    world_size: int = 0                         # 0: whatever torchrun started; N: launch / require N ranks
    tiebreak: str = "string"                    # rank order of equal-count items (utils.jvm.item_tiebreak_key)
    extra: dict = field(default_factory=dict)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        prog="python -m fastapriori_amd",
        description="MI355X-native FastApriori: frequent itemsets + association-rule recommendations")
    p.add_argument("input", help="input prefix: reads <input>D.dat and <input>U.dat")
    p.add_argument("output", help="output prefix: writes <output>freqItemset/ and <output>recommends/")
    p.add_argument("temp", nargs="?", default="", help="temporary path (per-level checkpoints)")
    p.add_argument("--min-support", type=float, default=_env("FA_MIN_SUPPORT", 0.092))
    p.add_argument("--device", choices=["auto", "cuda", "cpu"], default=_env("FA_DEVICE", "auto"))
    p.add_argument("--dedup", choices=["auto", "on", "off"], default="auto")
    p.add_argument("--pair-strategy", choices=["auto", "horizontal", "gram"],
                   default="auto")
    p.add_argument("--with-counts", action="store_true")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--rules-only", action="store_true")
    p.add_argument("--no-checkpoint", dest="checkpoint", action="store_false", default=True)
    p.add_argument("--overwrite", action="store_true")
    p.add_argument("--profile", action="store_true", default=_env("FA_PROFILE", False))
    p.add_argument("--metrics", dest="metrics_path", default=os.environ.get("FA_METRICS"))
    p.add_argument("--max-level", type=int, default=0)
    p.add_argument("--strategy", choices=["count", "candidate"], default=_env("FA_STRATEGY", "count"),
                   help="count: shard transactions, all-reduce counts; candidate: replicate the DB on every "
                        "rank and split pairs by rows, level candidates by rank")
    p.add_argument("--world-size", type=int, default=0,
                   help="number of ranks (one per GPU). Without a torchrun environment the job "
                        "re-launches itself under torch.distributed.run; under torchrun the process "
                        "group must have exactly this many ranks")
    p.add_argument("--tiebreak", choices=["string", "numeric"], default="string",
                   help="order of frequent items with equal counts (it orders the tokens inside an itemset "
                        "line; the reference's Spark order is not reproducible): string = java.lang.String "
                        "order, numeric = integer tokens by value first")
    return p


def parse_args(argv=None) -> JobConfig:
    a = build_parser().parse_args(argv)
    warn_unread_env()
    return JobConfig(input=a.input, output=a.output, temp=a.temp, min_support=a.min_support, device=a.device,
                     dedup=a.dedup, pair_strategy=a.pair_strategy, with_counts=a.with_counts, resume=a.resume,
                     rules_only=a.rules_only, checkpoint=a.checkpoint, overwrite=a.overwrite,
                     profile=a.profile, metrics_path=a.metrics_path, max_level=a.max_level,
                     strategy=a.strategy, world_size=a.world_size, tiebreak=a.tiebreak)
