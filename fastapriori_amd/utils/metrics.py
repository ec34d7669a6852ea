"""Observability: the reference's "==== " log lines plus a JSON-lines metrics stream.

The reference prints ``println("==== ...")`` lines with counts and millisecond
timings per level and per phase (FastApriori.scala:103-127,
AssociationRules.scala:75,153-181, Main.scala:32,37).  We print the same
human lines (rank 0 only) so runs can be compared side by side, and optionally
append machine-readable records (``FA_METRICS=<path>`` or ``metrics_path``).
"""
from __future__ import annotations

import json
import os
import sys
import time
from contextlib import contextmanager


class Logger:
    def __init__(self, rank: int = 0, enabled: bool = True, metrics_path: str | None = None,
                 stream=None):
        self.rank = rank
        self.enabled = enabled and rank == 0
        self.metrics_path = metrics_path or os.environ.get("FA_METRICS")
        self.stream = stream or sys.stdout
        self.records: list[dict] = []

    def line(self, msg: str) -> None:
        if self.enabled:
            print("==== " + msg, file=self.stream, flush=True)

    def metric(self, **rec) -> None:
        rec.setdefault("rank", self.rank)
        rec.setdefault("ts", time.time())
        self.records.append(rec)
        if self.metrics_path and self.rank == 0:
            with open(self.metrics_path, "a") as f:
                f.write(json.dumps(rec) + "\n")


class Timer:
    """Wall-clock phase timer; synchronises the device at the edges when asked."""

    def __init__(self, device=None, sync: bool = False):
        self.device = device
        self.sync = sync
        self.t = {}

    def _sync(self):
        if self.sync and self.device is not None and getattr(self.device, "type", "") == "cuda":
            import torch
            torch.cuda.synchronize(self.device)

    @contextmanager
    def phase(self, name: str):
        self._sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self._sync()
            self.t[name] = self.t.get(name, 0.0) + (time.perf_counter() - t0) * 1e3

    def ms(self, name: str) -> float:
        return self.t.get(name, 0.0)


@contextmanager
def roctx_range(name: str):
    """roctx range visible in rocprofv3 --marker-trace (no-op without a GPU)."""
    pushed = False
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:
        pushed = False
    try:
        yield
    finally:
        if pushed:
            import torch
            torch.cuda.nvtx.range_pop()
