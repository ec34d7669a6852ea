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
    """Phase timer.

    * host wall-clock per phase (always); with ``sync`` the device is synchronised at
      the phase edges (MinerConfig.timing = "sync": exact but perturbing);
    * with ``events`` (cuda only) a pair of timing hipEvents is recorded around every
      phase on the current stream -- no synchronisation -- and read back by
      ``finish()`` once the run's final readback has drained the stream
      (``gpu_ms``: device time between the phase's first and last queued work).
    ``trace()`` turns the phases into Chrome trace events (chrome://tracing, Perfetto).
    """

    def __init__(self, device=None, sync: bool = False, events: bool = False):
        self.device = device
        self.sync = sync
        is_cuda = getattr(device, "type", "") == "cuda"
        self.events = bool(events and is_cuda)
        self.t = {}
        self.gpu: dict = {}
        self.spans: list = []            # (name, host t0 s, host t1 s, ev0, ev1)

    def _sync(self):
        if self.sync and self.device is not None and getattr(self.device, "type", "") == "cuda":
            import torch
            torch.cuda.synchronize(self.device)

    @contextmanager
    def phase(self, name: str):
        self._sync()
        e0 = e1 = None
        if self.events:
            import torch
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self._sync()
            t1 = time.perf_counter()
            if self.events:
                import torch
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
            self.t[name] = self.t.get(name, 0.0) + (t1 - t0) * 1e3
            self.spans.append((name, t0, t1, e0, e1))

    def finish(self) -> dict:
        """Device time per phase name (ms), from the recorded events."""
        if self.events and self.spans:
            last = self.spans[-1][4]
            if last is not None:
                last.synchronize()
            self.gpu = {}
            for name, _, _, e0, e1 in self.spans:
                if e0 is not None and e1 is not None:
                    self.gpu[name] = self.gpu.get(name, 0.0) + e0.elapsed_time(e1)
        return self.gpu

    def span_gpu_ms(self, i: int):
        name, _, _, e0, e1 = self.spans[i]
        return e0.elapsed_time(e1) if (e0 is not None and e1 is not None) else None

    def trace(self, pid: int = 0, t_origin: float | None = None) -> list[dict]:
        """Chrome trace events: one "X" event per phase on the host track (tid 0), and
        its device span on tid 1 when events were recorded (placed at the host start
        of the phase; the device duration is the recorded one)."""
        if not self.spans:
            return []
        t_origin = self.spans[0][1] if t_origin is None else t_origin
        out = []
        for i, (name, t0, t1, e0, e1) in enumerate(self.spans):
            ts = (t0 - t_origin) * 1e6
            out.append({"name": name, "ph": "X", "pid": pid, "tid": 0, "ts": ts, "dur": (t1 - t0) * 1e6,
                        "cat": "host"})
            g = self.span_gpu_ms(i) if self.events else None
            if g is not None:
                out.append({"name": name, "ph": "X", "pid": pid, "tid": 1, "ts": ts, "dur": g * 1e3,
                            "cat": "gpu"})
        return out

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
