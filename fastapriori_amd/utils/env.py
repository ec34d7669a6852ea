"""Process environment helpers (thread counts, device selection)."""
from __future__ import annotations

import os


_BOUND_THREADS = 0     # set by parallel.affinity.bind_local_rank: this rank's NUMA-local CPU share


def set_num_threads(n: int) -> None:
    global _BOUND_THREADS
    _BOUND_THREADS = max(0, int(n))


def num_threads() -> int:
    """Host worker threads: FA_NUM_THREADS, else the rank's bound CPU share
    (parallel.affinity), else OMP_NUM_THREADS (16 on the GPU boxes), else the CPU count.

    Capped at 16 without a binding: on the GPU box os.cpu_count() reports the whole
    machine while this process only owns a 16-CPU share.
    """
    v = os.environ.get("FA_NUM_THREADS")
    if not v and _BOUND_THREADS:
        return _BOUND_THREADS
    v = v or os.environ.get("OMP_NUM_THREADS")
    if v:
        try:
            return max(1, int(v))
        except ValueError:
            pass
    return max(1, min(16, os.cpu_count() or 1))
