"""Process environment helpers (thread counts, device selection)."""
from __future__ import annotations

import os


def num_threads() -> int:
    """Host worker threads: OMP_NUM_THREADS if set (16 on the GPU boxes), else the CPU count.

    Capped at 16: on the GPU box os.cpu_count() reports the whole machine while
    this process only owns a 16-CPU share.
    """
    v = os.environ.get("FA_NUM_THREADS") or os.environ.get("OMP_NUM_THREADS")
    if v:
        try:
            return max(1, int(v))
        except ValueError:
            pass
    return max(1, min(16, os.cpu_count() or 1))
