"""Local multi-process launcher (tests and CPU rehearsal of the distributed path).

Production runs use ``torchrun --nproc-per-node N`` (one process per GPU,
RCCL).  ``spawn_local`` starts ``world`` processes on this host with the gloo
backend, rendezvous on 127.0.0.1, and returns each rank's return value, so the
sharding / all-reduce / gather logic can be proven without GPUs.
"""
from __future__ import annotations

import os
import pickle
import socket
import tempfile
import time
import traceback


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, fn, args, outdir: str, env: dict):
    os.environ.update(env)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    if env.get("FA_TUNE"):
        # the knobs were read when fn's module imported the package, before this update
        from ..tuning import TUNING
        TUNING.apply(env["FA_TUNE"])
    try:
        res = fn(*args)
        payload = ("ok", res)
    except BaseException as e:  # report, then fail the process
        payload = ("err", f"{type(e).__name__}: {e}\n{traceback.format_exc()}")
    with open(os.path.join(outdir, f"rank{rank}.pkl"), "wb") as f:
        pickle.dump(payload, f)
    if payload[0] == "err":
        raise SystemExit(1)


def spawn_local(fn, world: int, *args, env: dict | None = None, timeout: float = 600):
    """Run ``fn(*args)`` in ``world`` gloo ranks; returns the list of per-rank results."""
    import torch.multiprocessing as mp

    env = dict(env or {})
    env.setdefault("FA_NUM_THREADS", str(max(1, (os.cpu_count() or 2) // world)))
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_worker, args=(world, free_port(), fn, args, d, env), nprocs=world,
                                 join=False, start_method="spawn")
        # fail fast: a rank that dies makes join() raise; a hang (ranks blocked in a
        # collective their peer never reaches) runs into the deadline instead
        deadline = time.monotonic() + timeout
        timed_out = False
        while True:
            try:
                if ctx.join(max(0.1, min(5.0, deadline - time.monotonic()))):
                    break
            except Exception:
                break          # a rank failed: its result file says why
            if time.monotonic() >= deadline:
                timed_out = True
                break
        alive = [r for r, p in enumerate(ctx.processes) if p.is_alive()]
        for p in ctx.processes:
            if p.is_alive():
                p.terminate()
        for p in ctx.processes:
            p.join(10)
            if p.is_alive():
                p.kill()
                p.join(5)
        if timed_out:
            raise TimeoutError(f"spawn_local: ranks {alive} still running after {timeout:.0f} s")
        errors = []
        for r in range(world):
            p = os.path.join(d, f"rank{r}.pkl")
            if os.path.exists(p):
                # our own file, written just above by our own worker
                status, val = pickle.load(open(p, "rb"))
                if status != "ok":
                    errors.append(f"rank {r} failed:\n{val}")
        if errors:
            raise RuntimeError("\n".join(errors))
        out = []
        for r in range(world):
            p = os.path.join(d, f"rank{r}.pkl")
            if not os.path.exists(p):
                raise RuntimeError(f"rank {r} produced no result")
            # our own file, written just above by our own worker
            status, val = pickle.load(open(p, "rb"))
            if status != "ok":
                raise RuntimeError(f"rank {r} failed:\n{val}")
            out.append(val)
        return out
