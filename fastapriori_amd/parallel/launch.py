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
import traceback


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, fn, args, outdir: str, env: dict):
    os.environ.update(env)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
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
        ok = True
        try:
            ok = ctx.join(timeout)
            while not ok:
                ok = ctx.join(timeout)
        except Exception:
            ok = False
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
