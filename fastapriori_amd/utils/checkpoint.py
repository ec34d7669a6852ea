"""Per-level checkpoint / resume.

The reference documents a temporary-path argument but never reads it
(Main.scala:24-25), and ships an unused manual reload helper (Utils.getAll,
Utils.scala:65-81).  Here the temp path gets a real job: after every mined
level rank 0 atomically writes ``<temp>/fastapriori_ckpt/level_<k>.npz`` plus a
``meta.json`` (vocabulary in rank order, F1 counts, min_count, an input
fingerprint).  ``--resume`` reloads the completed levels and mines on from the
next one; ``--rules-only`` skips mining entirely (the getAll use case).

Fault injection for testing recovery: ``FA_FAULT_AT_LEVEL=k`` makes rank
``FA_FAULT_RANK`` (default 0) exit with status 17 right after level k is
checkpointed.
"""
from __future__ import annotations

import json
import os

import numpy as np

from ..models.data import MiningResult


class InjectedFault(SystemExit):
    pass


class Checkpointer:
    def __init__(self, temp: str, rank: int = 0, fingerprint: dict | None = None):
        self.dir = os.path.join(temp, "fastapriori_ckpt")
        self.rank = rank
        self.fingerprint = fingerprint or {}
        self._thread = None           # background writer of save_levels(background=True)
        self._error = None
        if rank == 0:
            os.makedirs(self.dir, exist_ok=True)

    def _atomic(self, path: str, write) -> None:
        tmp = path + ".tmp"
        write(tmp)
        os.replace(tmp, path)

    @staticmethod
    def fault_level(rank: int) -> int:
        """FA_FAULT_AT_LEVEL for this rank (0: no injected fault)."""
        fault = os.environ.get("FA_FAULT_AT_LEVEL")
        if fault and rank == int(os.environ.get("FA_FAULT_RANK", "0")):
            return int(fault)
        return 0

    def _write_level(self, result: MiningResult, k: int, meta: bool = True, rows=None, counts=None) -> None:
        """level_k.npz, then (meta) meta.json saying levels 1..k are done: the level file
        lands before the meta that counts it, so a crash leaves a consistent checkpoint.
        rows / counts: the level's arrays when result does not hold them yet (the device
        level loop's staged copies, before its results readback)."""
        if rows is None and k > len(result.levels):
            return
        if self.rank == 0:
            if rows is None:
                rows, counts = result.levels[k - 1], result.counts[k - 1]

            def w(tmp):
                with open(tmp, "wb") as f:
                    np.savez(f, rows=rows, counts=counts)
            self._atomic(os.path.join(self.dir, f"level_{k}.npz"), w)
            if meta:
                self._write_meta(result, k)

    def submit(self, fn) -> None:
        """Run fn on the checkpoint thread after everything submitted before it (the
        device level loop hands each bundle's staged results over this way); an error
        is raised by the next wait()."""
        import threading
        prev = self._thread

        def work():
            try:
                if prev is not None:
                    prev.join()
                if self._error is None:
                    fn()
            except BaseException as e:       # surfaced by wait()
                self._error = e

        self._thread = threading.Thread(target=work, name="fa-ckpt", daemon=True)
        self._thread.start()

    def _write_meta(self, result: MiningResult, k: int, complete: bool = False) -> None:
        if self.rank != 0:
            # rank 0 alone publishes the checkpoint: another rank's meta could count levels
            # whose files rank 0 has not written yet (or land in a directory that does not
            # exist on its node)
            return
        meta = {"items": result.items, "min_count": result.min_count, "n_lines": result.n_lines,
                "levels_done": k, "fingerprint": self.fingerprint}
        if complete:
            meta["complete"] = True
        self._atomic(os.path.join(self.dir, "meta.json"),
                     lambda tmp: open(tmp, "w", encoding="utf-8").write(json.dumps(meta)))

    def save_level(self, result: MiningResult, k: int) -> None:
        self.wait()
        self._write_level(result, k)
        if self.fault_level(self.rank) == k:
            raise InjectedFault(17)

    def save_levels(self, result: MiningResult, ks, background: bool = False) -> None:
        """Levels ks (ascending), then one meta.json counting them (a crash part-way
        leaves the previous meta: a consistent checkpoint of the levels before the
        batch).  background: written by
        a thread while the caller goes on (the device level loop hands its levels over
        in one go after its single results readback); wait() joins it.  An injected
        fault at one of the levels is taken synchronously: the levels up to it are
        written, then the process exits as save_level's would."""
        self.wait()
        ks = list(ks)
        fault = self.fault_level(self.rank)
        if fault and fault in ks:
            for k in ks[:ks.index(fault) + 1]:
                self._write_level(result, k)
            raise InjectedFault(17)
        if self.rank != 0 or not ks:
            return
        def batch():
            for k in ks:
                self._write_level(result, k, meta=False)
            self._write_meta(result, ks[-1])

        if not background:
            batch()
            return
        import threading

        def work():
            try:
                batch()
            except BaseException as e:       # surfaced by wait()
                self._error = e

        self._thread = threading.Thread(target=work, name="fa-ckpt", daemon=True)
        self._thread.start()

    def wait(self) -> None:
        t, self._thread = self._thread, None
        if t is not None:
            t.join()
        if self._error is not None:
            e, self._error = self._error, None
            raise e

    def mark_complete(self, result: MiningResult, background: bool = False) -> None:
        """Every level written (the missing ones now), then the meta marked complete.
        background: after the level writes already queued, on the checkpoint thread, so the
        mining window does not wait for checkpoint files; wait() (the job's end) joins it."""
        if self.rank != 0:
            return
        if not background:
            self.wait()
            self._complete(result)
            return
        import threading
        prev = self._thread

        def work():
            try:
                if prev is not None:
                    prev.join()
                if self._error is None:
                    self._complete(result)
            except BaseException as e:       # surfaced by wait()
                self._error = e

        self._thread = threading.Thread(target=work, name="fa-ckpt-complete", daemon=True)
        self._thread.start()

    def _complete(self, result: MiningResult) -> None:
        for k in range(1, len(result.levels) + 1):
            f = os.path.join(self.dir, f"level_{k}.npz")
            if not os.path.exists(f):
                self._write_level(result, k, meta=False)
        self._write_meta(result, len(result.levels), complete=True)

    def load(self, require_complete: bool = False) -> MiningResult | None:
        path = os.path.join(self.dir, "meta.json")
        if not os.path.exists(path):
            return None
        meta = json.load(open(path, encoding="utf-8"))
        if self.fingerprint and meta.get("fingerprint") and meta["fingerprint"] != self.fingerprint:
            raise ValueError("checkpoint was written for different input data")
        if require_complete and not meta.get("complete"):
            return None
        levels, counts = [], []
        for k in range(1, int(meta["levels_done"]) + 1):
            z = np.load(os.path.join(self.dir, f"level_{k}.npz"), allow_pickle=False)
            levels.append(np.ascontiguousarray(z["rows"], dtype=np.int32).reshape(-1, k))
            counts.append(np.ascontiguousarray(z["counts"], dtype=np.int64))
        res = MiningResult(meta["items"], levels, counts, int(meta["min_count"]), int(meta["n_lines"]))
        res.stats["complete"] = bool(meta.get("complete"))
        return res


def input_fingerprint(path: str, min_support: float) -> dict:
    st = os.stat(path)
    return {"path": os.path.abspath(path), "size": st.st_size, "mtime": int(st.st_mtime),
            "min_support": min_support}
