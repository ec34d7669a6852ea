"""Transaction shards, vocabularies and mining results."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch


class Vocabulary:
    """Token id space of one shard.

    numeric: id = int(token) + 1 for canonical decimal tokens, id 0 = the empty
             token "" (blank line).  Identical on every rank by construction.
    dict:    shard-local ids with their 64-bit hashes; ranks agree on identity
             through the hashes (FastApriori._frequent_items).  The strings stay
             one UTF-8 byte blob + offsets (a 5M-entry vocabulary is never turned
             into Python objects); ``decode(ids)`` materialises only the ones asked for.
    """

    def __init__(self, numeric: bool, size: int, strings: list[str] | None = None,
                 hashes: np.ndarray | None = None, blob: np.ndarray | None = None,
                 offsets: np.ndarray | None = None, file_src: tuple | None = None):
        self.numeric = bool(numeric)
        self.size = int(size)
        self.hashes = hashes
        self.blob, self.offsets = blob, offsets
        # device-parsed shards: (path, byte offset of the parsed range, first-occurrence
        # offsets int64 [V], lengths int32 [V]) -- strings are read back from the file
        self.file_src = file_src
        self._strings = strings
        if strings is not None and blob is None and not numeric:
            enc = [t.encode("utf-8") for t in strings]
            self.offsets = np.zeros(len(enc) + 1, dtype=np.int64)
            if enc:
                self.offsets[1:] = np.cumsum([len(e) for e in enc])
            self.blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)

    @property
    def strings(self) -> list[str] | None:
        """Every string of the vocabulary (decoded on first use; avoid for wide ones)."""
        if self._strings is None and (self.blob is not None or self.file_src is not None):
            self._strings = self.decode(np.arange(self.size))
        return self._strings

    def decode(self, ids) -> list[str]:
        ids = np.asarray(ids, dtype=np.int64).ravel()
        if self._strings is not None:
            return [self._strings[i] for i in ids.tolist()]
        if self.file_src is not None:
            import os
            path, base, pos, lens = self.file_src
            fd = os.open(path, os.O_RDONLY)
            try:
                return [os.pread(fd, int(lens[i]), base + int(pos[i])).decode("utf-8", "replace")
                        for i in ids.tolist()]
            finally:
                os.close(fd)
        raw = self.blob.tobytes() if ids.size > 64 else None
        out = []
        for i in ids.tolist():
            a, b = int(self.offsets[i]), int(self.offsets[i + 1])
            out.append((raw[a:b] if raw is not None else self.blob[a:b].tobytes()).decode("utf-8", "replace"))
        return out

    def token(self, i: int) -> str:
        if self.numeric:
            return "" if i == 0 else str(i - 1)
        return self.decode([i])[0]

    @staticmethod
    def numeric_id(token: str) -> int:
        """Numeric-mode id of a token, or -1 when it is not canonical decimal."""
        if token == "":
            return 0
        if not token.isascii() or not token.isdigit() or (len(token) > 1 and token[0] == "0"):
            return -1
        v = int(token)
        return v + 1 if v <= 2147483646 else -1


def hash_tokens(tokens: list[str]) -> np.ndarray:
    """64-bit hashes of token strings, identical to the parser's dictionary hashes."""
    from ..ops import _native
    from ..utils.env import num_threads
    enc = [t.encode("utf-8") for t in tokens]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        off[1:] = np.cumsum([len(e) for e in enc])
    blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
    out = np.zeros(max(len(enc), 1), dtype=np.uint64)
    _native.host().fa_hash_tokens(blob.ctypes.data, off.ctypes.data, len(enc), out.ctypes.data, num_threads())
    return out[:len(enc)]


@dataclass
class TransactionShard:
    """This rank's slice of a transaction file, CSR on one device.

    ``items`` holds DISTINCT ids per line; ``extras`` lists one id per repeated
    occurrence inside a line (the reference counts occurrences for F1 only).
    """
    offsets: torch.Tensor          # int64 [n+1]
    items: torch.Tensor            # int32 [nnz]
    extras: np.ndarray             # int32
    vocab: Vocabulary
    line_base: int = 0             # global index of this shard's first line
    # numeric mode: occurrences per id (items + extras), int64 [vocab.size], counted by
    # the device parser (F1 then needs no pass over the items); None: not counted
    hist: torch.Tensor | None = None

    @property
    def n_lines(self) -> int:
        return self.offsets.numel() - 1

    def to(self, device) -> "TransactionShard":
        return TransactionShard(self.offsets.to(device), self.items.to(device), self.extras, self.vocab,
                                self.line_base, None if self.hist is None else self.hist.to(device))


@dataclass
class MiningResult:
    """All frequent itemsets, in rank space, identical on every rank."""
    items: list[str]                       # rank -> token
    levels: list[np.ndarray]               # levels[k-1]: int32 [F_k, k], rows ascending, lexicographic
    counts: list[np.ndarray]               # int64 [F_k]
    min_count: int
    n_lines: int
    stats: dict = field(default_factory=dict)
    # dictionary mode: the parser's 64-bit hash of every frequent item (rank order), so
    # U.dat tokens are matched on the raw bytes' identity, not on re-encoded strings
    # (a token with invalid UTF-8 decodes with U+FFFD and would hash differently)
    item_hashes: np.ndarray | None = None

    @property
    def n_itemsets(self) -> int:
        return int(sum(len(c) for c in self.counts))

    def digest(self) -> str:
        """SHA-256 (hex) of the result as a set of (itemset, count) in token space:
        independent of the rank order of equal-count items (--tiebreak), of the level
        row order and of the device that mined it, so a GPU run at benchmark scale can be
        checked against the C++ CPU path's digest (benchmarks/cpu_baselines.json).
        Items are numbered by their tokens' sorted order; every itemset becomes its
        ascending item numbers, rows are sorted, and each level hashes as
        (k, F_k, rows int32 LE, counts int64 LE) after the sorted token list."""
        import hashlib
        toks = [str(t) for t in self.items]
        order = sorted(range(len(toks)), key=lambda r: toks[r])
        canon = np.empty(max(len(toks), 1), dtype=np.int32)
        canon[np.asarray(order, dtype=np.int64)] = np.arange(len(toks), dtype=np.int32)
        h = hashlib.sha256()
        h.update("\n".join(toks[r] for r in order).encode("utf-8", "surrogatepass") + b"\0")
        for k, (rows, cnt) in enumerate(zip(self.levels, self.counts), 1):
            rows = np.asarray(rows, dtype=np.int64).reshape(-1, k)
            cnt = np.asarray(cnt, dtype=np.int64).ravel()
            c = np.sort(canon[rows], axis=1) if rows.size else np.zeros((0, k), np.int32)
            idx = np.lexsort(c.T[::-1]) if len(c) else np.zeros(0, np.int64)
            h.update(np.array([k, len(c)], dtype="<i8").tobytes())
            h.update(np.ascontiguousarray(c[idx], dtype="<i4").tobytes())
            h.update(np.ascontiguousarray(cnt[idx], dtype="<i8").tobytes())
        return h.hexdigest()

    def as_dict(self) -> dict[frozenset, int]:
        out = {}
        for rows, cnt in zip(self.levels, self.counts):
            for r, c in zip(rows.tolist(), cnt.tolist()):
                out[frozenset(r)] = int(c)
        return out
