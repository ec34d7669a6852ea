"""Transaction shards, vocabularies and mining results."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch


@dataclass
class Vocabulary:
    """Token id space of one shard.

    numeric: id = int(token) + 1 for canonical decimal tokens, id 0 = the empty
             token "" (blank line).  Identical on every rank by construction.
    dict:    shard-local ids with their strings and 64-bit hashes; ranks agree
             on identity through the hashes (parallel/vocab_exchange in the miner).
    """
    numeric: bool
    size: int
    strings: list[str] | None = None
    hashes: np.ndarray | None = None

    def token(self, i: int) -> str:
        if self.numeric:
            return "" if i == 0 else str(i - 1)
        return self.strings[i]

    @staticmethod
    def numeric_id(token: str) -> int:
        """Numeric-mode id of a token, or -1 when it is not canonical decimal."""
        if token == "":
            return 0
        if not token.isascii() or not token.isdigit() or (len(token) > 1 and token[0] == "0"):
            return -1
        v = int(token)
        return v + 1 if v <= 2147483646 else -1


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

    @property
    def n_lines(self) -> int:
        return self.offsets.numel() - 1

    def to(self, device) -> "TransactionShard":
        return TransactionShard(self.offsets.to(device), self.items.to(device), self.extras, self.vocab,
                                self.line_base)


@dataclass
class MiningResult:
    """All frequent itemsets, in rank space, identical on every rank."""
    items: list[str]                       # rank -> token
    levels: list[np.ndarray]               # levels[k-1]: int32 [F_k, k], rows ascending, lexicographic
    counts: list[np.ndarray]               # int64 [F_k]
    min_count: int
    n_lines: int
    stats: dict = field(default_factory=dict)

    @property
    def n_itemsets(self) -> int:
        return int(sum(len(c) for c in self.counts))

    def as_dict(self) -> dict[frozenset, int]:
        out = {}
        for rows, cnt in zip(self.levels, self.counts):
            for r, c in zip(rows.tolist(), cnt.tolist()):
                out[frozenset(r)] = int(c)
        return out
