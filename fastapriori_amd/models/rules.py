"""AssociationRules: rule generation, redundancy cut, ordering, recommendation.

Reference: AssociationRules.scala (class AssociationRules, :17-190).

  reference (Spark)                                  here
  -------------------------------------------------  -----------------------------------------------
  removeRedundancy: zipWithIndex, map to rank sets,  native parse of this rank's U.dat byte range,
    reduceByKey dedup, collectAsMap (:33-64)         LUT to ranks on the device (empty -> "0")
  genRules: linear scan for S - {s} (:122-145)       HIP subset index: one thread per (S, position)
                                                     binary-searches level k-1 (csrc/hip/rules.hip)
  cut, level by level (:147-182)                     HIP dense lookup of the child rule through the
                                                     subset index (no hash table, no broadcast)
  sortWith(conf desc, token.toInt) (:74, :116-120)   device stable sorts on a packed key; HIP emit
                                                     (CPU runs: the same in C++, csrc/host/rules.cpp)
  per-basket first-match scan (:80-106)              HIP: one wave per basket, 64 rules per step,
                                                     __ballot + ffs for the earliest match; big rule
                                                     tables scan only the per-item rule lists of the
                                                     basket's items (k_recommend_indexed)
  collect to driver + saveRecommends                 gather of rank ids to rank 0

Divergences (documented): when there are no rules at all the reference throws
on ``rules.keys.min`` (:147); we recommend "0" for every user.  Non-integer
consequent tokens in a confidence tie would throw NumberFormatException there;
we order them after the integers by Java string order.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops
from ..ops.host import RuleTable, rules_build
from ..parallel.comm import Comm
from ..utils.jvm import rule_tiebreak_key
from ..utils.metrics import Logger
from .data import MiningResult, TransactionShard, Vocabulary, hash_tokens


class AssociationRules:
    def __init__(self, result: MiningResult, comm: Comm | None = None, logger: Logger | None = None,
                 device: torch.device | str | None = None):
        self.result = result
        self.comm = comm or Comm()
        self.log = logger or Logger(self.comm.rank)
        # rules are built where the job runs: the GPU kernels on a GPU rank, C++ on a CPU one
        self.device = torch.device(device) if device is not None else self.comm.device
        self._rules: RuleTable | None = None
        self._rules_dev = None
        self.use_index = True      # per-item rule lists for big rule tables (k_recommend_indexed)

    # ------------------------------------------------------------------
    def rules(self) -> RuleTable:
        if self._rules is None:
            items = self.result.items
            order = sorted(range(len(items)), key=lambda r: rule_tiebreak_key(items[r]))
            tie_pos = np.empty(len(items), dtype=np.int64)
            tie_pos[np.asarray(order, dtype=np.int64)] = np.arange(len(items), dtype=np.int64)
            if self.device.type == "cuda":
                d = ops.primitives.rules_build_device(self.result.levels, self.result.counts, tie_pos, self.device)
                self._rules = RuleTable(d["ante_off"].cpu().numpy(), d["ante"].cpu().numpy(),
                                        d["cons"].cpu().numpy(), d["conf"].cpu().numpy(), d["level_stats"],
                                        d["level_ms"])
                self._rules_dev = (self.device, d["ante_off"], d["ante"], d["cons"])
            else:
                self._rules = rules_build(self.result.levels, self.result.counts, tie_pos)
            # the cut's log lines per antecedent size (AssociationRules.scala:155,177,181),
            # then the rule total (:75)
            ms = list(self._rules.level_ms) + [0.0] * len(self._rules.level_stats)
            for (size, before, after), t in zip(self._rules.level_stats[1:], ms[1:]):
                self.log.line(f"Before cut level {size} Nums: {before}")
                self.log.line(f"After cut level {size} Nums: {after}")
                self.log.line(f"Use Time cut leaves {size} Time: {int(t)}")
                self.log.metric(phase="rule_cut", level=size, before=before, after=after, ms=round(t, 3))
            self.log.line(f"Size association rules {self._rules.n_rules}")
        return self._rules

    def rule_list(self) -> list[tuple[tuple[int, ...], int, float]]:
        rt = self.rules()
        return [(tuple(rt.antecedent(i).tolist()), int(rt.cons[i]), float(rt.conf[i]))
                for i in range(rt.n_rules)]

    # ------------------------------------------------------------------
    def _rank_lut(self, vocab: Vocabulary) -> np.ndarray:
        """User-shard id -> rank (-1 when the token is not a frequent item)."""
        lut = np.full(max(vocab.size, 1), -1, dtype=np.int32)
        if vocab.numeric:
            for r, t in enumerate(self.result.items):
                i = Vocabulary.numeric_id(t)
                if 0 <= i < vocab.size:
                    lut[i] = r
        elif vocab.size and self.result.items:
            # through the parser's 64-bit token hashes: no loop over the users' vocabulary
            rh = self.result.item_hashes
            if rh is None or len(rh) != len(self.result.items):
                rh = hash_tokens(self.result.items)     # e.g. results reloaded from files
            rh = np.asarray(rh, dtype=np.uint64)
            ro = np.argsort(rh)
            vh = vocab.hashes.astype(np.uint64)
            pos = np.minimum(np.searchsorted(rh[ro], vh), rh.size - 1)
            hit = rh[ro][pos] == vh
            lut[:vocab.size][hit] = ro[pos[hit]].astype(np.int32)
        return lut

    def recommend_shard(self, users: TransactionShard) -> torch.Tensor:
        """Recommended rank per local U.dat line (-1 = "0"), on the users' device.

        Identical baskets are recommended once (removeRedundancy's reduceByKey of the
        rank sets, AssociationRules.scala:51-58): baskets are canonicalised (ranks
        sorted), grouped by a 128-bit row hash, every group is verified equal to its
        representative element by element, and the representatives' results fan out
        to all lines of their group.  Cost O(distinct baskets) instead of O(lines) in
        the first-match scan."""
        rt = self.rules()
        dev = users.items.device
        lut = torch.from_numpy(self._rank_lut(users.vocab)).to(dev)
        n = users.n_lines
        if n == 0:
            return torch.zeros(0, dtype=torch.int32, device=dev)
        F1 = len(self.result.items)
        r = lut[users.items.to(torch.int64)] if users.items.numel() else users.items
        keep = r >= 0
        lens = users.offsets[1:] - users.offsets[:-1]
        row = torch.repeat_interleave(torch.arange(n, device=dev), lens)
        rk, rr = row[keep], r[keep].to(torch.int64)
        # canonical basket = its ranks ascending (the basket is a set)
        key, _ = torch.sort(rk * max(F1, 1) + rr)
        bask = (key % max(F1, 1)).to(torch.int32).contiguous()
        bcnt = torch.bincount(rk, minlength=n)
        boff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(bcnt, 0, out=boff[1:])
        if self._rules_dev is None or self._rules_dev[0] != dev:
            self._rules_dev = (dev, torch.from_numpy(rt.ante_off).to(dev), torch.from_numpy(rt.ante).to(dev),
                               torch.from_numpy(rt.cons).to(dev))
        _, a_off, ante, cons = self._rules_dev[:4]
        index = None
        if dev.type == "cuda" and cons.numel() >= ops.primitives.RECOMMEND_INDEX_MIN_RULES and self.use_index:
            if len(self._rules_dev) == 4:
                self._rules_dev = self._rules_dev + (ops.primitives.recommend_index(a_off, ante, F1),)
            index = self._rules_dev[4]
        groups = self._basket_groups(boff, bask, bcnt) if (self.dedup_baskets and n > 1) else None
        if groups is None:
            self.stats["distinct_baskets"] = n
            return ops.recommend(a_off, ante, cons, F1, boff, bask, index=index)
        rep, inv = groups
        self.stats["distinct_baskets"] = int(rep.numel())
        rcnt = bcnt[rep]
        roff = torch.zeros(rep.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(rcnt, 0, out=roff[1:])
        # gather the representatives' baskets into their own CSR
        pos = torch.repeat_interleave(boff[rep] - roff[:-1], rcnt) + torch.arange(int(roff[-1]), device=dev)
        rbask = bask[pos].contiguous()
        rec = ops.recommend(a_off, ante, cons, F1, roff, rbask, index=index)
        return rec[inv]

    dedup_baskets = True

    @property
    def stats(self) -> dict:
        if not hasattr(self, "_stats"):
            self._stats = {}
        return self._stats

    @staticmethod
    def _basket_groups(boff: torch.Tensor, bask: torch.Tensor, bcnt: torch.Tensor):
        """(representative basket per group, group of every basket), or None when
        dedup does not pay (few repeats) or a hash group fails the exact check."""
        n = bcnt.numel()
        h1, h2 = ops.row_hash(boff, bask)
        # empty baskets hash alike: give them a key of their own (length is part of it)
        key = torch.stack([h1, h2 ^ bcnt.to(torch.int64)], dim=1)
        uk, inv = torch.unique(key, dim=0, return_inverse=True)
        G = uk.shape[0]
        if G > 0.9 * n:
            return None
        first = torch.full((G,), n, dtype=torch.int64, device=bask.device)
        first.scatter_reduce_(0, inv, torch.arange(n, device=bask.device), reduce="amin")
        # exact check: every basket equals its group's representative
        rep_of = first[inv]
        if not torch.equal(bcnt, bcnt[rep_of]):
            return None
        if bask.numel():
            row = torch.repeat_interleave(torch.arange(n, device=bask.device), bcnt)
            j = torch.arange(bask.numel(), device=bask.device) - boff[row]
            if not torch.equal(bask, bask[boff[rep_of][row] + j]):
                return None
        return first, inv

    def run(self, users: TransactionShard) -> list[str] | None:
        """Recommendations for every U.dat line, in file order, on rank 0 (None elsewhere)."""
        ops.primitives.reset_fallbacks()     # the rules phase reports its own fallbacks
        rec = self.recommend_shard(users)
        if ops.primitives.FALLBACKS:
            self.stats["fallbacks"] = list(ops.primitives.FALLBACKS)
            for f in ops.primitives.FALLBACKS:
                self.log.metric(phase="fallback", what=f, stage="rules")
        parts = self.comm.gather_varlen(rec)
        if parts is None:
            return None
        items = self.result.items
        out = []
        for p in parts:
            out.extend("0" if v < 0 else items[v] for v in p.tolist())
        return out
