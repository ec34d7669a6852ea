"""Brute-force CPU oracle: the reference's observable behaviour, implemented literally.

This module is the ground truth every fast path (HIP kernels, the distributed
miner, the native host code) is tested against.  It deliberately shares no
code with the fast paths except the JVM-semantics helpers in
``fastapriori_amd.utils.jvm``.

Semantics reproduced:

* F1 counts token *occurrences* (``FastApriori.scala:55``: ``flatMap(_.map((_,1)))``);
  k >= 2 counts distinct sets over transactions that keep >= 2 frequent items
  (``FastApriori.scala:66-70``).
* ``minCount = ceil(minSupport * N)`` with N = all lines (``FastApriori.scala:38-39``).
* Rank = position after sort by count desc (``FastApriori.scala:60``); ties in the
  reference follow Spark's hash-partition collect order, which is not
  reproducible, so we break ties by Java string order (documented).
* Rules ``A -> s`` for every frequent S, |S| >= 2, A = S - {s},
  conf = count(S) / count(A) in IEEE double (``AssociationRules.scala:129-144``).
* Cut (``AssociationRules.scala:147-182``), sort (``:116-120``), first-match
  recommendation (``:80-106``).
"""
from __future__ import annotations

import itertools
from collections import Counter
from dataclasses import dataclass, field

from ..utils.jvm import item_tiebreak_key, java_split_ws, java_string_key, min_count, rule_tiebreak_key


@dataclass
class OracleResult:
    items: list[str]                       # rank -> token
    counts1: list[int]                     # rank -> occurrence count
    itemsets: dict[frozenset, int]         # frozenset of ranks -> count (all sizes)
    min_count: int
    n_lines: int
    rules: list[tuple[frozenset, int, float]] = field(default_factory=list)


def rank_items(counts: dict[str, int], mc: int, tiebreak: str = "string") -> list[str]:
    freq = [(t, c) for t, c in counts.items() if c >= mc]
    freq.sort(key=lambda tc: (-tc[1], item_tiebreak_key(tc[0], tiebreak)))
    return [t for t, _ in freq]


def mine(lines: list[list[str]], min_support: float, max_enum_len: int = 16, tiebreak: str = "string") -> OracleResult:
    n = len(lines)
    mc = min_count(min_support, n)
    occ = Counter()
    for toks in lines:
        occ.update(toks)
    items = rank_items(occ, mc, tiebreak)
    rank = {t: i for i, t in enumerate(items)}
    itemsets: dict[frozenset, int] = {frozenset([i]): occ[t] for i, t in enumerate(items)}

    txns: Counter = Counter()
    for toks in lines:
        s = frozenset(rank[t] for t in toks if t in rank)
        if len(s) > 1:
            txns[s] += 1

    if all(len(s) <= max_enum_len for s in txns):
        # independent brute force: every subset of every compressed transaction
        sub = Counter()
        for s, w in txns.items():
            srt = sorted(s)
            for k in range(2, len(srt) + 1):
                for c in itertools.combinations(srt, k):
                    sub[frozenset(c)] += w
        for s, c in sub.items():
            if c >= mc:
                itemsets[s] = c
    else:
        # level-wise fallback for long transactions
        prev = [frozenset([i]) for i in range(len(items))]
        k = 2
        while len(prev) >= k or k == 2:
            prevset = set(prev)
            cands = set()
            if k == 2:
                cands = {frozenset(p) for p in itertools.combinations(range(len(items)), 2)}
            else:
                for a, b in itertools.combinations(prev, 2):
                    u = a | b
                    if len(u) == k and all(u - {x} in prevset for x in u):
                        cands.add(u)
            cnt = Counter()
            for s, w in txns.items():
                for c in cands:
                    if c <= s:
                        cnt[c] += w
            prev = [c for c in cands if cnt[c] >= mc]
            for c in prev:
                itemsets[c] = cnt[c]
            k += 1
            if not prev:
                break
    return OracleResult(items=items, counts1=[occ[t] for t in items], itemsets=itemsets,
                        min_count=mc, n_lines=n)


def gen_rules(res: OracleResult) -> list[tuple[frozenset, int, float]]:
    """All rules, then the level-wise cut.  Returns the surviving rules unsorted."""
    by_level: dict[int, list[tuple[frozenset, int, float]]] = {}
    for s, c in res.itemsets.items():
        if len(s) < 2:
            continue
        for x in s:
            a = s - {x}
            by_level.setdefault(len(a), []).append((a, x, c / res.itemsets[a]))
    if not by_level:
        return []
    lo, hi = min(by_level), max(by_level)
    kept = list(by_level[lo])
    low = {(a, r): conf for a, r, conf in by_level[lo]}
    for i in range(lo + 1, hi + 1):
        nxt = {}
        for a, r, conf in by_level.get(i, []):
            ok = True
            for x in a:
                sub = a - {x}
                lc = low.get((sub, r))
                if lc is None or lc >= conf:
                    ok = False
                    break
            if ok:
                nxt[(a, r)] = conf
                kept.append((a, r, conf))
        low = nxt
    return kept


def sort_rules(rules, items: list[str]):
    """conf desc, then consequent as Int (AssociationRules.scala:116-120).  Remaining ties
    (same conf and consequent) are Spark collect order in the reference; they cannot change a
    recommendation, and we fix them as (antecedent size, antecedent ranks) for determinism."""
    return sorted(rules, key=lambda t: (-t[2], rule_tiebreak_key(items[t[1]]), len(t[0]),
                                        tuple(sorted(t[0]))))


def recommend(res: OracleResult, user_lines: list[list[str]]) -> list[str]:
    rules = sort_rules(gen_rules(res), res.items)
    rank = {t: i for i, t in enumerate(res.items)}
    out = []
    for toks in user_lines:
        u = frozenset(rank[t] for t in toks if t in rank)
        if not u:
            out.append("0")
            continue
        rec = "0"
        for a, r, _ in rules:
            if r not in u and a <= u:
                rec = res.items[r]
                break
        out.append(rec)
    return out


def freq_itemset_lines(res: OracleResult) -> list[str]:
    """``Utils.saveFreqItemset``: tokens rank-descending, lines in Java String order."""
    lines = [" ".join(res.items[r] for r in sorted(s, reverse=True)) for s in res.itemsets]
    lines.sort(key=java_string_key)
    return lines


def mining_log_lines(n_items: int, itemsets) -> list[str]:
    """The reference's mining lines (FastApriori.scala:226, :107-108, :111-119, :127) with
    the millisecond values masked as '#', replayed from the frequent itemsets alone:
    the loop runs while |F_{k-1}| >= k, and a level prints the number of
    (prefix, extensions) groups genCandidates keeps (:173-190), |F_k| and its time.
    ``itemsets``: an iterable of rank sets (every size; sizes 1 are ignored)."""
    by: dict[int, set] = {}
    for s in itemsets:
        s = frozenset(s)
        by.setdefault(len(s), set()).add(s)
    F1 = n_items
    out = [f"2 candidates items {F1 * (F1 - 1) // 2}", f"2 freq items {len(by.get(2, ()))}", "Use Time 2 items #"]
    k = 3
    while len(by.get(k - 1, ())) >= k:
        prev = by[k - 1]
        # y must at least pass the subset test for x's largest item, (x - max x) + y:
        # only the largest items of x's class mates are tried
        mates: dict[frozenset, list[int]] = {}
        for x in prev:
            mates.setdefault(x - {max(x)}, []).append(max(x))
        groups = 0
        for x in prev:
            top = max(x)
            for y in mates[x - {top}]:
                if y > top and all((x - {xi}) | {y} in prev for xi in x):
                    groups += 1
                    break
        out += [f"{k} candidate items {groups}", f"{k} freq items {len(by.get(k, ()))}", f"Use Time {k} items #"]
        k += 1
    out.append(f"Total freq items sets {sum(len(v) for kk, v in by.items() if kk >= 2)}")
    return out


def run_oracle(d_lines: list[str], u_lines: list[str], min_support: float, tiebreak: str = "string"):
    D = [java_split_ws(l) for l in d_lines]
    U = [java_split_ws(l) for l in u_lines]
    res = mine(D, min_support, tiebreak=tiebreak)
    return freq_itemset_lines(res), recommend(res, U), res
