"""CPU model of the slab kernel's LDS bank conflicts (count.hip k_count_slab_rec).

A piece record's reads are its m prefix rows then its n_ext extension rows, one
slab row per read position, SW / 2 ds_read_b128 per row.  ds_read_b128 serves a wave
in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32); a group's read
takes one LDS cycle per distinct row that lands on its busiest 16-B slot, where row r
sits at slot (r * RS) mod 16 (RS = (SW + 2) / 2).  This replays the planner's record
order on real candidate sets (a T10I4 shard mined on the CPU) and reports the LDS
cycles per read relative to conflict-free (1.0) for

  * plan order (lexicographic within each n_ext bucket),
  * the lane deal (levels.hip k_dl_lane_assign: records re-dealt to lane groups,
    windows of 4 wave steps),
  * the deal plus a per-lane reorder of read positions: a lane's prefix rows may be
    ANDed in any order and its extensions counted in any order (the extension's slot
    in the record travels with its id), so each group's positions are re-scheduled
    step by step with a bipartite matching of lanes to free slots.

Usage: python benchmarks/lds_bank_model.py [--n 1000000] [--sw 8]
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import defaultdict

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
GROUPS += [[x + 32 for x in g] for g in GROUPS]


def mine(n: int, ms: float, avg_len: float = 10.0, pat: float = 4.0):
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger
    sh = generate_shard(n, Comm(), "cpu", avg_len, pat, 2000, 1000, 1)
    res = FastApriori(ms, config=MinerConfig(min_support=ms), logger=Logger(0, enabled=False)).run(sh)
    return res


def pieces(levels, counts1, k: int):
    """Level-k pieces (prefix ranks, extension ranks) in the planner's order: parents
    (F_{k-1} rows) lexicographic, extensions ascending, chunks of <= 8, bucketed by
    chunk size."""
    prev = np.asarray(levels[k - 2])
    rank = {}
    order = np.argsort(-np.asarray(counts1), kind="stable")
    for r, i in enumerate(order):
        rank[int(np.asarray(levels[0])[i]) if np.asarray(levels[0]).ndim == 1 else int(np.asarray(levels[0])[i][0])] = r
    prev_r = np.vectorize(lambda x: rank[int(x)])(prev) if prev.size else prev
    prev_r = np.sort(prev_r, axis=1)
    prev_r = prev_r[np.lexsort(prev_r.T[::-1])]
    fset = set(map(tuple, prev_r.tolist()))
    by_pre = defaultdict(list)
    for row in prev_r.tolist():
        by_pre[tuple(row[:-1])].append(row[-1])
    out = defaultdict(list)
    for row in prev_r.tolist():
        exts = []
        for c in by_pre[tuple(row[:-1])]:
            if c <= row[-1]:
                continue
            cand = row + [c]
            if all(tuple(cand[:j] + cand[j + 1:]) in fset for j in range(len(cand) - 2)):
                exts.append(c)
        for j in range(0, len(exts), 8):
            ch = exts[j:j + 8]
            out[len(ch)].append((row, ch))
    return out


def replay(recs, rs: int, reorder: bool = False, seg_only: int = -1) -> tuple[float, int]:
    """LDS cycles / conflict-free cycles over wave steps of 64 records (lane = index);
    seg_only 0 / 1: prefix / extension reads only."""
    cyc = base = 0
    for w0 in range(0, len(recs) - 63, 64):
        for g in GROUPS:
            lanes = [recs[w0 + x] for x in g]
            segs = [[r[0] for r in lanes], [r[1] for r in lanes]]
            for si, seg in enumerate(segs):
                if seg_only >= 0 and si != seg_only:
                    continue
                n = len(seg[0])
                steps = schedule(seg, rs) if reorder else [[lane[s] for lane in seg] for s in range(n)]
                for rows in steps:
                    occ = defaultdict(set)
                    for r in rows:
                        occ[(r * rs) & 15].add(r)
                    cyc += max(len(v) for v in occ.values())
                    base += 1
    return cyc / max(base, 1), base


def schedule(seg, rs: int):
    """Per step, a maximum matching of lanes to distinct slots among each lane's
    remaining rows (augmenting paths); unmatched lanes take any remaining row."""
    rem = [list(x) for x in seg]
    n = len(rem[0])
    steps = []
    for _ in range(n):
        owner = {}                              # slot -> (lane, row)
        pick = [None] * len(rem)

        def aug(l, seen):
            for r in rem[l]:
                s = (r * rs) & 15
                if s in seen:
                    continue
                seen.add(s)
                if s not in owner or owner[s][1] == r or aug(owner[s][0], seen):
                    if s in owner and owner[s][1] == r and owner[s][0] != l:
                        pick[l] = r            # same row: broadcast, share the slot
                        return True
                    owner[s] = (l, r)
                    pick[l] = r
                    return True
            return False

        # lanes with the fewest distinct slots first
        for l in sorted(range(len(rem)), key=lambda l: len({(r * rs) & 15 for r in rem[l]})):
            aug(l, set())
        for l in range(len(rem)):
            if pick[l] is None or pick[l] not in rem[l]:
                pick[l] = rem[l][0]
            rem[l].remove(pick[l])
        steps.append(pick)
    return steps


def deal(recs, rs: int, ws: int = 4, tail: bool = False):
    """levels.hip k_dl_lane_assign: windows of 64 * ws records re-dealt greedily;
    tail: the run's last partial window too (its whole wave steps)."""
    out = list(recs)
    starts = list(range(0, len(recs) - 64 * ws + 1, 64 * ws))
    end = starts[-1] + 64 * ws if starts else 0
    if tail and len(recs) - end >= 64:
        starts.append(end)
    for b in starts:
        NW = min(64 * ws, (len(recs) - b) // 64 * 64)
        NG = NW // 16
        lane_of = [[64 * (g >> 2) + x for x in GROUPS[g & 3]] for g in range(NG)]
        win = recs[b:b + NW]
        st = [defaultdict(dict) for _ in range(NG)]   # group -> pos -> slot -> {row: count}
        fill = [0] * NG
        for rec in win:
            rows = rec[0] + rec[1]
            best, bc = 0, None
            for g in range(NG):
                if fill[g] >= 16:
                    continue
                c = 0
                for p, r in enumerate(rows):
                    d = st[g][p].get((r * rs) & 15)
                    if d and r not in d:
                        c += sum(d.values())
                if bc is None or c < bc:
                    best, bc = g, c
            for p, r in enumerate(rows):
                d = st[best][p].setdefault((r * rs) & 15, {})
                d[r] = d.get(r, 0) + 1
            out[b + lane_of[best][fill[best]]] = rec
            fill[best] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--ms", type=float, default=0.001)
    ap.add_argument("--sw", type=int, default=8)
    ap.add_argument("--levels", default="3,4")
    ap.add_argument("--t40", action="store_true", help="T40I10 shape (|T| = 40, |I| = 10)")
    a = ap.parse_args()
    rs = (a.sw + 2) // 2
    res = mine(a.n, a.ms, *((40.0, 10.0) if a.t40 else (10.0, 4.0)))
    c1 = np.asarray(res.counts[0])
    for k in map(int, a.levels.split(",")):
        if k - 2 >= len(res.levels):
            continue
        pcs = pieces(res.levels, c1, k)
        used = sorted({x for b in pcs.values() for p, e in b for x in p + e})
        row = {r: i for i, r in enumerate(used)}
        for ne in sorted(pcs, reverse=True):
            recs = [([row[x] for x in p], [row[x] for x in e]) for p, e in pcs[ne]]
            if len(recs) < 256:
                continue
            r0, nb = replay(recs, rs)
            dl = deal(recs, rs)
            r1, _ = replay(dl, rs)
            p0, e0 = replay(recs, rs, seg_only=0)[0], replay(recs, rs, seg_only=1)[0]
            p1, e1 = replay(dl, rs, seg_only=0)[0], replay(dl, rs, seg_only=1)[0]
            r8, _ = replay(deal(recs, rs, 8, True), rs)
            r16, _ = replay(deal(recs, rs, 16, True), rs)
            r4t, _ = replay(deal(recs, rs, 4, True), rs)
            print(f"level {k} n_ext {ne}: {len(recs)} records, {nb} group reads: plan {r0:.2f}x (prefix {p0:.2f}x, "
                  f"ext {e0:.2f}x)  deal {r1:.2f}x (prefix {p1:.2f}x, ext {e1:.2f}x)  tail-dealt: ws4 {r4t:.2f}x ws8 {r8:.2f}x  ws16 {r16:.2f}x")


if __name__ == "__main__":
    main()
