"""Host-side native ops (libfa_host.so): candidate generation and rule building."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from ..utils.env import num_threads
from . import _native


def apriori_gen(prev: np.ndarray):
    """Join + full-prune candidate generation (csrc/host/apriori_gen.cpp).

    prev: int32 [n, m] frequent m-itemsets (rows ascending, lexicographic).
    Returns (prefix_idx int32 [G], ext_off int64 [G+1], ext int32 [C]).
    """
    prev = np.ascontiguousarray(prev, dtype=np.int32)
    n, m = prev.shape
    sizes = np.zeros(2, dtype=np.int64)
    lib = _native.host()
    h = lib.fa_apriori_gen(prev.ctypes.data, n, m, num_threads(), sizes.ctypes.data)
    G, Cn = int(sizes[0]), int(sizes[1])
    prefix = np.zeros(max(G, 1), dtype=np.int32)
    ext_off = np.zeros(G + 1, dtype=np.int64)
    ext = np.zeros(max(Cn, 1), dtype=np.int32)
    lib.fa_cands_export(h, prefix.ctypes.data, ext_off.ctypes.data, ext.ctypes.data)
    lib.fa_cands_free(h)
    return prefix[:G], ext_off, ext[:Cn]


@dataclass
class RuleTable:
    """Rules after the cut, in recommendation order (conf desc, tiebreak)."""
    ante_off: np.ndarray   # int64 [R+1]
    ante: np.ndarray       # int32 concatenated antecedent ranks (ascending)
    cons: np.ndarray       # int32 [R]
    conf: np.ndarray       # float64 [R]
    level_stats: list      # [(antecedent size, before cut, after cut)]
    level_ms: list = field(default_factory=list)   # [ms of each level's cut], same order

    @property
    def n_rules(self) -> int:
        return int(self.cons.size)

    def antecedent(self, i: int) -> np.ndarray:
        return self.ante[self.ante_off[i]:self.ante_off[i + 1]]


def rules_build(levels: list[np.ndarray], counts: list[np.ndarray], tie_pos: np.ndarray) -> RuleTable:
    K = len(levels)
    lv = [np.ascontiguousarray(l, dtype=np.int32) for l in levels]
    ct = [np.ascontiguousarray(c, dtype=np.int64) for c in counts]
    rows_p = (C.c_void_p * max(K, 1))(*[l.ctypes.data for l in lv])
    cnt_p = (C.c_void_p * max(K, 1))(*[c.ctypes.data for c in ct])
    sizes = np.array([l.shape[0] for l in lv] or [0], dtype=np.int64)
    tie = np.ascontiguousarray(tie_pos, dtype=np.int64)
    if tie.size == 0:
        tie = np.zeros(1, dtype=np.int64)
    nr = np.zeros(1, dtype=np.int64)
    lib = _native.host()
    h = lib.fa_rules_build(C.cast(rows_p, C.c_void_p), C.cast(cnt_p, C.c_void_p), sizes.ctypes.data, K,
                           tie.ctypes.data, num_threads(), nr.ctypes.data)
    R = int(nr[0])
    na = int(lib.fa_rules_nante(h))
    ns = int(lib.fa_rules_nstats(h))
    ante_off = np.zeros(R + 1, dtype=np.int64)
    ante = np.zeros(max(na, 1), dtype=np.int32)
    cons = np.zeros(max(R, 1), dtype=np.int32)
    conf = np.zeros(max(R, 1), dtype=np.float64)
    stats = np.zeros(max(ns, 1), dtype=np.int64)
    lib.fa_rules_export(h, ante_off.ctypes.data, ante.ctypes.data, cons.ctypes.data, conf.ctypes.data,
                        stats.ctypes.data)
    lib.fa_rules_free(h)
    st = stats[:ns].reshape(-1, 3)
    level_stats = [(i + 1, int(b), int(a)) for i, (b, a, _) in enumerate(st.tolist())]
    level_ms = [us / 1e3 for _, _, us in st.tolist()]
    return RuleTable(ante_off, ante[:na], cons[:R], conf[:R], level_stats, level_ms)


@dataclass
class TriePlan:
    """Work items of the trie-shared level kernel (csrc/host/plan.cpp)."""
    pieces: np.ndarray     # int32 [NP, 4]: (gpre offset, ext begin, ext end, flags), ext pass-local
    witems: np.ndarray     # int32 [NW, 2]: piece ranges, cost-sorted within each pass
    passes: np.ndarray     # int64 [npass, 3]: (work-item begin, end, ext base)
    d1: int
    d2: int
    reads: int             # estimated slab-row reads (per tile)
    reads_unshared: int    # the same without prefix sharing


def plan_trie(prefix: np.ndarray, ext_off: np.ndarray, emax: int, cap: int, d1: int = -1, d2: int = -1) -> TriePlan:
    """prefix: int32 [G, m] prefix rows in lexicographic order; ext_off: int64 [G+1]."""
    P = np.ascontiguousarray(prefix, dtype=np.int32)
    G, m = P.shape
    eo = np.ascontiguousarray(ext_off, dtype=np.int64)
    C = int(eo[-1] - eo[0])
    maxp = G + C // max(emax, 1) + 2
    pieces = np.zeros((maxp, 4), dtype=np.int32)
    witems = np.zeros((maxp, 2), dtype=np.int32)
    passes = np.zeros((maxp, 3), dtype=np.int64)
    info = np.zeros(8, dtype=np.int64)
    rc = _native.host().fa_plan_trie(P.ctypes.data, G, m, eo.ctypes.data, emax, cap, d1, d2, pieces.ctypes.data,
                                     witems.ctypes.data, passes.ctypes.data, maxp, info.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"fa_plan_trie failed ({rc})")
    npc, nw, npass = int(info[0]), int(info[1]), int(info[2])
    return TriePlan(pieces[:npc], witems[:nw], passes[:npass], int(info[3]), int(info[4]), int(info[5]),
                    int(info[6]))


def trie_records(plan: TriePlan, gpre: np.ndarray, gext: np.ndarray, m: int) -> np.ndarray:
    """32-B piece records of k_count_trie (plan.cpp fa_trie_records): int32 [n_pieces, 8].
    gpre: int32 [G, m] slab-row ids of the prefixes; gext: int32 [C] of the extensions."""
    pieces = np.ascontiguousarray(plan.pieces, dtype=np.int32)
    witems = np.ascontiguousarray(plan.witems, dtype=np.int32)
    passes = np.ascontiguousarray(plan.passes, dtype=np.int64)
    gp = np.ascontiguousarray(gpre, dtype=np.int32)
    ge = np.ascontiguousarray(gext, dtype=np.int32)
    rec = np.zeros((max(pieces.shape[0], 1), 8), dtype=np.int32)
    rc = _native.host().fa_trie_records(pieces.ctypes.data, witems.ctypes.data, passes.ctypes.data,
                                        passes.shape[0], gp.ctypes.data, ge.ctypes.data, m, plan.d1,
                                        rec.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"fa_trie_records failed ({rc})")
    return rec[:pieces.shape[0]]
