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
