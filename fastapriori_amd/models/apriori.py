"""FastApriori: level-wise frequent-itemset mining, count-distributed over GPUs.

Reference: FastApriori.scala (class FastApriori, :18-248).  Same observable
result — every itemset with support >= ceil(minSupport * N), F1 counted over
token occurrences, k >= 2 over distinct sets of transactions keeping >= 2
frequent items — computed the MI355X way:

  reference (Spark)                               here (per rank, then RCCL)
  ---------------------------------------------   --------------------------------------------
  flatMap/reduceByKey histogram (:55-58)          HIP LDS histogram + all_reduce(int64[V])
  rank by count (:60-62)                          identical host sort on every rank
  map->set->filter(size>1)->reduceByKey (:66-79)  HIP compress to sorted rank rows (+ optional
                                                  hash dedup into weight classes)
  F1 Spark jobs -> Boolean[T] per item (:195-210) HIP LDS-tiled build of uint64 bitmaps [F1][W]
  broadcast bitmaps, pairs parallelize (:212-241) HIP pair kernel (sparse: LDS pair tile from
                                                  rank rows; dense: bit-matrix Gram) +
                                                  all_reduce of the pair counts
  genCandidates (:167-193)                        C++ apriori_gen (identical on all ranks)
  genNextFreqItemsets (:132-160)                  HIP prefix-shared AND+popcount per group +
                                                  all_reduce(int64[C_k])

Transactions are sharded (count distribution); candidate lists and results
are replicated, so the only traffic is one count vector per level.
"""
from __future__ import annotations

import gc
import math
import os
import time
from dataclasses import dataclass

import numpy as np
import torch

from .. import ops
from ..ops.host import apriori_gen
from ..parallel.comm import Comm
from ..tuning import TUNING
from ..utils.jvm import item_tiebreak_key, min_count
from ..utils.metrics import Logger, Timer, roctx_range
from .data import MiningResult, TransactionShard

# Cost-model constants for choosing the k = 2 kernel (calibrated on MI355X; see
# docs/PERF.md).  Work units: pair increments for the horizontal kernel, 64-bit
# word pairs for the Gram kernel (the FP4 matrix-core form with its bitmap build:
# T40I10D100M 7.8e11 word pairs in a 46 ms pair phase).
HORIZONTAL_PAIRS_PER_S = 2.0e11
GRAM_WORDPAIRS_PER_S = 1.7e13
# numeric vocabularies at least this wide count F1 with the sketch + exact pass
F1_SKETCH_MIN_VOCAB = 1 << 20
# numeric vocabularies up to this wide read the whole F1 histogram back at once
F1_HIST_READBACK = 1 << 16
F1_MAX_CANDIDATES = ops.primitives.F1_MAX_CANDIDATES
_TRIU_CACHE: dict = {}
_POW10 = 10 ** np.arange(1, 11, dtype=np.int64)           # numeric token order (_frequent_items)
_POW10_PAD = 10 ** (10 - np.arange(0, 12).clip(max=10)).astype(np.int64)


class _Deferred:
    """Host work whose result is needed only later: run while a long kernel is in
    flight (FastApriori._run_deferred), or on first use."""

    def __init__(self, fn):
        self.fn, self.value, self.done = fn, None, False

    def result(self):
        if not self.done:
            self.value, self.done = self.fn(), True
        return self.value


@dataclass
class MinerConfig:
    min_support: float = 0.092
    dedup: str = "auto"             # auto | on | off
    pair_strategy: str = "auto"     # auto | horizontal | gram
    dedup_threshold: float = 0.8    # dedup when distinct/T below this (auto)
    max_level: int = 0              # 0 = unlimited
    level_kernel: str = "auto"      # auto (= slab) | slab | bitmap
    trim: bool = True               # transaction trimming before every level k >= 3
    f1: str = "auto"                # auto | sketch | histogram  (frequent-item counting)
    trim_min_rows: int = 1 << 20    # no trimming below this many rows (fixed cost > gain)
    timing: str = "off"             # off | events (hipEvent phase times) | sync (host-synchronised phases)
    trace: bool = False             # Chrome trace of the phases in stats["trace"] (--profile)
    tiebreak: str = "string"        # rank order of equal-count items: string | numeric (utils.jvm.item_tiebreak_key)
    parallelism: str = "count"      # count: rows sharded, counts all-reduced (default)
                                    # candidate: every rank holds the whole DB; pairs split by rows,
                                    #   level candidates split by rank: the device bundles' piece
                                    #   records, the host loop's prefix groups (FastApriori.scala:98-100,140)


class FastApriori:
    """Level-wise miner.  ``run(shard)`` on every rank returns the same MiningResult."""

    def __init__(self, min_support: float = 0.092, comm: Comm | None = None, config: MinerConfig | None = None,
                 logger: Logger | None = None, checkpoint=None):
        self.cfg = config or MinerConfig(min_support=min_support)
        self.cfg.min_support = min_support if config is None else self.cfg.min_support
        self.comm = comm or Comm()
        self.log = logger or Logger(self.comm.rank)
        self.ckpt = checkpoint
        self.stats: dict = {}

    # fluent setters of the reference (FastApriori.scala:21-29)
    def set_min_support(self, v: float) -> "FastApriori":
        self.cfg.min_support = float(v)
        return self

    # ------------------------------------------------------------------
    def run(self, shard: TransactionShard, resume: MiningResult | None = None) -> MiningResult:
        # no cyclic-GC passes inside a run: a generation-2 collection over the torch /
        # numpy heap costs milliseconds of host time between kernels (the run's own
        # temporaries are freed by reference counting)
        gc_on = gc.isenabled()
        gc.disable()
        try:
            return self._run(shard, resume)
        finally:
            if gc_on:
                gc.enable()

    def _run(self, shard: TransactionShard, resume: MiningResult | None = None) -> MiningResult:
        t_start = time.perf_counter()
        ops.primitives.reset_fallbacks()     # this run reports its own fallbacks only
        self._f2_dev = None                  # F_2 rows on the device (the first device bundle's input)
        self._f2_n_dev = None                # |F_2| on the device (F_2 not read back yet: _dl_flush)
        dev = shard.items.device
        # candidate parallelism: the data is replicated, so data-side collectives
        # (line count, F1, layout decisions) are local; only count vectors move
        self.cand_par = self.cfg.parallelism == "candidate" and self.comm.distributed
        self._deferred = []
        self.dcomm = Comm(device=self.comm.device) if self.cand_par else self.comm
        comm = self.dcomm
        # line total and numeric vocabulary width in one collective
        g = comm.all_gather_ints([shard.n_lines, shard.vocab.size if shard.vocab.numeric else 0])
        n_global, self._V_max = int(g[:, 0].sum()), int(g[:, 1].max())
        mc = min_count(self.cfg.min_support, n_global)
        self.stats = {"n_lines": n_global, "min_count": mc}
        # hipEvent phase timing (no synchronisation) whenever metrics are recorded
        gpu_timing = self.cfg.timing in ("events", "sync") or bool(self.log.metrics_path)
        tm = Timer(dev, sync=self.cfg.timing == "sync", events=gpu_timing)
        self._timer = tm
        self._level_recs = []     # per-level metric records, emitted by _finish with device times

        self._f1_pending = None
        cmp_pending = None
        with roctx_range("F1"), tm.phase("f1"):
            items, counts1, lut = self._frequent_items(shard, mc)
        f1p = self._f1_pending
        if f1p is not None:
            # ranked on the device: compression goes out right behind the ranking (its
            # block layout sized by the vocabulary width, which bounds F1) and the host
            # reads the ranking back while it runs -- no GPU idle between F1 and compression
            with roctx_range("compress"), tm.phase("compress"):
                if TUNING.early_compress:
                    cmp_pending = self._compress_start(shard, lut, f1p.V)
            with roctx_range("F1"):
                ids, counts1 = f1p.finish()
            items = _Deferred(lambda: ["" if i == 0 else str(i - 1) for i in ids.tolist()])
            self._deferred.append(items)
        F1 = len(counts1)
        self._F1, self._dev = F1, dev
        self._counts1 = counts1
        # compression's kernels go out right behind the LUT's copy: the host work below
        # (result, logs, checkpoint) overlaps them instead of idling the GPU
        # (the phase's two spans add up: Timer sums spans of one name)
        if f1p is None:
            with roctx_range("compress"), tm.phase("compress"):
                cmp_pending = self._compress_start(shard, lut, F1) if F1 >= 2 and TUNING.early_compress else None
        self.log.metric(phase="f1", frequent=F1)
        levels = [np.arange(F1, dtype=np.int32).reshape(-1, 1)]
        counts = [counts1]
        result = MiningResult(items, levels, counts, mc, n_global, self.stats,
                              item_hashes=None if shard.vocab.numeric else self._item_hashes)
        self._result = result
        # the device level loop reads its levels back once, at the end: its checkpoint
        # levels are written by a background thread from each bundle's staged copy
        # (_ckpt_staged), else per level
        self._ckpt_saved = 0
        self._ckpt_deferred = self.ckpt is not None and self._device_levels_planned(resume)
        self._result_items(result, wait=resume is not None or (self.ckpt is not None and not self._ckpt_deferred))
        if resume is not None:
            self._check_resume(resume, result)
        self._ckpt_level(result, 1)
        self._logged_upto, self._log_stop = 1, False     # the last level whose lines were printed
        if F1 < 2:
            # the reference still prints level 2 (FastApriori.scala:226, :107-108)
            self.log.line("2 candidates items 0")
            self.log.line("2 freq items 0")
            self.log.line("Use Time 2 items 0")
            self._logged_upto = 2
            return self._finish(result, t_start)

        with roctx_range("compress"), tm.phase("compress"):
            if cmp_pending is None and F1 >= 2:
                cmp_pending = self._compress_start(shard, lut, F1)
            db = self._compress(shard, lut, F1, cmp_pending)
        self._db_local = db

        # ---- k = 2 -----------------------------------------------------
        t0 = time.perf_counter()
        b0 = self._bytes_moved()
        # F_2 may stay on the device (no readback between the pair kernel and the first
        # device bundle): its host copy then arrives with the run's one results readback
        resumed = 0 if resume is None else len(resume.levels)
        self._f2_defer = self._device_levels_planned(resume) and resumed < 2
        if resumed >= 2:
            levels.append(resume.levels[1]); counts.append(resume.counts[1])
        else:
            with roctx_range("pairs"), tm.phase("pairs"):
                rows2, cnt2 = self._pairs(db, F1, mc)
            levels.append(rows2); counts.append(cnt2)
            self._ckpt_level(result, 2)
        self.log.line(f"2 candidates items {F1 * (F1 - 1) // 2}")
        self._level2_ms, self._level2_bytes = (time.perf_counter() - t0) * 1e3, self._bytes_moved() - b0
        if levels[1] is not None:
            self._log_level2(len(levels[1]))

        # ---- k >= 3 ----------------------------------------------------
        k = 3
        while resumed >= k:                  # levels the checkpoint already holds
            levels.append(resume.levels[k - 1]); counts.append(resume.counts[k - 1])
            k += 1
        self._logged_upto = max(self._logged_upto, resumed)
        if self._device_levels_ok(resume, levels):
            # device bundles while every bundle fits one accumulator pass; None when
            # mining is complete, else the level the host loop continues from
            k = self._mine_device(db, levels, counts, mc, result)
        if k is not None and self._ckpt_deferred:
            # the host loop checkpoints per level from here: the levels before it first
            self._ckpt_deferred = False
            self._result_items(result)
            self._ckpt_upto(result, len(levels), background=False)
        while k is not None and len(levels[-1]) >= k and (self.cfg.max_level == 0 or k <= self.cfg.max_level):
            t0 = time.perf_counter()
            b0 = self._bytes_moved()
            with roctx_range(f"level{k}"), tm.phase(f"level{k}"):
                fused = self._gen_bundle_fused(k, levels[-1])
                if fused is None:
                    with tm.phase("apriori_gen"), roctx_range("gen"):
                        prefix_idx, ext_off, ext, cand_rows = self._gen(levels[-1], want_rows=True)
                else:
                    prefix_idx, ext_off, ext, cand_rows = fused[0] if fused else (None, None, np.zeros(0, np.int32),
                                                                                  None)
                C = int(ext.size)
                # the reference logs candidates.length: its (prefix, extensions) groups
                # (FastApriori.scala:114, :189-190)
                self.log.line(f"{k} candidate items {0 if prefix_idx is None else int(prefix_idx.size)}")
                if C == 0:
                    levels.append(np.zeros((0, k), np.int32)); counts.append(np.zeros(0, np.int64))
                    self._log_level(levels, k, 0, 0, (time.perf_counter() - t0) * 1e3, cand_line=False)
                    break
                # level bundling: count the next levels' candidates, generated from this
                # level's candidates, in the same launch (see _plan_bundle)
                if fused is not None:
                    bundle = self._bundle_from_chain(k, levels[-1], fused)
                else:
                    with tm.phase("apriori_gen"), roctx_range("bundle"):
                        bundle = self._plan_bundle(db, k, levels[-1], prefix_idx, ext_off, ext, cand_rows)
                # later bundled levels only use items of level k's candidates
                mark = np.zeros(max(db["F1"], 1), dtype=bool)
                mark[self._bundle_rows[0].ravel()] = True
                used = np.flatnonzero(mark)
                with tm.phase(f"trim{k}"), roctx_range("trim"):
                    self._trim(db, used, k, sum(int(b[4].size) for b in bundle))
                with tm.phase("count"), roctx_range("count"):
                    cnts = self._count_bundle(db, bundle)
                if tm.sync:
                    self.stats.setdefault("level_info", {})[k] = dict(ops.primitives.LAST_LEVEL_PLAN,
                                                                      groups=int(prefix_idx.size),
                                                                      bundled=len(bundle))
                for cand_k, cnt in zip(self._bundle_rows, cnts):
                    keep = cnt >= mc          # candidate rows are in count order
                    levels.append(np.ascontiguousarray(cand_k[keep], dtype=np.int32))
                    counts.append(cnt[keep].astype(np.int64))
            ms = (time.perf_counter() - t0) * 1e3
            plan = ops.primitives.LAST_LEVEL_PLAN
            hbm_b, moved = self._level_hbm_bytes(db, plan), self._bytes_moved() - b0
            c_tot = max(sum(int(b[4].size) for b in bundle), 1)
            for j, (kk, pv, pi, eo, ex) in enumerate(bundle):
                Fk = levels[kk - 1]
                # one launch counts the bundle: each level gets its candidates' share.  The
                # reference logs the groups generated from F_{k-1}; a bundled level counted
                # a superset generated from C_{k-1}
                share = int(ex.size) / c_tot
                self._log_level(levels, kk, lambda kk=kk: int(apriori_gen(levels[kk - 2])[0].size), len(Fk),
                                ms * share, cand_line=kk > k)
                rec = dict(phase="level", k=kk, candidates=int(ex.size), frequent=len(Fk),
                           ms=ms * share, groups=int(pi.size), bundled_with=k, bytes_reduced=int(moved * share),
                           kernel=plan.get("kernel"), hbm_bytes_est=int(hbm_b * share) + 4 * int(ex.size) * (kk + 3),
                           _share=share)
                self._level_recs.append((rec, f"level{k}"))
                self._ckpt_level(result, kk)
            self.stats["host_levels"] = self.stats.get("host_levels", 0) + len(bundle)
            k += len(bundle)
        # drop a trailing empty level (the reference never emits empty levels)
        while len(levels) > 1 and len(levels[-1]) == 0:
            levels.pop(); counts.pop()
        return self._finish(result, t_start)

    @staticmethod
    def _entered(levels: list, kk: int) -> bool:
        """The reference runs level kk while |F_{kk-1}| >= kk (FastApriori.scala:111)."""
        return 2 <= kk - 1 <= len(levels) and len(levels[kk - 2]) >= kk

    def _log_level(self, levels: list, kk: int, groups, n_freq: int, ms: float, cand_line: bool = True) -> None:
        """The three lines of a level the reference enters (FastApriori.scala:114, :118-119);
        none for a level it never enters -- a bundled level past the stop rule, empty
        by construction -- nor for any level after it.  groups: the candidate group
        count, or a callable computing it (only when the lines are printed)."""
        if self._log_stop or not self._entered(levels, kk):
            self._log_stop = True
            return
        if cand_line and self.log.enabled:
            self.log.line(f"{kk} candidate items {groups() if callable(groups) else int(groups)}")
        self.log.line(f"{kk} freq items {n_freq}")
        self.log.line(f"Use Time {kk} items {int(ms)}")
        self._logged_upto = kk

    def _log_tail(self, levels: list) -> None:
        """Levels the reference enters after the last counted one: |F_{k-1}| >= k with no
        candidates (the device loop stops on C_k = 0 without counting anything)."""
        if self.cfg.max_level or self._log_stop:
            return
        kk = self._logged_upto + 1
        while self._entered(levels, kk):
            n = len(levels[kk - 1]) if kk - 1 < len(levels) else 0
            self._log_level(levels, kk, lambda kk=kk: int(apriori_gen(levels[kk - 2])[0].size), n, 0.0)
            kk += 1

    def _log_level2(self, n2: int) -> None:
        F1 = self._F1
        self.log.line(f"2 freq items {n2}")
        self.log.line(f"Use Time 2 items {int(self._level2_ms)}")
        self._logged_upto = max(self._logged_upto, 2)
        self._level_recs.append((dict(phase="level", k=2, candidates=F1 * (F1 - 1) // 2, frequent=n2,
                                      ms=self._level2_ms, strategy=self.stats.get("pair_strategy"),
                                      bytes_reduced=self._level2_bytes,
                                      hbm_bytes_est=self.stats.get("pair_hbm_bytes_est", 0)),
                                 "pairs"))

    # ------------------------------------------------------------------
    # k >= 3 on the device (FastApriori.scala:110-121, :132-160)
    # ------------------------------------------------------------------
    def _device_levels_planned(self, resume) -> bool:
        return (TUNING.device_levels and self._dev.type == "cuda"
                and 2 <= self._F1 <= ops.primitives.DL_MAX_F1
                and self.cfg.level_kernel in ("auto", "slab") and self.stats["n_lines"] < (1 << 31)
                and (self.cfg.max_level == 0 or self.cfg.max_level >= 3))

    def _device_levels_ok(self, resume, levels: list) -> bool:
        """F_2 on the device (_pairs_on_device / _pairs), or a resumed checkpoint's last
        level, uploaded by _mine_device as the first bundle's parent rows."""
        if not self._device_levels_planned(resume):
            return False
        return self._f2_dev is not None or (resume is not None and len(levels) >= 2 and levels[-1] is not None)

    def _ckpt_level(self, result: MiningResult, k: int) -> None:
        """Checkpoint level k now (host level loop), unless the device loop's levels are
        written from their staged copies by the checkpoint thread (_ckpt_deferred, _ckpt_staged)."""
        if self.ckpt is not None and not self._ckpt_deferred:
            self.ckpt.save_level(result, k)
            self._ckpt_saved = max(self._ckpt_saved, k)

    def _ckpt_upto(self, result: MiningResult, K: int, background: bool) -> None:
        if self.ckpt is not None and K > self._ckpt_saved:
            self.ckpt.save_levels(result, range(self._ckpt_saved + 1, K + 1), background=background)
            self._ckpt_saved = K

    def _mine_device(self, db, levels: list, counts: list, mc: int, result: MiningResult):
        self._piece_part(True)
        try:
            return self._mine_device_loop(db, levels, counts, mc, result)
        finally:
            self._piece_part(False)

    def _mine_device_loop(self, db, levels: list, counts: list, mc: int, result: MiningResult):
        """Level bundles with no host round trip beyond the generator's (csrc/hip/gen.hip
        fa_hip_dl_level0 / fa_hip_dl_more, csrc/hip/levels.hip).

        Per bundle: level k's candidates from F_{k-1} rows already on the GPU (F_2, or
        the previous bundle's thresholded rows, their number read by the kernels from
        device memory) and the speculative levels k+1.. accepted on the device, all
        queued before ONE synchronisation that returns C_k.., the used items
        (trimming, slab width) and whether level k fits one accumulator pass; then the
        piece plan, the slab count, the count all-reduce and the threshold into F
        rows, queued on the stream.  The results reach the host once, after the last
        bundle.
        Returns None when mining is complete, or the level from which the host loop
        continues (a level that needs several accumulator passes, or prefixes too long
        for inline piece records): levels/counts then hold F_1 .. F_{k-1}."""
        Pm = ops.primitives
        S = Pm.device_level_state(self._dev)
        F1 = self._F1
        lds = Pm.dl_lds_budget(F1)
        # LDS bytes per slab accumulator: packed u16 counters for unit weights (the rows'
        # weighting does not change while mining: trimming keeps the dedup layout) in
        # window-by-window levels; u32 in one-pass bundles (TUNING.dl_acc16)
        unit = db["wword"] is None
        self._dl_mp_accb = 2.0 if TUNING.dl_acc16 and unit else 4.0
        accb = self._dl_accb = 2.0 if TUNING.dl_acc16_bundles and unit else 4.0
        c_bound = int(lds // accb)
        st = torch.cuda.current_stream(self._dev).cuda_stream
        f2 = self._f2_dev
        m0, k = 2, 3
        if f2 is None:
            # resumed from a checkpoint: its last level's rows are the first parents
            last = np.ascontiguousarray(levels[-1], dtype=np.int32)
            m0, k = last.shape[1], last.shape[1] + 1
            f2 = self._resume_rows = torch.from_numpy(last.reshape(-1, m0)).to(self._dev)
        if self._f2_n_dev is not None:      # |F_2| only on the device; n_bound sizes the buffers
            P0, n_src, n_const, n_bound = f2.data_ptr(), self._f2_n_dev.data_ptr(), 0, self._f2_bound
        else:
            P0, n_src, n_const, n_bound = f2.data_ptr(), None, int(f2.shape[0]), int(f2.shape[0])
        if self.ckpt is not None and self._ckpt_deferred:
            # the levels already on the host (F_1; F_2 when it was read back) before any bundle
            self._result_items(result)
            n_host = next((i for i, lv in enumerate(levels) if lv is None), len(levels))
            self._ckpt_upto(result, n_host, background=True)
        pend = []
        tm = self._timer
        nxt = None
        self._dl_stg = dict(n=0, rows=[], cnt=[], f2=None, ev=None, stream=getattr(self, "_dl_stage_stream", None))
        while True:
            if self.cfg.max_level and k > self.cfg.max_level:
                break
            if m0 > Pm.DL_MAX_M:
                nxt = k
                break
            t0 = time.perf_counter()
            b0 = self._bytes_moved()
            with roctx_range(f"dlevel{k}"), tm.phase(f"level{k}"):
                max_lv = min(Pm.DL_MAX_M - m0 + 1, Pm.DL_MAX_LEVELS)
                if self.cfg.max_level:
                    max_lv = min(max_lv, self.cfg.max_level - k + 1)
                if not TUNING.bundle_levels or k - 1 > TUNING.bundle_max_prefix:
                    max_lv = 1
                post = TUNING.dl_post and max_lv > 1
                S.rows_hint = int(self._count_view(db)["ncols"])
                if post:
                    self._dl_post_setup(S, db, k, F1, c_bound, n_bound, lds)
                # the results not staged yet go to the host on a copy stream while this
                # bundle runs: when the generator finds the mining over, _dl_flush only waits
                if pend:
                    self._dl_stage(S, pend)
                with roctx_range("gen"):
                    c = Pm.dl_bundle_gen(S, P0, n_src, n_const, n_bound, m0, F1, c_bound, lds, TUNING.bundle_growth,
                                         max_lv, st, post=post, accb=accb)
                if c[4]:
                    raise RuntimeError(f"device bundle at level {k}: |F_{k - 1}| exceeds its bound {n_bound}")
                if c[7]:
                    break                               # |F_{k-1}| < k or no candidates: done
                multi = None
                if c[5]:
                    # level k alone needs several accumulator passes: counted on the device
                    # window by window (else the host loop takes over from level k)
                    multi = self._dl_multipass(S, db, k, F1, c, P0, n_src, n_const, n_bound, m0, lds, st)
                    if multi is None:
                        nxt = k
                        break
                    c = multi[0]
                L, n_used = int(c[1]), int(c[6])
                Cs = S.desc[:L, 6].copy()
                C = int(Cs.sum())
                done = int(S.post.done) if post else 0
                sw = int(S.post.sw) if done else 0
                if multi is not None:
                    cnt = multi[1]
                    sw = int(Pm.LAST_LEVEL_PLAN.get("sw", 0))
                elif done == 2:
                    # planned and counted by fa_hip_dl_more's post step (no trim due)
                    cnt = S.post_bufs["out"][:C]
                else:
                    nwd = (F1 + 63) // 64
                    bits = np.unpackbits(c[Pm.DL_BITS:Pm.DL_BITS + nwd].view(np.uint8), bitorder="little")[:F1]
                    used = np.flatnonzero(bits)
                    if done == 1:
                        plan = Pm.dl_plan_from_post(S, n_used)
                    else:
                        with roctx_range("plan"):
                            plan = Pm.dl_plan(S, L, F1, n_used, C, lds, self._dev, accb)
                    with tm.phase(f"trim{k}"), roctx_range("trim"):
                        self._trim(db, used, k, C, decided=bool(done == 1 and S.post.trim))
                    with tm.phase("count"), roctx_range("count"):
                        v = self._count_view(db)
                        cnt = Pm.dl_count(S, plan, v["roff"], v["ranks"], v["src"], v["ncols"], F1, v["wword"])
                    sw = int(plan["sw"])
                # candidate distribution: the candidates this rank counted (non-zero
                # before the sum; read back with the results, for the stats)
                nz = torch.count_nonzero(cnt) if self.cand_par else None
                with tm.phase("count"), roctx_range("count"):
                    self.comm.all_reduce_(cnt)
                    rows_a, cnt_a, ro, co = Pm.dl_threshold(S, L, cnt, mc, k)
            # HBM bytes the bundle's slab count streams (rows + offsets, one pass)
            hbm_rows = (db["ranks"].numel() * db["ranks"].element_size()
                        + db["roff"].numel() * db["roff"].element_size())
            pend.append(dict(k=k, L=L, m0=m0, C=Cs, rows=rows_a, cnt=cnt_a, ro=ro, co=co, hbm_rows=int(hbm_rows),
                             n_par=S.desc[:L, 5].copy(), sw=sw, used=n_used, T=int(db["roff"].numel() - 1),
                             ms=(time.perf_counter() - t0) * 1e3, bytes=self._bytes_moved() - b0,
                             G=c[72:72 + L].copy(), nz=nz))
            P0 = rows_a.data_ptr() + 4 * int(ro[L - 1])
            n_src, n_const, n_bound = S.fsz.data_ptr() + 8 * (k + L - 1), 0, int(Cs[-1])
            m0 += L
            k += L
            # the next bundle's generator would only find the end (one more host round
            # trip): |F_{k-1}| <= C_{k-1} < k fails the reference's loop test
            # (FastApriori.scala:111), or the chain already found no k-candidates from
            # C_{k-1}, a superset of F_{k-1}
            if int(Cs[-1]) < k or (multi is None and int(c[Pm.DL_EMPTY])):
                break
        self._dl_flush(S, pend, levels, counts, result)
        if self.cand_par and pend:
            self.stats["cand_counted"] = int(sum(int(p["nz"]) for p in pend if p["nz"] is not None))
            self.stats["cand_total"] = int(sum(int(p["C"].sum()) for p in pend))
        self.stats["device_bundles"] = len(pend)
        self.stats["device_levels"] = int(sum(p["L"] for p in pend))
        return nxt

    def _dl_multipass(self, S, db, k: int, F1: int, c, P0, n_src, n_const: int, n_bound: int, m0: int, lds: int,
                      st):
        """Level k of a device bundle whose candidates exceed one accumulator pass
        (FastApriori.scala:132-160 at any size): its candidates generated again with
        room for all of them when the bounded generation stopped short, the level's
        rows trimmed as the host loop would, then counted window by window from the used
        items' bitmap (ops.primitives.dl_count_multipass).  Returns (control block,
        int32 counts [C] on the device) or None (TUNING.dl_multi off: the host loop).  When
        not even 4-word slabs of the used items fit the LDS (wide levels: thousands of
        used items), the level is counted by the bitmap kernel instead (_dl_bitmap_count)."""
        Pm = ops.primitives
        if not TUNING.dl_multi or self.cfg.max_level and k > self.cfg.max_level:
            return None
        C0 = int(c[40])
        if int(c[1]) == 0:
            # the bounded generation reported the size only: again, one level, room for C0
            c = Pm.dl_bundle_gen(S, P0, n_src, n_const, n_bound, m0, F1, C0, lds, TUNING.bundle_growth, 1, st,
                                 accb=self._dl_accb)
            if c[4] or c[7] or int(c[1]) != 1 or int(c[40]) != C0:
                raise RuntimeError(f"device level {k}: regeneration of {C0} candidates disagrees ({c[:8]})")
        nwd = (F1 + 63) // 64
        bits = np.unpackbits(c[Pm.DL_BITS:Pm.DL_BITS + nwd].view(np.uint8), bitorder="little")[:F1]
        used = np.flatnonzero(bits)
        n_used = int(used.size)
        wide = Pm.dl_slab_width(n_used, min(C0, 8192), lds, self._dl_mp_accb)[0] == 0
        with self._timer.phase(f"trim{k}"), roctx_range("trim"):
            self._trim(db, used, k, C0)
        v = self._count_view(db)
        if wide:
            with self._timer.phase("count"), roctx_range("count_bitmap"):
                cnt = self._dl_bitmap_count(S, v, used)
            self.stats["device_bitmap_levels"] = self.stats.get("device_bitmap_levels", 0) + 1
            return c, cnt
        with self._timer.phase("count"), roctx_range("count_multi"):
            bm, bmap = self._bitmaps(v, used, blocked=True)
            used_t = torch.from_numpy(used.astype(np.int64)).to(self._dev)
            bm_rows = (bmap[used_t] if bmap is not None else used_t).to(torch.int32).contiguous()
            wr = None
            if (self.cfg.trim and TUNING.window_trim and v["wword"] is None and v["src"] is None
                    and v["T"] >= self.cfg.trim_min_rows
                    and v.get("T0", v["T"]) >= TUNING.window_trim_min_rows):
                wr = lambda used_w, nc: self._window_rows(v, used_w, k, bm, bmap, nc)        # noqa: E731
            cnt = Pm.dl_count_multipass(S, F1, n_used, C0, lds, v["roff"], v["ranks"], v["src"], v["ncols"],
                                        v["wword"], bm, bm_rows,
                                        self.stats["min_count"] / max(1, self.stats["n_lines"]), self._dev,
                                        bmap=bmap, window_rows=wr)
            plan = Pm.LAST_LEVEL_PLAN
            if plan.get("windows_trimmed"):
                self.stats["window_trims"] = self.stats.get("window_trims", 0) + int(plan["windows_trimmed"])
        if cnt is None:
            return None
        self.stats["device_multipass"] = self.stats.get("device_multipass", 0) + 1
        return c, cnt

    def _window_rows(self, db, used_w: np.ndarray, k: int, bm, bmap, n_cand: int):
        """Rows of one window of a multi-pass level (ops.primitives.dl_count_multipass):
        a window's candidates use only its own items (used_w), so a row holding fewer
        than k of them contains none of its k-candidates.  Unless the binomial estimate
        (_trim_worth_it's, with the window's items) keeps most of the level's rows, the
        level's bitmap bm is compressed to the rows that hold >= k of the window's items
        (ops.primitives.window_bitmap: count.hip k_win_alive / k_win_compact, in the
        bitmap domain, no pass over the transaction rows), and the window counts from
        that: (ncols, bitmap [len(used_w), Wp], bitmap row u = slab row u).  Deep T40I10
        levels: windows use a third to a half of their level's items, so a third to half
        of the level's rows drop out of a window.  None: the window counts the level's
        rows: the rows kept would save less than the compaction costs.  That cost follows
        the window's items x the level's bitmap words, the window's count its candidates x
        ~(k + 1) slab rows read per candidate, so the window is compacted only below
        1 - TUNING.window_trim_cost * items / (candidates * (k + 1)) of the level's rows
        (capped at TUNING.window_trim_rows_frac; T40I10D100M: ~0.8 for a level-5 window of
        ~370 items, ~0.97 for a level-9 one of ~150).
        (FastApriori.scala:132-160 counts every row per candidate.)"""
        if bm is None or used_w.size > ops.primitives.WINDOW_MAX_ITEMS:
            return None
        keep = min(TUNING.window_trim_rows_frac,
                   1.0 - TUNING.window_trim_cost * used_w.size / max(1, n_cand * (k + 1)))
        est = self._trim_estimate(db, used_w, k)
        wlog = self.stats.setdefault("window_log", [])
        rec = dict(k=k, items=int(used_w.size), cand=int(n_cand), keep=round(keep, 3),
                   est=None if est is None else round(est / max(1, db["T"]), 3))
        wlog.append(rec)
        if keep <= 0 or est is None or est >= TUNING.window_trim_est_frac * db["T"]:
            return None
        dev = db["ranks"].device
        used_t = torch.from_numpy(used_w.astype(np.int64)).to(dev)
        rows_w = (bmap[used_t] if bmap is not None else used_t).to(torch.int32).contiguous()
        with roctx_range("window_rows"):
            got = ops.primitives.window_bitmap(bm, rows_w, (int(db["ncols"]) + 63) // 64, k,
                                               max_keep=int(keep * db["T"]))
        rec["kept"] = None if got is None else round(got[0] / max(1, db["T"]), 3)
        return got

    @staticmethod
    def _trim_estimate(db, used: np.ndarray, k: int, with_nnz: bool = False):
        """Rows expected to keep >= k of the items `used` (and, with_nnz, the item
        occurrences they keep): item occurrences survive with probability p = (supports
        of `used`) / (supports of the items still in the rows), a row of length L keeps
        >= k with P[Binom(L, p) >= k] = I_p(k, L - k + 1) (regularised incomplete beta).
        None without a length histogram or items."""
        from scipy.special import betainc
        hist = db.get("len_hist")
        if hist is None:
            return None
        c1, alive = db["c1"], db["alive"]
        denom = float(c1[alive].sum())
        if denom <= 0:
            return None
        p = min(float(c1[used].sum()) / denom, 1.0)
        L = np.arange(hist.size)
        sf = np.zeros(hist.size)
        ok = L >= k
        if p > 0:
            sf[ok] = betainc(k, L[ok] - k + 1, p)
        rows = float((hist * sf).sum())
        return (rows, float((hist * L * p).sum())) if with_nnz else rows

    def _dl_bitmap_count(self, S, db, used: np.ndarray) -> torch.Tensor:
        """Counts (int32 [C], bundle order) of the device bundle's single level from the
        used items' bitmap with the bitmap kernel (ops.count_candidates: every group's
        prefix ANDed once per word tile, FastApriori.scala:143-154): the candidate rows
        are read where the generator wrote them (its workspace), grouped by prefix on
        the device; one readback of the group offsets."""
        Pm = ops.primitives
        m, C = int(S.desc[0, 4]), int(S.desc[0, 6])
        off = int(S.desc[0, 3]) - S.ws.data_ptr()
        if off < 0 or off % 4 or off + 4 * C * (m + 1) > S.ws.numel():
            raise RuntimeError("device bundle: candidate rows outside the generator workspace")
        rows = S.ws[off:off + 4 * C * (m + 1)].view(torch.int32).view(C, m + 1)
        pre, ext = rows[:, :m], rows[:, m]
        starts = torch.zeros(1, dtype=torch.int64, device=self._dev)
        if C > 1:
            starts = torch.cat([starts, torch.nonzero((pre[1:] != pre[:-1]).any(1)).flatten() + 1])
        gs = starts.cpu().numpy()
        ext_off = np.append(gs, C).astype(np.int64)
        bm, bmap = self._bitmaps(db, used)
        prefix = pre[starts].to(torch.int64)
        ext64 = ext.to(torch.int64)
        if bmap is not None:
            prefix, ext64 = bmap[prefix], bmap[ext64]
        if self.cand_par:
            # candidate distribution: this rank's extension-balanced range of the groups,
            # the other counts 0 (the all-reduce assembles them, as _count_level)
            r, nr = self.comm.rank, self.comm.world_size
            g0, g1 = (int(np.searchsorted(ext_off, C * q // nr, side="left")) for q in (r, r + 1))
            g1 = gs.size if r == nr - 1 else g1
            e0, e1 = int(ext_off[g0]), int(ext_off[g1])
            cnt = torch.zeros(C, dtype=torch.int32, device=self._dev)
            if g1 > g0:
                part = ops.count_candidates(bm, db["W"], prefix[g0:g1].to(torch.int32).contiguous(),
                                            ext_off[g0:g1 + 1] - e0, ext64[e0:e1].to(torch.int32).contiguous(),
                                            db["wword"])
                cnt[e0:e1] = part.to(torch.int32)
            return cnt
        cnt = ops.count_candidates(bm, db["W"], prefix.to(torch.int32).contiguous(), ext_off,
                                   ext64.to(torch.int32).contiguous(), db["wword"])
        Pm.LAST_LEVEL_PLAN.clear()
        Pm.LAST_LEVEL_PLAN.update(kernel="bitmap_dev", rows=int(db["roff"].numel() - 1), used=int(used.size), C=C, m=m)
        return cnt.to(torch.int32)

    def _count_view(self, db) -> dict:
        """The rows the device bundles count: all of this rank's rows -- its shard (count
        distribution), or the whole replicated DB (candidate distribution: the rank
        counts its share of the plan's pieces over every row, _piece_part)."""
        return db

    def _piece_part(self, on: bool) -> None:
        """Candidate distribution of the device bundles (FastApriori.scala:98-100,140):
        every slab count launched from here on counts only this rank's chunks of the
        piece records (count.hip fa_hip_set_piece_part), so each candidate is counted
        by one rank over all rows and the all-reduce assembles the full vector."""
        r, n = (self.comm.rank, self.comm.world_size) if (on and self.cand_par) else (0, 1)
        ops.primitives.set_piece_part(r, n)

    def _dl_post_setup(self, S, db, k: int, F1: int, c_bound: int, n_bound: int, lds: int) -> None:
        """Fill the post step of fa_hip_dl_more (ops.primitives.DlPostC): buffers, the
        current rows and the trimming inputs of level k (FastApriori._trim_worth_it)."""
        Pm = ops.primitives
        m0 = k - 1
        # prefixes past 12 ids ride in gpre (levels.hip); a bundle needing more than this
        # room is planned by dl_plan with the exact size instead
        gpre_n = n_bound * m0 if m0 > 12 else (c_bound * (m0 + 4) if m0 + Pm.DL_MAX_LEVELS > 12 else 0)
        b = S.post_buffers(F1, c_bound, n_bound + c_bound, min(gpre_n, 1 << 24))
        P = S.post
        P.item_map, P.rec, P.part, P.out = (b["item_map"].data_ptr(), b["rec"].data_ptr(), b["part"].data_ptr(),
                                            b["out"].data_ptr())
        P.rec_cap, P.part_cap, P.out_cap = b["c_cap"], b["part"].numel(), b["c_cap"]
        P.gpre, P.gpre_cap = b["gpre"].data_ptr(), b["gpre"].numel()
        # counted rows: all of the rank's rows (candidate mode: the whole DB, this rank's
        # piece chunks, _piece_part); every rank takes the same trimming decision
        v = self._count_view(db)
        P.roff, P.ranks = v["roff"].data_ptr(), v["ranks"].data_ptr()
        P.src = v["src"].data_ptr() if v["src"] is not None else None
        P.wword = v["wword"].data_ptr() if v["wword"] is not None else None
        P.ncols, P.lds_kernel, P.lds_budget = int(v["ncols"]), float(TUNING.slab_lds_bytes), float(lds)
        P.accb = self._dl_accb
        c1 = np.ascontiguousarray(db["c1"], dtype=np.int64)
        alive = np.ascontiguousarray(db["alive"], dtype=np.uint8)
        hist = db.get("len_hist")
        hist = np.ascontiguousarray(hist, dtype=np.int64) if hist is not None and hist.size == 256 else None
        S.post_keep = (c1, alive, hist)                # alive while the native call reads them
        P.c1, P.alive = c1.ctypes.data, alive.ctypes.data
        P.len_hist = hist.ctypes.data if hist is not None else None
        P.T, P.nnz = int(db["T"]), int(db["ranks"].numel())
        P.trim_min_rows, P.trim_ok, P.k = int(self.cfg.trim_min_rows), int(bool(self.cfg.trim) and db["T"] > 0), k
        P.trim_rows_frac, P.trim_nnz_frac = float(TUNING.trim_rows_frac), float(TUNING.trim_nnz_frac)

    def _dl_stage(self, S, pend: list) -> None:
        """Queue the D2H copies of the results not staged yet (F_2 once, then each new
        bundle's rows and counts) into pinned buffers, on a copy stream that waits for
        the compute stream's work so far: the copies overlap the next bundles' kernels,
        and every bundle's results cross PCIe once.  (Copying all results so far again
        at every bundle, on the compute stream, cost T40I10D100M ~10 ms per run.)"""
        Pm = ops.primitives
        stg = self._dl_stg
        todo = []
        if self._f2_n_dev is not None and stg["f2"] is None:
            nb = self._f2_bound
            stg["f2"] = [None] * 3
            todo += [("f2", 0, self._f2_n_dev.view(torch.int32)), ("f2", 1, self._f2_dev[:nb].reshape(-1)),
                     ("f2", 2, self._f2_cnt_dev[:nb])]
        for i in range(stg["n"], len(pend)):
            todo += [("rows", i, pend[i]["rows"]), ("cnt", i, pend[i]["cnt"])]
            stg["rows"].append(None)
            stg["cnt"].append(None)
        first, stg["n"] = stg["n"], len(pend)
        if not todo:
            return
        dev = self._dev
        cs = stg.get("stream")
        if cs is None:
            cs = stg["stream"] = self._dl_stage_stream = torch.cuda.Stream(dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        ckpt = self.ckpt is not None and self._ckpt_deferred
        with torch.cuda.stream(cs):
            for kind, i, t in todo:
                h = Pm.pinned_stage(f"dl_{kind}{i}").get(4 * t.numel()).view(torch.int32)
                h.copy_(t, non_blocking=True)
                stg[kind][i] = h
            if ckpt:
                # the F sizes of every level thresholded so far, for the checkpoint thread
                fsz_h = Pm.pinned_stage(f"dl_fsz{len(pend)}").get(8 * S.fsz.numel()).view(torch.int64)
                fsz_h.copy_(S.fsz, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cs)
        stg["ev"] = ev
        if ckpt:
            self._ckpt_staged(pend, first, todo[0][0] == "f2", fsz_h, ev)

    def _dl_decode_f2(self, n2_h, rows_h, cnt_h):
        n2 = int(n2_h.numpy()[:2].view(np.int64)[0])
        return rows_h.numpy()[:2 * n2].reshape(n2, 2), cnt_h.numpy()[:n2]

    @staticmethod
    def _dl_decode(p: dict, rows_h: np.ndarray, cnt_h: np.ndarray, fsz: np.ndarray) -> list:
        """(k, rows [F_k, k], int32 counts [F_k]) of every level of staged bundle p (views)."""
        out = []
        for l in range(p["L"]):
            kk, w = p["k"] + l, p["m0"] + l + 1
            F = int(fsz[kk])
            a, b = int(p["ro"][l]), int(p["co"][l])
            out.append((kk, rows_h[a:a + F * w].reshape(F, w), cnt_h[b:b + F]))
        return out

    def _ckpt_staged(self, pend: list, first: int, with_f2: bool, fsz_h, ev) -> None:
        """Checkpoint the device loop's levels as their staged copies land:
        the checkpoint thread waits for the copy stream's event, decodes F_2 (when it
        is in this batch) and bundles pend[first:], and writes their level files and
        one meta.json -- so a crash inside the device loop leaves every level up to the
        last staged bundle.  FA_FAULT_AT_LEVEL at one of these levels: the levels up to
        it are written, then this rank exits (at this bundle boundary, not at the end)."""
        ck, result, stg = self.ckpt, self._result, self._dl_stg
        ks = ([2] if with_f2 else []) + [p["k"] + l for p in pend[first:] for l in range(p["L"])]
        if not ks:
            return
        fault = ck.fault_level(self.comm.rank)
        upto = fault if fault in ks else ks[-1]
        f2 = stg["f2"] if with_f2 else None
        bufs = [(p, stg["rows"][i], stg["cnt"][i]) for i, p in enumerate(pend[first:], first)]

        def work():
            ev.synchronize()
            fsz = fsz_h.numpy()
            lv = []
            if f2 is not None:
                lv.append((2,) + self._dl_decode_f2(*f2))
            for p, rh, ch in bufs:
                lv += self._dl_decode(p, rh.numpy(), ch.numpy(), fsz)
            for k, rows, cnt in lv:
                if k <= upto:
                    ck._write_level(result, k, meta=False, rows=np.ascontiguousarray(rows, np.int32),
                                    counts=cnt.astype(np.int64))
            ck._write_meta(result, upto)

        if ck.rank == 0:
            # (every rank holds the same levels; only rank 0 writes them)
            ck.submit(work)
        self._ckpt_saved = max(self._ckpt_saved, upto)
        if fault in ks:
            ck.wait()
            from ..utils.checkpoint import InjectedFault
            raise InjectedFault(17)

    def _dl_flush(self, S, pend: list, levels: list, counts: list, result: MiningResult) -> None:
        """Every device level to the host (the run's one results readback); F_2 too when
        it stayed on the device (_pairs with _f2_defer).  When the last bundle's
        synchronisation already covered a copy of all of them (_dl_stage), that copy."""
        f2 = self._f2_n_dev is not None
        if not pend and not f2:
            return
        # the staged copies (_dl_stage) of whatever is not staged yet, then the F sizes
        self._dl_stage(S, pend)
        stg = self._dl_stg
        fsz = S.fsz.cpu().numpy()                        # (the stream's last work: the thresholds)
        stg["ev"].synchronize()
        if f2:
            r2, c2 = self._dl_decode_f2(*stg["f2"])
            levels[1] = r2.copy()                                    # (pinned buffer: reused)
            counts[1] = c2.astype(np.int64)
            self._log_level2(len(c2))
            self._f2_n_dev = None
        if not pend:
            return
        for i, p in enumerate(pend):
            for l, (kk, rows, cnt) in enumerate(self._dl_decode(p, stg["rows"][i].numpy(), stg["cnt"][i].numpy(),
                                                                fsz)):
                F = len(cnt)
                levels.append(rows.copy())
                counts.append(cnt.astype(np.int64))
                # the reference logs the groups generated from F_{k-1}; a bundled level
                # counted a superset generated from C_{k-1}.  One launch counts the whole
                # bundle: a level's time, device time and streamed bytes are its
                # candidates' share of the bundle's
                share = float(p["C"][l]) / max(float(p["C"].sum()), 1.0)
                groups = (lambda kk=kk: int(apriori_gen(levels[kk - 2])[0].size)) if kk > p["k"] else int(p["G"][l])
                self._log_level(levels, kk, groups, F, p["ms"] * share)
                m = p["m0"] + l              # parent row length of level kk
                hbm = int(share * p["hbm_rows"] + 4 * int(p["n_par"][l]) * m
                          + 4 * int(p["C"][l]) * (m + 1) + 3 * 4 * int(p["C"][l]))
                self._level_recs.append((dict(phase="level", k=kk, candidates=int(p["C"][l]), frequent=F,
                                              ms=p["ms"] * share, groups=int(p["G"][l]), bundled_with=p["k"],
                                              bytes_reduced=int(p["bytes"] * share), kernel="slab_rec_dev",
                                              hbm_bytes_est=hbm, slab_words=p["sw"], used_items=p["used"],
                                              rows=p["T"], _share=share),
                                         f"level{p['k']}"))

    def _run_deferred(self) -> None:
        for d in self._deferred:
            d.result()
        self._deferred = []

    @staticmethod
    def _result_items(result: MiningResult, wait: bool = True) -> None:
        """Numeric-mode tokens are formatted while the pair kernel runs (the order is
        already fixed); this puts the finished list into the result."""
        if wait and not isinstance(result.items, list):
            result.items = result.items.result()

    def _bytes_moved(self) -> int:
        b = self.comm.bytes_reduced
        if getattr(self, "dcomm", self.comm) is not self.comm:
            b += self.dcomm.bytes_reduced
        return b

    @staticmethod
    def _level_hbm_bytes(db, plan: dict) -> int:
        """HBM bytes a level's count kernel reads (estimate from its plan): every pass
        rebuilds the slabs from the compressed rows (ranks + row offsets), or copies
        the materialised bitmap of the used items."""
        if not plan:
            return 0
        passes = int(plan.get("passes", 1) or 1)
        rows = int(db["ranks"].numel()) * 4 + int(db["roff"].numel()) * 8
        return passes * rows

    def _emit_level_metrics(self) -> None:
        tm = getattr(self, "_timer", None)
        gpu = tm.finish() if (tm is not None and tm.events) else {}
        if tm is not None and tm.events:
            self.stats["gpu_phase_ms"] = {k: round(v, 3) for k, v in gpu.items()}
        for rec, span in getattr(self, "_level_recs", []):
            share = rec.pop("_share", 1.0)
            if span is not None and span in gpu:
                rec["gpu_ms"] = round(gpu[span] * share, 3)
            self.log.metric(**rec)
        self._level_recs = []
        if self.cfg.trace and tm is not None:
            self.stats["trace"] = tm.trace(pid=self.comm.rank)

    def _finish(self, result: MiningResult, t_start: float) -> MiningResult:
        self._result_items(result)
        if getattr(self, "_ckpt_deferred", False):
            # the levels not handed over yet (none after the device loop), written by the
            # background thread while the caller writes the outputs (Checkpointer.wait /
            # mark_complete join it)
            self._ckpt_upto(result, len(result.levels), background=True)
        db = getattr(self, "_db_local", None)
        if db is not None:
            sizes = getattr(self, "_layout_sizes", None)
            if sizes is None:
                # layout sizes for the metrics (deduplicated layouts), one collective after the last level
                g = self.dcomm.all_gather_ints([db["T0"], db["ncols0"]])
                sizes = int(g[:, 0].sum()), int(g[:, 1].sum())
            self.stats.update(T=sizes[0], distinct=sizes[1])
            self._db_local = None
        if len(result.levels) >= 2:
            self._log_tail(result.levels)
        total_k2 = sum(len(c) for c in result.counts[1:])
        self.log.line(f"Total freq items sets {total_k2}")
        self.stats["mine_ms"] = (time.perf_counter() - t_start) * 1e3
        self.stats["n_itemsets"] = result.n_itemsets
        self.stats["bytes_reduced"] = self.comm.bytes_reduced
        if ops.primitives.FALLBACKS:
            self.stats["fallbacks"] = list(ops.primitives.FALLBACKS)
            for f in ops.primitives.FALLBACKS:
                self.log.metric(phase="fallback", what=f)
        self._emit_level_metrics()
        if getattr(self, "_timer", None) is not None and self._timer.sync:
            self.stats["phase_ms"] = {k: round(v, 3) for k, v in self._timer.t.items()}
        return result

    def _check_resume(self, resume: MiningResult, fresh: MiningResult) -> None:
        if resume.items != fresh.items or not np.array_equal(resume.counts[0], fresh.counts[0]):
            raise ValueError("checkpoint does not match the input data (different F1)")

    # ------------------------------------------------------------------
    # F1: histogram, all-reduce, ranking (FastApriori.scala:46-62)
    # ------------------------------------------------------------------
    def _frequent_items(self, shard: TransactionShard, mc: int):
        comm, vocab, dev = self.dcomm, shard.vocab, shard.items.device
        thr = max(mc, 1)   # only tokens that occur can be frequent (even at minSupport 0)
        if vocab.numeric:
            V = self._V_max
            got = None
            if self.cfg.f1 == "sketch" or (self.cfg.f1 == "auto" and dev.type == "cuda"
                                              and V >= F1_SKETCH_MIN_VOCAB):
                got = self._f1_heavy_hitters(shard, V, thr)
            if got is None:
                hist = self._parsed_hist(shard, V)
                if hist is None:
                    hist = ops.histogram(shard.items, V)
                    if shard.extras.size:
                        hist += torch.bincount(torch.from_numpy(shard.extras.astype(np.int64)), minlength=V).to(dev)
                comm.all_reduce_(hist)
                if (dev.type == "cuda" and TUNING.f1_rank_device and 2 <= V <= ops.primitives.F1_RANK_DEVICE_MAX
                        and self.cfg.tiebreak in ("string", "numeric")):
                    # narrow vocabulary: ranked on the device (prep.hip k_f1_rank); the LUT is
                    # there at once and the ranking comes back while compression runs (_run)
                    self._f1_pending = ops.primitives.f1_rank_start(hist, thr, self.cfg.tiebreak == "numeric")
                    return None, None, self._f1_pending.lut
                if V <= F1_HIST_READBACK and dev.type == "cuda" and self.cfg.tiebreak == "string":
                    # narrow vocabulary: the whole histogram in one readback (no nonzero sync),
                    # ranked and mapped to the LUT in one native call (csrc/host/f1.cpp)
                    hh = np.ascontiguousarray(hist.cpu().numpy(), dtype=np.int64)
                    Vh = max(V, 1)
                    st = ops.primitives.pinned_stage("f1_lut")
                    buf = st.get(4 * Vh)
                    ids = np.empty(Vh, np.int64)
                    cnt = np.empty(Vh, np.int64)
                    F = int(ops._native.host().fa_f1_rank_numeric(hh.ctypes.data, V, thr, ids.ctypes.data,
                                                                   cnt.ctypes.data, buf.data_ptr()))
                    if V == 0:
                        buf.view(torch.int32)[0] = -1      # the native call writes lut[0 .. V) only
                    lut = buf.to(dev, non_blocking=True).view(torch.int32)
                    st.event = torch.cuda.Event()
                    st.event.record()
                    ids = ids[:F]
                    items = _Deferred(lambda: ["" if i == 0 else str(i - 1) for i in ids.tolist()])
                    self._deferred.append(items)
                    return items, cnt[:F].copy(), lut
                if V <= F1_HIST_READBACK:
                    # narrow vocabulary: the whole histogram in one readback (no nonzero sync)
                    hh = hist.cpu().numpy()
                    fid = np.flatnonzero(hh >= thr)
                    got = fid, hh[fid]
                else:
                    fid = torch.nonzero(hist >= thr).flatten()
                    h = torch.stack([fid, hist[fid].to(torch.int64)]).cpu().numpy()     # one readback
                    got = h[0], h[1]
            fid, fcnt = got
            # numeric tokens are ASCII decimal strings, and Java String order of decimals
            # is the order of (digits left-aligned to 10 places, then length): ties of
            # equal counts sort without building strings ("" = id 0 sorts first)
            fid = np.asarray(fid, dtype=np.int64)
            if self.cfg.tiebreak == "numeric":
                # integer value (id - 1), the empty token (id 0) after every integer
                key = np.where(fid == 0, np.iinfo(np.int64).max, fid - 1)
                order = np.lexsort((key, -np.asarray(fcnt, dtype=np.int64))) if fid.size else np.zeros(0, np.int64)
            else:
                v = fid - 1
                d = np.searchsorted(_POW10, v, side="right") + 1
                key = v * _POW10_PAD[d]
                key[fid == 0], d[fid == 0] = -1, 0
                order = (np.lexsort((d, key, -np.asarray(fcnt, dtype=np.int64))) if fid.size
                         else np.zeros(0, np.int64))
            ids = fid[order]
            items = _Deferred(lambda: ["" if i == 0 else str(i - 1) for i in ids.tolist()])
            self._deferred.append(items)
            counts1 = np.asarray(fcnt)[order].astype(np.int64)
            if V <= F1_HIST_READBACK and dev.type == "cuda":
                # the id -> rank LUT built on the host, one asynchronous copy
                lut_h = np.full(max(V, 1), -1, dtype=np.int32)
                lut_h[ids] = np.arange(len(order), dtype=np.int32)
                return items, counts1, ops.primitives.pinned_stage("f1_lut").h2d(lut_h, dev)
            lut = torch.full((max(V, 1),), -1, dtype=torch.int32, device=dev)
            if len(order):
                lut[torch.from_numpy(fid[order].astype(np.int64)).to(dev)] = torch.arange(
                    len(order), dtype=torch.int32, device=dev)
            return items, counts1, lut
        # dictionary mode: agree on identity through 64-bit token hashes.  Everything
        # over the vocabulary runs as tensor ops on the shard's device (a webdocs-scale
        # shard has ~5M distinct strings); only the frequent items' strings are ever
        # decoded.  Both parsers give every distinct token of a shard a distinct hash
        # (a 64-bit collision is a parse error), so hashes identify ids.
        Vl = vocab.size
        hist = ops.histogram(shard.items, max(Vl, 1))[:Vl].to(torch.int64)
        if shard.extras.size:
            hist += torch.bincount(torch.from_numpy(shard.extras.astype(np.int64)), minlength=Vl)[:Vl].to(dev)
        hashes_t = torch.from_numpy(vocab.hashes.astype(np.uint64).view(np.int64)).to(dev)
        if comm.distributed:
            # hash-partitioned counting (the reference's HashPartitioner shuffle,
            # FastApriori.scala:55-58): owner = (hash >> 1) mod world
            W = comm.world_size
            owner = torch.remainder(torch.bitwise_right_shift(hashes_t, 1) & ((1 << 62) - 1), W)
            by_owner = torch.argsort(owner, stable=True)
            bounds = torch.searchsorted(owner[by_owner], torch.arange(W + 1, device=dev)).cpu().numpy()
            sh_np = hashes_t[by_owner].cpu().numpy()
            sc_np = hist[by_owner].cpu().numpy()
            send_h = [sh_np[bounds[r]:bounds[r + 1]] for r in range(W)]
            send_c = [sc_np[bounds[r]:bounds[r + 1]] for r in range(W)]
            rh = np.concatenate(comm.all_to_all_varlen(send_h))
            rc = np.concatenate(comm.all_to_all_varlen(send_c))
            uh, inv = np.unique(rh, return_inverse=True)
            tot = np.bincount(inv, weights=rc, minlength=uh.size).astype(np.int64)
            ok = tot >= thr
            parts = comm.all_gather_varlen_np(np.stack([uh[ok], tot[ok]]).ravel())
            fh = np.concatenate([q.reshape(2, -1)[0] for q in parts])
            fc = np.concatenate([q.reshape(2, -1)[1] for q in parts])
            # strings of the frequent tokens this shard has; every rank contributes its own
            hs_sorted, hs_order = torch.sort(hashes_t)
            fh_t = torch.from_numpy(fh).to(dev)
            pos = torch.clamp(torch.searchsorted(hs_sorted, fh_t), max=max(Vl - 1, 0))
            have = (hs_sorted[pos] == fh_t) if Vl else torch.zeros(fh_t.numel(), dtype=torch.bool, device=dev)
            loc = hs_order[pos[have]].cpu().numpy()
            have = have.cpu().numpy()
            mine = vocab.decode(loc) if loc.size else []
            allstrs = {}
            for hs, ss in comm.all_gather_object((fh[have].tolist(), mine)):
                allstrs.update(zip(hs, ss))
            fstr = [allstrs[h] for h in fh.tolist()]
        else:
            sel = torch.nonzero(hist >= thr).flatten()
            got = torch.stack([sel, hashes_t[sel], hist[sel]]).cpu().numpy()
            sel_np, fh, fc = got[0], got[1], got[2]
            fstr = vocab.decode(sel_np)
        tb = self.cfg.tiebreak
        order = sorted(range(len(fstr)), key=lambda e: (-int(fc[e]), item_tiebreak_key(fstr[e], tb)))
        items = [fstr[e] for e in order]
        self._item_hashes = np.asarray(fh, dtype=np.int64)[order].view(np.uint64) if order else \
            np.zeros(0, np.uint64)
        counts1 = np.asarray(fc, dtype=np.int64)[order] if order else np.zeros(0, np.int64)
        lut = torch.full((max(Vl, 1),), -1, dtype=torch.int32, device=dev)
        if order and Vl:
            rank_h = torch.from_numpy(np.asarray(fh, dtype=np.int64)[order]).to(dev)
            rs, ro = torch.sort(rank_h)
            pos = torch.clamp(torch.searchsorted(rs, hashes_t), max=rank_h.numel() - 1)
            hit = rs[pos] == hashes_t
            lut[:Vl][hit] = ro[pos[hit]].to(torch.int32)
        return items, counts1, lut

    @staticmethod
    def _parsed_hist(shard: TransactionShard, V: int):
        """The occurrence histogram the device parser counted while compacting the ids
        (csrc/hip/parse.hip k_tcompact), widened to the ranks' common V; None when
        the shard has none (then F1 reads the items)."""
        h = shard.hist
        if h is None or h.device != shard.items.device or h.numel() > V:
            return None
        out = torch.zeros(V, dtype=torch.int64, device=h.device)
        out[:h.numel()] = h
        return out

    def _f1_heavy_hitters(self, shard: TransactionShard, V: int, thr: int):
        """Numeric-mode F1 for wide vocabularies without a V-bin histogram.

        A count-min sketch never under-estimates, so every id with support >=
        thr is a candidate; exact counts of the candidates then decide.  The
        sketch (2 x 16K int64) and the candidate counts are the only all-reduces
        (instead of V int64).  Returns None (-> plain histogram) when the sketch
        is too crowded to leave at most ops.F1_MAX_CANDIDATES candidates; the
        decision is identical on every rank since the reduced sketch is."""
        comm, dev = self.dcomm, shard.items.device
        sk = ops.f1_sketch(shard.items)
        ex = torch.from_numpy(shard.extras.astype(np.int64)) if shard.extras.size else None
        if ex is not None:
            sk += ops.f1_sketch(ex).to(dev)
        comm.all_reduce_(sk)
        cand = torch.nonzero(ops.sketch_estimate(sk, torch.arange(V, device=dev)) >= thr).flatten()
        if cand.numel() > F1_MAX_CANDIDATES:
            return None
        cnt = ops.f1_exact(shard.items, cand)
        if ex is not None:
            cnt += ops.f1_exact(ex, cand.cpu()).to(dev)
        comm.all_reduce_(cnt)
        keep = cnt >= thr
        return cand[keep].cpu().numpy(), cnt[keep].cpu().numpy()

    # ------------------------------------------------------------------
    # Compression (FastApriori.scala:66-79) and the vertical layout
    # ------------------------------------------------------------------
    def _compress_start(self, shard: TransactionShard, lut: torch.Tensor, F1: int):
        """Queue the fused two-pass compression (ops.primitives.compress_rows_start) when
        it applies; _compress finishes it.  None: _compress runs the general path."""
        dev = shard.items.device
        n_rows = shard.offsets.numel() - 1
        if (dev.type == "cuda" and n_rows > 0 and TUNING.fused_compress
                and shard.items.numel() <= TUNING.fused_compress_mean_len * n_rows):
            # the dedup estimate's probe rides along with the compression sizes (one readback)
            self._dedup_probe = {} if self.cfg.dedup == "auto" else None
            return ops.primitives.compress_rows_start(shard.offsets, shard.items, lut, F1, probe=self._dedup_probe)
        return None

    def _compress(self, shard: TransactionShard, lut: torch.Tensor, F1: int, pending=None) -> dict:
        dev = shard.items.device
        if pending is not None:
            # fused two-pass path: kept rows, offsets, sorted ranks and the length histogram
            # (started before F1 was known when F1 was ranked on the device: its block
            # layout then has ceil(V / 256) blocks, the ones past F1's empty)
            pending["F1"] = F1
            kept, roff, ranks, hist_t, bcnt = ops.primitives.compress_rows_finish(pending)
            T = kept.numel()
            hist = np.asarray(hist_t, dtype=np.int64).copy()
        else:
            self._dedup_probe = None
            cnt = ops.txn_freq_count(shard.offsets, shard.items, lut)
            kept = torch.nonzero(cnt >= 2).flatten().to(torch.int32)
            T = kept.numel()
            roff = torch.zeros(T + 1, dtype=torch.int64, device=dev)
            if T:
                torch.cumsum(cnt[kept.to(torch.int64)].to(torch.int64), 0, out=roff[1:])
            ranks = ops.compress(shard.offsets, shard.items, lut, kept, roff, F1)
            hist = ops.histogram(torch.clamp(cnt, max=255), 256).cpu().numpy() if cnt.numel() else np.zeros(256, np.int64)
            bcnt = None
        db = {"roff": roff, "ranks": ranks, "T": T, "src": None, "ncols": T, "wword": None, "wrow": None,
              "bm": None, "W": 0, "F1": F1, "alive": np.ones(F1, dtype=bool), "c1": self._counts1,
              "bcnt": bcnt}      # 256-item block counts of these rows (pair layout); dropped on re-layout
        # row-length histogram (lengths >= 255 share the last bin): drives the pair
        # cost model, the trimming model and the u8 per-block count guard
        hist[:2] = 0                         # rows with < 2 frequent items are not kept
        L = np.arange(256, dtype=np.int64)
        db["pair_work"] = int((hist * (L * (L - 1) // 2)).sum())
        db["len_hist"] = hist
        # every rank must take the same layout decisions: long rows, dedup and (when the
        # layout stays undeduplicated) the pair strategy, agreed in one collective
        # (the kept rows ride along: without dedup they are also the layout's columns,
        # the run's T / distinct metrics, and _finish needs no collective of its own)
        g = self.dcomm.all_gather_ints([int(hist[255] > 0), int(self._want_dedup(db)),
                                        int(self._pick_gram_local(db, F1)), db["pair_work"], T])
        db["long_rows"] = bool(g[:, 0].max())
        db["pair_work_all"] = int(g[:, 3].sum())      # pair increments of every rank (bounds |F_2|)
        db["pair_pick"] = None
        self._layout_sizes = None if g[:, 1].max() else (int(g[:, 4].sum()),) * 2
        if g[:, 1].max():
            db["bcnt"] = None
            self._dedup(db)
            db.pop("len_hist", None)
        else:
            db["pair_pick"] = bool(g[:, 2].max())
        db["T0"] = T
        db["ncols0"] = db["ncols"] if db["src"] is None else db["n_distinct"]
        self.log.metric(phase="compress", T=T, distinct=db.get("n_distinct", T), nnz=int(ranks.numel()))
        return db

    def _want_dedup(self, db) -> bool:
        mode = self.cfg.dedup
        if mode == "off" or db["T"] < 2:
            decision = False
        elif mode == "on":
            decision = True
        else:
            # estimate the distinct fraction on a prefix sample of the rows: linear
            # counting (occupied slots of a 4M-slot bitmap of the row hashes: one
            # scatter + one sum, instead of sorting the sample)
            m = 1 << 22
            probe = getattr(self, "_dedup_probe", None)
            if probe and probe.get("n"):
                n, filled = probe["n"], probe["filled"]      # computed with the compression (device)
            else:
                n = min(db["T"], ops.primitives.DEDUP_PROBE_ROWS)
                h1, _ = ops.row_hash(db["roff"][: n + 1], db["ranks"])
                occ = torch.zeros(m, dtype=torch.uint8, device=h1.device)
                occ[h1 & (m - 1)] = 1
                filled = int(occ.sum().item())
            est = -m * math.log(max(1.0 - filled / m, 1.0 / m))
            frac = est / max(n, 1)
            decision = frac < self.cfg.dedup_threshold
        # local decision: the caller agrees on it across ranks (the layout differs)
        return decision

    def _dedup(self, db) -> None:
        """Merge identical compressed rows into weight classes (FastApriori.scala:71-79).

        Columns are ordered by weight (unit weight first) and every class is padded
        to a multiple of 64 columns, so each bitmap word carries exactly one weight.
        """
        roff, ranks, T = db["roff"], db["ranks"], db["T"]
        dev = ranks.device
        if T == 0:
            # a shard without kept rows still takes the agreed (weighted) layout
            db.update(wrow=torch.zeros(0, dtype=torch.int32, device=dev), n_distinct=0)
            self._layout_weighted(db)
            return
        h1, h2 = ops.row_hash(roff, ranks)
        o = torch.argsort(h2, stable=True)
        o = o[torch.argsort(h1[o], stable=True)]
        a1, a2 = h1[o], h2[o]
        new = torch.ones(T, dtype=torch.bool, device=dev)
        new[1:] = (a1[1:] != a1[:-1]) | (a2[1:] != a2[:-1])
        run = torch.cumsum(new.to(torch.int64), 0) - 1
        nd = int(run[-1].item()) + 1
        weight = torch.bincount(run, minlength=nd)
        rep = o[new]                                   # one representative kept row per run
        wrow = torch.zeros(T, dtype=torch.int32, device=dev)
        wrow[rep] = weight.to(torch.int32)
        db.update(wrow=wrow, n_distinct=nd)
        self._layout_weighted(db)

    @staticmethod
    def _layout_weighted(db) -> None:
        """Columns = rows with weight > 0, grouped by weight (unit weight first), each
        class padded to 64 so every bitmap word carries one weight."""
        wrow = db["wrow"]
        dev = wrow.device
        rep = torch.nonzero(wrow > 0).flatten()
        weight = wrow[rep].to(torch.int64)
        nd = rep.numel()
        if nd == 0:
            db.update(src=torch.full((64,), -1, dtype=torch.int32, device=dev), ncols=64,
                      wword=torch.ones(1, dtype=torch.int32, device=dev),
                      wcls=(np.ones(1, np.int64), np.ones(1, np.int64)))
            return
        wo = torch.argsort(weight, stable=True)
        w_sorted, rep_sorted = weight[wo], rep[wo]
        cls_w, cls_n = torch.unique_consecutive(w_sorted, return_counts=True)
        padded = (cls_n + 63) // 64 * 64
        cls_col0 = torch.cumsum(padded, 0) - padded
        cls_first = torch.cumsum(cls_n, 0) - cls_n
        cls_of = torch.repeat_interleave(torch.arange(cls_n.numel(), device=dev), cls_n)
        col = cls_col0[cls_of] + (torch.arange(nd, device=dev) - cls_first[cls_of])
        # the weight classes on the host (one readback): (weight, words) per class, the
        # matrix-core Gram's launch list (ops.primitives.gram_segments)
        wcls = torch.stack([cls_w.to(torch.int64), padded // 64]).cpu().numpy()
        ncols = int(wcls[1].sum()) * 64
        src = torch.full((ncols,), -1, dtype=torch.int32, device=dev)
        src[col] = rep_sorted.to(torch.int32)
        wword = torch.repeat_interleave(cls_w.to(torch.int32), padded // 64)
        db.update(src=src, ncols=ncols, wword=wword, wcls=(wcls[0], wcls[1]))

    def _trim_worth_it(self, db, used: np.ndarray, k: int, C: int = 0) -> bool:
        """Binomial estimate of the rows that would survive trimming.

        Item occurrences survive with probability p = (occurrences of the level's
        candidate items) / (occurrences of the items still in the rows); a row of
        length L keeps >= k of them with probability P[Binom(L, p) >= k].  Trimming
        costs two passes over the rows (and a rebuild of the bitmaps), so it runs
        only when it removes a lot.  A level of C candidates that needs several
        accumulator passes streams its slabs from the used items' bitmap, whose size
        depends on the rows only: then dropped items do not count.
        """
        if db["T"] < self.cfg.trim_min_rows:   # a trim's fixed cost (2 launches + a host sync) dominates
            return False
        got = self._trim_estimate(db, used, k, with_nnz=True)
        if got is None:
            return False
        est_rows, est_nnz = got
        rows_ok = est_rows < TUNING.trim_rows_frac * max(db["T"], 1)
        if C and db["ranks"].is_cuda and C > ops.primitives.slab_capacity(int(used.size), C):
            return rows_ok
        return rows_ok or est_nnz < TUNING.trim_nnz_frac * max(int(db["ranks"].numel()), 1)

    def _len_hist(self, db) -> np.ndarray:
        lens = db["roff"][1:] - db["roff"][:-1]
        return torch.bincount(lens).cpu().numpy() if lens.numel() else np.zeros(1, np.int64)

    def _trim(self, db, used: np.ndarray, k: int, C: int = 0, decided: bool = False) -> None:
        """Transaction trimming before level k (items outside C_k, rows with < k of them).
        decided: the estimate already said yes (fa_hip_dl_more's post step)."""
        if not self.cfg.trim or db["T"] == 0:
            return
        if "len_hist" not in db:
            db["len_hist"] = self._len_hist(db)
        if not decided and not self._trim_worth_it(db, used, k, C):
            return
        dev = db["ranks"].device
        alive = torch.zeros(db["F1"], dtype=torch.int8)
        alive[torch.from_numpy(used.astype(np.int64))] = 1
        kept, nroff, nranks, nw, hist = ops.trim_rows(db["roff"], db["ranks"], alive.to(dev), k, db["wrow"])
        K = kept.numel()
        # a level counted window by window streams its slabs from the used items' bitmap,
        # whose cost follows the rows only: fewer items alone do not pay for a new layout
        # (and the bitmap rebuild it forces)
        multi = bool(C) and db["ranks"].is_cuda and C > ops.primitives.slab_capacity(int(used.size), C)
        if K > 0.9 * db["T"] and (multi or nranks.numel() > 0.9 * db["ranks"].numel()):
            return   # not worth re-laying out
        db.update(roff=nroff, ranks=nranks, T=K, bm=None, W=0, bcnt=None, bm_items=None, bm_map=None)
        db["alive"] = np.zeros_like(db["alive"])
        db["alive"][used] = True
        db["len_hist"] = hist.cpu().numpy()
        if db["wrow"] is not None:
            db["wrow"] = nw
            self._layout_weighted(db)
        else:
            db.update(src=None, ncols=K)
        self.log.metric(phase="trim", k=k, rows=K, nnz=int(nranks.numel()))

    def _bitmaps(self, db, used: np.ndarray | None = None, blocked: bool = False):
        """Item-major bitmaps for the current row layout (built once, reused by the Gram
        pair kernel and every multi-pass level until a trim).

        used=None: every item's row, rank-indexed.  used (sorted ranks): only those rows
        -- a multi-pass level's items, which contain every later level's items (level
        k+1's candidates are built from F_k, whose items are level-k candidate items),
        so the rows of the next levels are a subset until the layout changes.  Returns
        (bm, bm_map): bm_map is the device rank -> bitmap row map, or None when the
        bitmap is rank-indexed.  blocked: the caller reads either layout (the Gram and
        the slab kernels' bitmap copies), and a full bitmap is built in 8-word blocks
        where the wave build applies (ops.build_bitmaps); count_candidates reads the
        row-major one, so a blocked bitmap is rebuilt for it."""
        have, bm = db.get("bm_items"), db["bm"]
        if bm is not None and (bm.dim() == 2 or blocked) and (have is None or (used is not None and have[used].all())):
            return bm, db.get("bm_map")
        with roctx_range("bitmaps"):
            if used is None:
                blk = (blocked and TUNING.bitmap_blocked and db["ranks"].is_cuda
                       and ops.primitives.blocked_bitmaps_ok(db["src"], db["F1"], db["ncols"]))
                bm, W = ops.build_bitmaps(db["roff"], db["ranks"], db["src"], db["ncols"], db["F1"], blocked=blk)
                self.stats["bm_blocked"] = bool(blk)
                db.update(bm=bm, W=W, bm_items=None, bm_map=None)
            else:
                dev = db["ranks"].device
                imap = np.full(max(db["F1"], 1), -1, dtype=np.int32)
                imap[used] = np.arange(used.size, dtype=np.int32)
                items = np.zeros(max(db["F1"], 1), dtype=bool)
                items[used] = True
                imap_t = torch.from_numpy(imap).to(dev)
                bm, W = ops.build_bitmaps(db["roff"], db["ranks"], db["src"], db["ncols"], int(used.size), imap_t,
                                          torch.from_numpy(np.ascontiguousarray(used, dtype=np.int32)).to(dev))
                db.update(bm=bm, W=W, bm_items=items, bm_map=imap_t)
        return db["bm"], db.get("bm_map")

    # ------------------------------------------------------------------
    # k = 2 (FastApriori.scala:212-241)
    # ------------------------------------------------------------------
    def _pick_pair_strategy(self, db, F1: int) -> str:
        s = self.cfg.pair_strategy
        if s != "auto":
            return s
        if db.get("pair_pick") is not None:     # agreed with the compress decisions
            return "gram" if db["pair_pick"] else "horizontal"
        # ranks must agree: any rank preferring the Gram kernel decides
        return "gram" if self.dcomm.allreduce_int(int(self._pick_gram_local(db, F1)), "max") else "horizontal"

    @staticmethod
    def _pick_gram_local(db, F1: int) -> bool:
        W = (db["ncols"] + 63) // 64
        t_h = db["pair_work"] / HORIZONTAL_PAIRS_PER_S
        t_g = (F1 * (F1 - 1) / 2) * W / GRAM_WORDPAIRS_PER_S
        return t_g < t_h

    @staticmethod
    def _slice_classes(wcls, w0: int, w1: int):
        """Weight classes (weights, words) restricted to the word range [w0, w1)."""
        if wcls is None:
            return None
        end = np.cumsum(wcls[1])
        beg = end - wcls[1]
        nw = np.clip(np.minimum(end, w1) - np.maximum(beg, w0), 0, None)
        keep = nw > 0
        return wcls[0][keep], nw[keep]

    def _pairs(self, db, F1: int, mc: int):
        strat = self._pick_pair_strategy(db, F1)
        self.stats["pair_strategy"] = strat
        r, nr = (self.comm.rank, self.comm.world_size) if self.cand_par else (0, 1)
        C2 = F1 * (F1 - 1) // 2
        rs = self.comm.distributed and C2 >= TUNING.pair_rs_min
        # F_2 compacted on the device (no readback before the first device bundle)
        on_dev = self._f2_defer and not rs and db["ranks"].is_cuda
        if strat == "gram":
            self._bitmaps(db, blocked=True)
            # candidate parallelism: each rank takes a 32-word-aligned slice of the columns
            W = db["W"]
            w0, w1 = (W * r // nr) // 32 * 32, (W if r == nr - 1 else (W * (r + 1) // nr) // 32 * 32)
            wword = db["wword"][w0:w1] if db["wword"] is not None else None
            pc = ops.pair_counts_gram(db["bm"], max(w1 - w0, 0), wword,
                                      self._slice_classes(db.get("wcls"), w0, w1), raw=on_dev, w0=w0)
        else:
            roff, ranks, wrow = db["roff"], db["ranks"], db["wrow"]
            if nr > 1:   # candidate parallelism: each rank takes a slice of the rows
                T = db["T"]
                a, b = T * r // nr, T * (r + 1) // nr
                ra, rb = int(roff[a].item()), int(roff[b].item())
                roff, ranks = roff[a:b + 1] - ra, ranks[ra:rb]
                wrow = wrow[a:b] if wrow is not None else None
            pc = ops.pair_counts_horizontal(roff, ranks, wrow, F1, db.get("long_rows", True),
                                            bcnt=db.get("bcnt") if nr == 1 and wrow is None else None, raw=on_dev)
        self._run_deferred()      # host-only work while the pair kernel runs
        T, nnz = int(db["T"]), int(db["ranks"].numel())
        if strat == "gram":
            self.stats["pair_hbm_bytes_est"] = int(F1 * max(db["W"], 1) * 8 * ((F1 + 63) // 64))
        else:
            nb = (F1 + 255) // 256
            self.stats["pair_hbm_bytes_est"] = int(2 * (4 * nnz + 8 * T) + nnz * (nb + 1) + T * nb * (nb + 1))
        if on_dev:
            return self._pairs_on_device(pc, mc, db)
        iu, fi = self._triu(F1, pc.device)
        flat = pc.reshape(-1)[fi]
        if rs:
            # X12 as reduce-scatter + local threshold + all-gather of the survivors
            # (F_2 << C_2): each rank thresholds its 1/world slice of the summed triangle
            keep, vals = self.comm.reduce_scatter_select(flat, mc, bound=self.stats["n_lines"])
        else:
            self.comm.all_reduce_(flat, bound=self.stats["n_lines"])
            keep = torch.nonzero(flat >= mc).flatten()
            vals = flat[keep]
        # one readback: rows (a, b) and counts
        keep = keep.to(iu.device)
        if iu.is_cuda and TUNING.device_levels:
            # F_2 rows stay on the device as the first device bundle's input
            self._f2_dev = torch.stack([iu[0][keep], iu[1][keep]], 1).to(torch.int32).contiguous()
        h = torch.stack([iu[0][keep], iu[1][keep], vals.to(device=iu.device, dtype=torch.int64)]).cpu().numpy()
        return np.ascontiguousarray(h[:2].T, dtype=np.int32), h[2].astype(np.int64)

    @staticmethod
    def _triu(F1: int, dev):
        """Upper-triangle positions of the F1 x F1 pair matrix and their flat offsets."""
        key = (F1, dev)
        if key not in _TRIU_CACHE:
            _TRIU_CACHE.clear()
            iu = torch.triu_indices(F1, F1, 1, device=dev)
            _TRIU_CACHE[key] = (iu, iu[0] * F1 + iu[1])
        return _TRIU_CACHE[key]

    def _pairs_on_device(self, pc: torch.Tensor, mc: int, db):
        """F_2 = pairs with count >= mc (FastApriori.scala:236-238), compacted on the
        device in pair order with no host synchronisation (count.hip
        fa_hip_pairs_compact: per-row keep counts, one scan, per-row emit).  pc: the
        pair kernel's raw int32 counts; across ranks its triangle is gathered and
        all-reduced first.  |F_2| stays on the device (the first device bundle reads
        it); the host copy of F_2 arrives with _dl_flush.  The readback bound: every
        frequent pair has count >= mc and the counts sum to the pair increments, so
        |F_2| <= pair increments / mc."""
        F1 = self._F1
        C2 = F1 * (F1 - 1) // 2
        if self.comm.distributed:
            _, fi = self._triu(F1, pc.device)
            flat = pc.reshape(-1)[fi] if pc.is_contiguous() else pc.contiguous().reshape(-1)[fi]
            self.comm.all_reduce_(flat, bound=self.stats["n_lines"])
            rows, cnt, n = ops.primitives.pairs_compact(flat.contiguous(), F1, mc, flat=True)
        else:
            rows, cnt, n = ops.primitives.pairs_compact(pc, F1, mc)
        pw = db.get("pair_work_all")      # exact only without rows of >= 255 items (histogram's last bin)
        exact = pw is not None and not db.get("long_rows", True) and not self.cand_par
        bound = min(C2, int(pw) // mc + 1) if exact and mc > 0 else C2
        self._f2_dev, self._f2_cnt_dev, self._f2_n_dev, self._f2_bound = rows, cnt, n, max(int(bound), 1)
        self.stats["f2_on_device"] = True
        return None, None

    # ------------------------------------------------------------------
    # k >= 3 (FastApriori.scala:132-160)
    # ------------------------------------------------------------------
    def _gen(self, prev: np.ndarray, want_rows: bool = False):
        """apriori-gen (FastApriori.scala:167-193): on the GPU for big levels (host
        call costs ~130 ns per candidate; the device path ~60 us per call), else the
        C++ host path.  Both return identical (prefix_idx, ext_off, ext) [+ the
        candidate rows [C, m+1] when want_rows]."""
        dev = self._dev
        n = prev.shape[0]
        if (dev.type == "cuda" and TUNING.gen_device and n >= TUNING.gen_device_min_rows and prev.shape[1] >= 2
                and self._F1 <= ops.primitives.AG_DEVICE_MAX_F1):
            return ops.apriori_gen_device(prev, self._F1, dev, want_rows)
        if dev.type == "cuda" and self._F1 > ops.primitives.AG_DEVICE_MAX_F1:
            ops.primitives.note_fallback(f"apriori-gen on the host: F1 = {self._F1} frequent items exceed the "
                                         f"device generator's {ops.primitives.AG_DEVICE_MAX_F1}-rank bitsets")
        pi, eo, ex = apriori_gen(prev)
        if not want_rows:
            return pi, eo, ex
        g = np.repeat(np.arange(pi.size), np.diff(eo))
        rows = np.concatenate([prev[pi[g]], ex[:, None]], axis=1) if ex.size else \
            np.zeros((0, prev.shape[1] + 1), np.int32)
        return pi, eo, ex, np.ascontiguousarray(rows, dtype=np.int32)

    def _gen_bundle_fused(self, k: int, prev: np.ndarray):
        """apriori-gen of level k and the speculative bundle levels in ONE native call
        (fa_hip_ag_chain, first_free): the candidate count of each level is the only
        readback.  None when the device chain does not apply (then _gen + _plan_bundle)."""
        dev = self._dev
        if not (dev.type == "cuda" and TUNING.gen_device and TUNING.gen_chain and TUNING.bundle_levels
                and self.cfg.level_kernel in ("auto", "slab") and k - 1 <= TUNING.bundle_max_prefix
                and prev.shape[0] >= TUNING.gen_device_min_rows and prev.shape[1] >= 2
                and self._F1 <= ops.primitives.AG_DEVICE_MAX_F1):
            return None
        max_lv = (self.cfg.max_level - k + 1) if self.cfg.max_level else 64
        with roctx_range("gen_bundle"), self._timer.phase("apriori_gen"):
            return ops.primitives.apriori_gen_chain(prev, self._F1, dev, max_lv, TUNING.bundle_growth, 0, 0,
                                                    first_free=True)

    def _bundle_from_chain(self, k: int, prev: np.ndarray, chain: list) -> list:
        bundle, rows, src = [], [], prev
        for j, (pi, eo, ex, nxt) in enumerate(chain):
            bundle.append((k + j, src, pi, eo, ex))
            rows.append(np.ascontiguousarray(nxt, np.int32))
            src = nxt
        self._bundle_rows = rows
        return bundle

    def _plan_bundle(self, db, k: int, prev: np.ndarray, prefix_idx, ext_off, ext, cand_rows=None) -> list:
        """Levels counted in one launch, starting with level k.

        Level k+1's candidates are generated from level k's *candidates* (not
        its frequent sets): a superset of apriori_gen(F_k) with exact counts, so
        thresholding it yields exactly F_{k+1} (every frequent (k+1)-itemset has
        frequent, hence candidate, k-subsets).  On T10I4 data these supersets are
        within 2-20 % of the real candidate sets, and one slab build + one launch
        replaces several.  Levels are added while the total fits one LDS
        accumulator pass, a level does not grow past TUNING.bundle_growth x the previous
        one, and prefixes stay short (deep levels prefer the trie kernel).
        Returns [(k, prefix rows source, prefix_idx, ext_off, ext), ...]."""
        bundle = [(k, prev, prefix_idx, ext_off, ext)]
        if cand_rows is None:
            g_of_e = np.repeat(np.arange(prefix_idx.size), np.diff(ext_off))
            cand_rows = np.concatenate([prev[prefix_idx[g_of_e]], ext[:, None]], axis=1)
        # candidate rows of every bundled level (result assembly: rows[count >= minCount])
        self._bundle_rows = [np.ascontiguousarray(cand_rows, np.int32)]
        if (not TUNING.bundle_levels or self.cfg.level_kernel not in ("auto", "slab")
                or k - 1 > TUNING.bundle_max_prefix):
            return bundle
        C = int(ext.size)
        items = np.zeros(db["F1"], dtype=bool)
        items[self._bundle_rows[0].ravel()] = True
        total = C
        n_used = int(items.sum())
        if total > ops.primitives.slab_capacity(n_used, total):
            return bundle
        cand = self._bundle_rows[0]
        last = C
        kk = k
        dev = self._dev
        if (dev.type == "cuda" and TUNING.gen_device and TUNING.gen_chain and cand.shape[1] >= 2
                and self._F1 <= ops.primitives.AG_DEVICE_MAX_F1):
            # all speculative levels in one native call (one 8-byte readback per level)
            max_lv = (self.cfg.max_level - k) if self.cfg.max_level else 64
            tmax = ops.primitives.slab_total_limit(n_used)
            for pi, eo, ex, nxt in ops.primitives.apriori_gen_chain(cand, self._F1, dev, max_lv,
                                                                    TUNING.bundle_growth, total, tmax):
                kk += 1
                bundle.append((kk, cand, pi, eo, ex))
                self._bundle_rows.append(nxt)
                cand = nxt
            return bundle
        while self.cfg.max_level == 0 or kk + 1 <= self.cfg.max_level:
            pi, eo, ex, nxt = self._gen(cand, want_rows=True)
            C2 = int(ex.size)
            if C2 == 0 or C2 > TUNING.bundle_growth * last:
                break
            # later levels only use items of level k's candidates: n_used is fixed
            if total + C2 > ops.primitives.slab_capacity(n_used, total + C2):
                break
            kk += 1
            bundle.append((kk, cand, pi, eo, ex))
            self._bundle_rows.append(np.ascontiguousarray(nxt, np.int32))
            total, last = total + C2, C2
            cand = nxt
        return bundle

    def _count_bundle(self, db, bundle: list) -> list:
        """Counts of every level of a bundle (one launch on the GPU).  The all-reduce is
        over the rank group in both modes: row shards (count mode) or this rank's share
        of the plan's pieces over the whole replicated DB (candidate mode, _piece_part)."""
        if len(bundle) == 1 or db["ranks"].device.type != "cuda":
            return [self._count_level(db, pv, pi, eo, ex) for _, pv, pi, eo, ex in bundle]
        full_db = db
        pre = [pv[pi] for _, pv, pi, _, _ in bundle]
        poff = np.concatenate([[0], np.cumsum(np.concatenate([np.full(p.shape[0], p.shape[1]) for p in pre]))])
        flat = np.concatenate([p.ravel() for p in pre]).astype(np.int32)
        sizes = [int(ex.size) for *_, ex in bundle]
        eoff = np.concatenate([[0], np.cumsum(np.concatenate([np.diff(eo) for _, _, _, eo, _ in bundle]))])
        ext = np.concatenate([ex for *_, ex in bundle]).astype(np.int32)
        self._piece_part(True)
        try:
            cnt = ops.count_level(db["roff"], db["ranks"], db["src"], db["ncols"], db["F1"], flat, eoff, ext,
                                  db["wword"], kernel="slab", poff=poff,
                                  full_bm=lambda u: self._bitmaps(db, u, blocked=True),
                                  sup_frac=self.stats["min_count"] / max(1, self.stats["n_lines"]))
        finally:
            self._piece_part(False)
        if cnt is None:
            return [self._count_level(full_db, pv, pi, eo, ex) for _, pv, pi, eo, ex in bundle]
        self.comm.all_reduce_(cnt, bound=self.stats["n_lines"])
        c = cnt.cpu().numpy()
        return np.split(c, np.cumsum(sizes)[:-1])

    def _count_level(self, db, prev: np.ndarray, prefix_idx, ext_off, ext) -> np.ndarray:
        if self.cand_par:
            # candidate parallelism: this rank counts a contiguous, extension-balanced
            # range of prefix groups over all rows; the other entries stay 0, so the
            # all-reduce assembles the full vector (FastApriori.scala:140-157)
            C, r, nr = int(ext.size), self.comm.rank, self.comm.world_size
            g0, g1 = (int(np.searchsorted(ext_off, C * q // nr, side="left")) for q in (r, r + 1))
            g1 = prefix_idx.size if r == nr - 1 else g1
            e0, e1 = int(ext_off[g0]), int(ext_off[g1])
            part = np.zeros(0, np.int64)
            if g1 > g0:
                part = self._count_groups(db, prev, prefix_idx[g0:g1], ext_off[g0:g1 + 1] - e0, ext[e0:e1])
            full = torch.zeros(C, dtype=torch.int64, device=self.comm.device)
            full[e0:e1] = torch.from_numpy(part).to(full.device)
            self.comm.all_reduce_(full, bound=self.stats["n_lines"])
            return full.cpu().numpy()
        cnt = self._count_groups(db, prev, prefix_idx, ext_off, ext)
        return cnt

    def _count_groups(self, db, prev: np.ndarray, prefix_idx, ext_off, ext) -> np.ndarray:
        """Local support counts of the groups (prefix_idx, ext_off, ext), all-reduced over
        the row shards in count parallelism (a no-op collective in candidate mode)."""
        dev = db["ranks"].device
        lk = self.cfg.level_kernel
        if dev.type == "cuda" and lk in ("auto", "slab"):
            cnt = ops.count_level(db["roff"], db["ranks"], db["src"], db["ncols"], db["F1"], prev[prefix_idx],
                                  ext_off, ext, db["wword"], kernel=lk, full_bm=lambda u: self._bitmaps(db, u, blocked=True),
                                  sup_frac=self.stats["min_count"] / max(1, self.stats["n_lines"]))
            if cnt is not None:
                self.dcomm.all_reduce_(cnt, bound=self.stats["n_lines"])
                return cnt.cpu().numpy()
        self._bitmaps(db)
        prefix = torch.from_numpy(np.ascontiguousarray(prev[prefix_idx], dtype=np.int32)).to(dev)
        ext_t = torch.from_numpy(np.ascontiguousarray(ext, dtype=np.int32)).to(dev)
        cnt = ops.count_candidates(db["bm"], db["W"], prefix, ext_off, ext_t, db["wword"])
        self.dcomm.all_reduce_(cnt, bound=self.stats["n_lines"])
        return cnt.cpu().numpy()


def mine(shard: TransactionShard, min_support: float = 0.092, comm: Comm | None = None, **kw) -> MiningResult:
    cfg = MinerConfig(min_support=min_support, **kw)
    return FastApriori(min_support, comm, cfg).run(shard)


__all__ = ["FastApriori", "MinerConfig", "mine", "math"]
