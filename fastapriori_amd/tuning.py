"""Internal tuning knobs: one dataclass, read at call time.

Product settings (what a user of the reference changes: support, device, strategy,
outputs) live in ``config.JobConfig`` (CLI > FA_* env > defaults) and
``models.apriori.MinerConfig``.  Everything here is a lab setting: the defaults are the
measured choices (docs/PERF.md, docs/PERF_HISTORY.md), code reads them through the
module-level ``TUNING`` instance when it runs (not at import), and tests change them
with ``override(...)``.  A/B experiments set ``FA_TUNE="name=value,name=value"`` --
the one environment variable this module reads -- e.g.
``FA_TUNE=bundle_growth=2.0,device_levels=0 python bench.py``.

The full table of knobs with their defaults is in docs/ARCHITECTURE.md
("Configuration").
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from dataclasses import dataclass, fields


@dataclass
class Tuning:
    # ---- level loop (models/apriori.py) -------------------------------------------
    bundle_levels: bool = True          # count speculative later levels in level k's launch
    bundle_growth: float = 1.5          # a bundled level may have <= this x the previous level's candidates
    bundle_max_prefix: int = 9          # no bundling past prefixes of this many items
    device_levels: bool = True          # level bundles generated / counted / thresholded on the GPU
    dl_post: bool = True                # the bundle's plan + count queued by the generator's native call
    dl_multi: bool = True               # multi-pass levels stay on the device (window by window)
    gen_device: bool = True             # apriori-gen on the GPU for big levels (host loop)
    gen_chain: bool = True              # speculative levels in one native call (host loop)
    gen_device_min_rows: int = 512      # smaller F_{k-1}: the C++ host generator
    # k = 2 across ranks: triangles of at least this many pairs are reduce-scattered and
    # thresholded per slice (Comm.reduce_scatter_select) instead of all-reduced; below it
    # the triangle is all-reduced and F_2 compacted on the device with no host round trip.
    # For the T10I4 triangle (474K pairs, 1.9 MB) one ring all-reduce over xGMI costs less
    # than the reduce-scatter's three collectives and two host syncs; 4M pairs (F1 ~ 2900,
    # 16 MB) is where the all-reduce's 2(W-1)/W volume starts to dominate.
    pair_rs_min: int = 1 << 22
    # ---- compression (ops/primitives.py) ------------------------------------------
    fused_compress: bool = True         # two-pass fused compression for short rows
    early_compress: bool = True         # compression queued before the F1 bookkeeping (host overlap)
    f1_rank_device: bool = True         # narrow numeric vocabularies ranked on the device (no F1 host round trip)
    fused_compress_mean_len: float = 12.0
    fused_layout: bool = True           # the emit pass writes the pair kernel's blocked layout
    compress_wave_mean_len: float = 48.0
    # ---- counting kernels (ops/primitives.py) -------------------------------------
    slab_lds_bytes: int = 160 * 1024 - 512   # LDS of the slab kernel (minus its static scratch)
    slab_cls: int = 1                   # class layout of host-planned slab passes: 0 off, 1 model, 2 always
    dense_min_rows: float = 4.0         # skip the all-zero-prefix test above this many rows per slab
    dl_acc16: bool = True               # packed u16 accumulators in window-by-window levels (unit weights)
    dl_acc16_bundles: bool = False      # ... and in one-pass device bundles
    mp_window_items: bool = True        # window-by-window levels: each window's slab holds only its own used items
    # window-by-window levels: a window counts only the rows holding >= k of its own items
    # (its items' bitmap compacted to them, count.hip k_win_compact) when the binomial
    # estimate keeps fewer than window_trim_est_frac of the level's rows and the count
    # (a sample, then exact) fewer than min(window_trim_rows_frac,
    # 1 - window_trim_cost * items / (candidates * (k + 1))) (FastApriori._window_rows)
    window_trim: bool = True
    window_trim_est_frac: float = 0.95
    window_trim_rows_frac: float = 0.97
    window_trim_cost: float = 100.0
    # ... when the rank's shard had at least this many rows after compression (T40I10D10M,
    # 10M rows: windows of a tenth of the work, where the compaction's fixed costs ate the
    # gain: 70.6 -> 73.6 ms; the shard's size, not the level's: T40I10D100M's level 11
    # keeps ~20M rows and still gains, 21.8 -> 16.5 ms)
    window_trim_min_rows: int = 1 << 25
    # bundle capacity = the largest over the slab widths (a bundle takes a narrower slab
    # when that holds all of it) instead of the first width holding 8192 candidates
    slab_cap_max: bool = False
    # bank-aware lane deal of device slab plans (levels.hip k_dl_lane_assign) from this many
    # rows (-1: off): ~0.18 ms per bundle against ~5 % of the slab counts (T10I4D100M
    # 42.1 -> 41.2 ms; the 12.5M-row shard 6.50 -> 6.85 ms, hence the threshold)
    lane_deal_min_rows: int = 1 << 25
    pair_wg: int = 0                    # k_pair_queue16 workgroups (0: one per CU)
    gram_mfma_min_class_words: int = 512   # shorter weight classes: the popcount Gram
    bitmap_blocked: bool = True         # the Gram's bitmap in 8-word blocks (count.hip BmView)
    # transaction trimming before a level (models/apriori.py _trim_worth_it, gen.hip dl_post):
    # when the binomial estimate keeps fewer than this share of the rows, or of the items
    trim_rows_frac: float = 0.75
    trim_nnz_frac: float = 0.6
    # ---- I/O (utils/io.py) -------------------------------------------------------
    gpu_parse: bool = True              # D.dat parsed on the GPU behind the H2D copies
    gpu_parse_dict: bool = True         # dictionary-mode tokens too
    stream_parse: bool = True           # parse each chunk as it lands
    ring_slots: int = 16                # pinned read-ring slots (pread threads)
    # ---- collectives (parallel/comm.py) --------------------------------------------
    bucket_mb: float = 64.0             # largest single all-reduce; longer vectors go in buckets

    @classmethod
    def from_env(cls, spec: str | None = None) -> "Tuning":
        t = cls()
        t.apply(os.environ.get("FA_TUNE", "") if spec is None else spec)
        return t

    def apply(self, spec: str) -> None:
        """'name=value,name=value' (bools as 0/1/true/false)."""
        types = {f.name: f.type for f in fields(self)}
        for part in filter(None, (p.strip() for p in spec.split(","))):
            name, _, val = part.partition("=")
            name = name.strip()
            if name not in types:
                raise ValueError(f"FA_TUNE: unknown knob {name!r} (known: {', '.join(sorted(types))})")
            cur = getattr(self, name)
            if isinstance(cur, bool):
                v = val.strip().lower() in ("1", "true", "yes", "on")
            else:
                v = type(cur)(float(val) if isinstance(cur, int) else val)
            setattr(self, name, v)


TUNING = Tuning.from_env()


@contextmanager
def override(**kw):
    """Temporarily change knobs of TUNING (tests, experiments)."""
    old = {k: getattr(TUNING, k) for k in kw}
    for k in kw:
        if not hasattr(TUNING, k):
            raise AttributeError(f"unknown tuning knob {k}")
    try:
        for k, v in kw.items():
            setattr(TUNING, k, v)
        yield TUNING
    finally:
        for k, v in old.items():
            setattr(TUNING, k, v)


__all__ = ["Tuning", "TUNING", "override"]
