"""Typed wrappers over the mining primitives.

Every op takes torch tensors and runs where they live:
  * CUDA (= HIP on ROCm) tensors -> the hand-written CDNA4 kernels in libfa_hip.so,
    launched on torch's current stream.  There is no silent fallback: a missing
    library raises.
  * CPU tensors -> the C++ reference implementations in libfa_host.so (used by
    the gloo multi-process tests and the CPU plumbing config).

Conventions: bitmaps are int64 tensors [F1, Wp] holding raw 64-bit words
(column c = bit c&63 of word c>>6); counts come back as int64.
"""
from __future__ import annotations

import ctypes as C
import ctypes
import os
import time
from dataclasses import dataclass

import numpy as np
import torch

from ..tuning import TUNING
from ..utils.env import num_threads
from . import _native

_I32, _I64 = torch.int32, torch.int64
PAIR_CHUNK_ROWS = 1 << 18   # rows per pair-kernel chunk (working set ~10 MB: L2 / Infinity Cache resident)


def _p(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class _PinnedStage:
    """Grow-only pinned host staging buffer for small per-level H2D copies.

    Fresh pinned allocations of varying sizes (tensor.pin_memory(), torch.empty(...,
    pin_memory=True)) each cost a host-allocator round trip of ~0.3-0.5 ms, which
    showed up as the largest host gaps between kernels of the level loop.  An event
    recorded after each copy guards the buffer against reuse while a copy from it
    may still be in flight."""

    def __init__(self):
        self.buf = None
        self.event = None

    def get(self, nbytes: int) -> torch.Tensor:
        if self.event is not None:
            self.event.synchronize()
            self.event = None
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(nbytes, 1 << 20, 2 * (self.buf.numel() if self.buf is not None else 0)),
                                   dtype=torch.uint8, pin_memory=True)
        return self.buf[:nbytes]

    def h2d(self, host: np.ndarray, dev) -> torch.Tensor:
        """Copy a host array to the device through the pinned stage (async)."""
        host = np.ascontiguousarray(host)
        st = self.get(host.nbytes)
        st.numpy()[:] = host.reshape(-1).view(np.uint8)
        out = st.to(dev, non_blocking=True).view(dtype=_np2torch(host.dtype)).reshape(host.shape)
        self.event = torch.cuda.Event()
        self.event.record()
        return out


def _np2torch(dt):
    return {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64, np.dtype(np.uint8): torch.uint8}[
        np.dtype(dt)]


_STAGES: dict = {}


def pinned_stage(key: str) -> _PinnedStage:
    st = _STAGES.get(key)
    if st is None:
        st = _STAGES[key] = _PinnedStage()
    return st


def _hip_call(name: str, *args) -> None:
    fn = getattr(_native.hip(), name)
    # ctypes passes surplus arguments as C varargs: a binding that lags its C signature
    # would silently truncate pointers, so the count must match
    if fn.argtypes is not None and len(args) != len(fn.argtypes):
        raise TypeError(f"{name}: {len(args)} arguments for a {len(fn.argtypes)}-argument binding")
    rc = fn(*args)
    _native.check(rc, name)


# ---------------------------------------------------------------------------
def histogram(items: torch.Tensor, V: int) -> torch.Tensor:
    """Occurrences of each id in ``items`` (int32) -> int64 [V]."""
    assert items.dtype == _I32 and items.is_contiguous()
    if items.is_cuda:
        out = torch.zeros(V, dtype=_I32, device=items.device)
        if items.numel():
            _hip_call("fa_hip_histogram", _p(items), items.numel(), V, _p(out), _stream(items))
        return out.to(_I64)
    out = torch.zeros(V, dtype=_I64)
    _native.host().fa_cpu_histogram(_p(items), items.numel(), V, _p(out), num_threads())
    return out


F1_RANK_DEVICE_MAX = 2048   # prep.hip kF1RankMax


class F1Pending:
    """The device F1 ranking of f1_rank_start: the id -> rank LUT is on the device
    already (kernels that read it can be queued); finish() waits for the ranking's copy
    to pinned memory and returns (frequent ids, their supports) in rank order."""

    def __init__(self, lut: torch.Tensor, host: torch.Tensor, ev, V: int):
        self.lut, self._host, self._ev, self.V = lut, host, ev, V
        self._got = None

    def finish(self):
        if self._got is None:
            self._ev.synchronize()
            h = self._host.numpy()
            F = int(h[0])
            self._got = h[1:1 + F].copy(), h[1 + self.V:1 + self.V + F].copy()
        return self._got


def f1_rank_start(hist: torch.Tensor, thr: int, numeric_tiebreak: bool) -> F1Pending:
    """Rank the frequent ids of an int64 [V] histogram on the device (prep.hip k_f1_rank:
    FastApriori.scala:55-62's order, csrc/host/f1.cpp fa_f1_rank_numeric's) and queue
    the ranking's copy to pinned memory, without waiting (F1Pending)."""
    V = hist.numel()
    assert hist.is_cuda and hist.dtype == _I64 and 1 <= V <= F1_RANK_DEVICE_MAX and thr >= 1
    dev = hist.device
    lut = torch.empty(V, dtype=_I32, device=dev)
    pack = torch.empty(2 * V + 1, dtype=_I64, device=dev)
    _hip_call("fa_hip_f1_rank", _p(hist), V, int(thr), int(bool(numeric_tiebreak)), _p(lut), _p(pack), _stream(hist))
    stage = pinned_stage("f1_rank")
    host = stage.get(8 * pack.numel()).view(_I64)
    host.copy_(pack, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    stage.event = ev
    return F1Pending(lut, host, ev, V)


# ---------------------------------------------------------------------------
# Heavy-hitter F1 (wide vocabularies; csrc/hip/prep.hip k_f1_sketch/k_f1_exact)
# ---------------------------------------------------------------------------
SK_LOG = 14                      # sketch bins per row (2 rows)
SK_A = (0x9E3779B1, 0x85EBCA77)  # multiplicative hash constants (mirrored in prep.hip)
F1_MAX_CANDIDATES = 1 << 13      # exact-pass LDS table: 16K slots at load <= 0.5


def sk_hash(ids: torch.Tensor, a: int, log: int = SK_LOG) -> torch.Tensor:
    """(uint32(id) * a) >> (32 - log), as int64."""
    return ((ids.to(_I64) * a) & 0xFFFFFFFF) >> (32 - log)


def f1_sketch(items: torch.Tensor) -> torch.Tensor:
    """2-row count-min sketch of the ids in ``items`` -> int64 [2, 2**SK_LOG]."""
    W = 1 << SK_LOG
    if items.is_cuda:
        nwg = C.c_int(0)
        partial = torch.empty(256 * 2 * W, dtype=_I32, device=items.device)
        _hip_call("fa_hip_f1_sketch", _p(items), items.numel(), _p(partial), C.addressof(nwg), _stream(items))
        # per-workgroup counts < 2^31 (a workgroup sees at most nnz/nwg tokens)
        return partial[: nwg.value * 2 * W].view(max(nwg.value, 1), 2, W).sum(0, dtype=_I64) if nwg.value else \
            torch.zeros(2, W, dtype=_I64, device=items.device)
    return torch.stack([torch.bincount(sk_hash(items, a), minlength=W) for a in SK_A])


def sketch_estimate(sk: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    return torch.minimum(sk[0][sk_hash(ids, SK_A[0])], sk[1][sk_hash(ids, SK_A[1])])


def f1_exact(items: torch.Tensor, cand: torch.Tensor) -> torch.Tensor:
    """Exact occurrence counts of the (distinct) ids ``cand`` in ``items`` -> int64 [len(cand)]."""
    n = cand.numel()
    assert n <= F1_MAX_CANDIDATES
    if n == 0:
        return torch.zeros(0, dtype=_I64, device=items.device)
    if items.is_cuda:
        log_s = max(6, (2 * n - 1).bit_length())
        ids = cand.to(_I64).cpu().contiguous()
        keys = torch.empty(1 << log_s, dtype=_I32)
        slot = torch.empty(n, dtype=_I64)
        _native.host().fa_build_probe_table(_p(ids), n, log_s, SK_A[0], _p(keys), _p(slot))
        counts = torch.zeros(1 << log_s, dtype=_I32, device=items.device)
        _hip_call("fa_hip_f1_exact", _p(items), items.numel(), _p(keys.to(items.device)), log_s, _p(counts),
                  _stream(items))
        return counts[slot.to(items.device)].to(_I64)
    srt, order = torch.sort(cand.to(_I64))
    pos = torch.searchsorted(srt, items.to(_I64)).clamp_(max=n - 1)
    hit = srt[pos] == items.to(_I64)
    out = torch.zeros(n, dtype=_I64)
    out[order] = torch.bincount(pos[hit], minlength=n)
    return out


def txn_freq_count(offsets: torch.Tensor, items: torch.Tensor, lut: torch.Tensor) -> torch.Tensor:
    """Number of frequent ids (``lut[id] >= 0``) per transaction -> int32 [n]."""
    n = offsets.numel() - 1
    out = torch.empty(n, dtype=_I32, device=items.device)
    if n <= 0:
        return out
    if items.is_cuda:
        _hip_call("fa_hip_txn_freq_count", _p(offsets), _p(items), n, items.numel(), _p(lut), _p(out),
                  _stream(items))
    else:
        _native.host().fa_cpu_txn_freq_count(_p(offsets), _p(items), n, _p(lut), _p(out), num_threads())
    return out


COMPRESS_WAVE_MAX_F1 = 65536
# mean row length above which the 64-token staged tier (64 KB input span per workgroup) runs first
COMPRESS_STAGED64_MEAN_LEN = 16.0


def compress(offsets, items, lut, kept, roff, F1: int | None = None) -> torch.Tensor:
    """Kept transaction x -> its frequent ranks sorted ascending, CSR by ``roff``.

    Device tiers (csrc/hip/prep.hip), chosen by row length L: L <= 16 LDS-staged
    register sort; L <= 64 register bitonic network; longer rows one wave per
    row with an LDS rank bitmap (no sort; F1 <= 65536) or, for wider F1, a
    workgroup LDS bitonic sort.  Long-document data (mean L large) skips the
    first two tiers."""
    T = kept.numel()
    nnz = int(roff[-1].item()) if T else 0
    ranks = torch.empty(max(nnz, 1), dtype=_I32, device=items.device)
    if T == 0:
        return ranks[:0]
    if not items.is_cuda:
        _native.host().fa_cpu_compress(_p(offsets), _p(items), _p(lut), _p(kept), T, _p(roff), _p(ranks),
                                       num_threads())
        return ranks[:nnz]
    st = _stream(items)
    wave_ok = F1 is not None and F1 <= COMPRESS_WAVE_MAX_F1
    if wave_ok and items.numel() > TUNING.compress_wave_mean_len * max(offsets.numel() - 1, 1):
        _hip_call("fa_hip_compress_wave", _p(offsets), _p(items), _p(lut), None, T, _p(kept), _p(roff),
                  _p(ranks), F1, None, st)
        return ranks[:nnz]
    flag = torch.empty(T, dtype=torch.int8, device=items.device)
    # long-ish rows (mean > COMPRESS_STAGED64_MEAN_LEN tokens): the 64-token staged tier first
    staged64 = items.numel() > COMPRESS_STAGED64_MEAN_LEN * max(offsets.numel() - 1, 1)
    if staged64:   # (F1 unknown: the u32 span)
        _hip_call("fa_hip_compress_staged64", _p(offsets), _p(items), _p(lut), T, _p(kept), _p(roff), _p(ranks),
                  _p(flag), int(F1 or 0), st)
    else:
        _hip_call("fa_hip_compress_staged", _p(offsets), _p(items), _p(lut), T, _p(kept), _p(roff), _p(ranks),
                  _p(flag), st)
    over = torch.nonzero(flag).flatten().to(_I32)
    n1 = over.numel()
    over2, n2 = over, n1                 # after the 64-token staged tier: rows of > 64 tokens
    if n1 and not staged64:
        flag2 = torch.empty(n1, dtype=torch.int8, device=items.device)
        _hip_call("fa_hip_compress_regs", 64, _p(offsets), _p(items), _p(lut), _p(over), n1, _p(kept),
                  _p(roff), _p(ranks), _p(flag2), st)
        over2 = over[torch.nonzero(flag2).flatten()].contiguous()
        n2 = over2.numel()
    if n2:
        if wave_ok:
            _hip_call("fa_hip_compress_wave", _p(offsets), _p(items), _p(lut), _p(over2), n2, _p(kept), _p(roff),
                      _p(ranks), F1, None, st)
        else:
            over3 = torch.empty(n2, dtype=_I32, device=items.device)
            n_over3 = torch.zeros(1, dtype=_I32, device=items.device)
            _hip_call("fa_hip_compress_lds", _p(offsets), _p(items), _p(lut), _p(over2), n2, _p(kept),
                      _p(roff), _p(ranks), _p(over3), _p(n_over3), st)
            n3 = int(n_over3.item())
            if n3:   # rows longer than 16384 tokens: sorted by torch, row by row
                _compress_torch(offsets, items, lut, kept, roff, ranks, over3[:n3])
    return ranks[:nnz]


PAIR_PAD_BATCHES = 3 * 16 + 2   # the pair kernel's pipeline reads up to this many batches past a chunk
# the emit pass of compress_rows also writes the pair kernel's blocked layout (TUNING.fused_layout off: the
# separate block-scatter pass of pair_counts_horizontal)


@dataclass
class BlockLayout:
    """The k = 2 blocked layout of compressed rows (pair_counts_horizontal): cnt = u8
    [nb * T + pad] per-row counts of 256-rank blocks; lr / base (optional) = the local
    ranks (u8, block-major, row order) and the int64 [nb * ceil(T / 64) + pad] 64-row
    batch bases, written by compress_rows' emit pass (no block-scatter pass)."""
    cnt: torch.Tensor
    lr: torch.Tensor | None = None
    base: torch.Tensor | None = None

    def cpu(self):
        return self.cnt.cpu()


# rows hashed by the dedup estimate (FastApriori._want_dedup): linear counting of 2^18
# row hashes in 2^22 slots estimates the distinct fraction to ~0.03 % (one standard
# error); the probe is a fixed cost per rank (1M rows: 0.22 ms)
DEDUP_PROBE_ROWS = 1 << 18


def compress_rows(offsets, items, lut, F1: int, block_counts: bool = True, probe: dict | None = None):
    """compress_rows_finish(compress_rows_start(...)).  Fused two-pass compression (device, short rows; csrc/hip/prep.hip k_cmp_agg /
    k_cmp_emit): returns (kept int32 [T], roff int64 [T+1], ranks int32 [nnz],
    length histogram (host int64 [256]), bcnt) with one host synchronisation.  Rows
    of more than 16 tokens are finished by the register / wave tiers of ``compress``
    (the rows the register tier leaves go to the wave tier by flag, no compaction).

    bcnt (block_counts and F1 <= 2048, else None): uint8 [nb * T + pad], the
    per-row item counts of 256-rank blocks that the pair kernel's blocked layout
    needs (pair_counts_horizontal), written by the emit pass while the sorted row
    is in registers instead of by a separate pass over the ranks.

    probe (a dict): also run the dedup probe (prep.hip k_dedup_probe) over the first
    min(T, DEDUP_PROBE_ROWS) rows, read back with the sizes: probe["n"] rows hashed,
    probe["filled"] occupied slots of its 2^22-slot bitmap."""
    return compress_rows_finish(compress_rows_start(offsets, items, lut, F1, block_counts, probe))


def compress_rows_start(offsets, items, lut, F1: int, block_counts: bool = True, probe: dict | None = None) -> dict:
    """Queue compress_rows' kernels and the copy of its sizes to pinned memory, without
    waiting: the caller's host work overlaps them until compress_rows_finish."""
    dev = items.device
    n = offsets.numel() - 1
    nwg = (n + 255) // 256
    st = _stream(items)
    nb = (F1 + 255) // 256
    blk = block_counts and 1 <= nb <= 8 and n > 0
    fused = blk and TUNING.fused_layout
    agg = torch.empty(3 * max(nwg, 1), dtype=_I32, device=dev)
    aggb = torch.empty(nb * nwg, dtype=_I32, device=dev) if fused else None
    hist = torch.zeros(64, 256, dtype=_I32, device=dev)
    _hip_call("fa_hip_cmp_agg", _p(offsets), _p(items), _p(lut), n, _p(agg), _p(hist), _p(aggb), nb, st)
    # exclusive scans of the aggregates (and block totals) + roff[0] = 0: prep.hip fa_hip_cmp_scan
    pre = torch.empty(3, nwg + 1, dtype=_I64, device=dev)
    preb = torch.empty(nb * nwg + 1, dtype=_I64, device=dev) if fused else None
    kept = torch.empty(max(n, 1), dtype=_I32, device=dev)
    roff = torch.empty(n + 1, dtype=_I64, device=dev)
    part = torch.empty(4 * ((max(nb, 1) * max(nwg, 1) + 4095) // 4096 + 1), dtype=_I64, device=dev)
    _hip_call("fa_hip_cmp_scan", _p(agg), _p(aggb), max(nwg, 1) if n > 0 else 0, nb, _p(part), _p(pre), _p(preb),
              _p(roff), st)
    if n <= 0:
        pre.zero_()
        roff[0] = 0
    ranks = torch.empty(max(items.numel(), 1), dtype=_I32, device=dev)
    over = torch.empty(max(n, 1), dtype=_I32, device=dev)
    bcnt = lr = lbase = ovb = None
    lr_cap = 0
    if blk:
        bcnt = torch.empty(nb * max(n, 1) + PAIR_PAD_BATCHES * 64 + 64, dtype=torch.uint8, device=dev)
    if fused:
        lr_cap = max(items.numel(), 1)
        lr = torch.empty(lr_cap + 1024, dtype=torch.uint8, device=dev)   # pad: aligned dword staging reads
        lbase = torch.zeros(nb * ((n + 63) // 64) + PAIR_PAD_BATCHES, dtype=_I64, device=dev)
        ovb = torch.empty(max(n, 1) * nb, dtype=_I64, device=dev)
    _hip_call("fa_hip_cmp_emit", _p(offsets), _p(items), _p(lut), n, _p(pre[0]), _p(pre[1]), _p(pre[2]), _p(kept),
              _p(roff), _p(ranks), _p(over), _p(bcnt), nb, _p(preb), _p(lr), lr_cap, _p(lbase), _p(ovb), st)
    if probe is not None:
        # the kernel reads T = pre[0, -1] on the device and hashes the rows the emit
        # pass has finished (<= 16 items; the later tiers write the longer ones)
        # scratch: the rows' slots + per-workgroup row counts (prep.hip, no zeroing)
        ws = torch.empty(DEDUP_PROBE_ROWS + (DEDUP_PROBE_ROWS + 255) // 256, dtype=_I32, device=dev)
        tail = torch.zeros(2, dtype=_I64, device=dev)
        _hip_call("fa_hip_dedup_probe", _p(roff), _p(ranks), pre[0].data_ptr() + 8 * (pre.shape[1] - 1),
                  DEDUP_PROBE_ROWS, _p(ws), _p(tail), st)
    # one readback: sizes, the probe's two counts, the row-length histogram
    hs = hist.sum(0, dtype=_I64)
    sizes = torch.cat([pre[:, -1], tail, hs] if probe is not None else [pre[:, -1], hs])
    host = pinned_stage("cmp_sizes")
    got = host.get(8 * sizes.numel())[:8 * sizes.numel()].view(_I64)
    got.copy_(sizes, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    host.event = ev
    return dict(offsets=offsets, items=items, lut=lut, F1=F1, probe=probe, got=got, ev=ev, kept=kept, roff=roff,
                ranks=ranks, over=over, bcnt=bcnt, lr=lr, lbase=lbase, ovb=ovb, lr_cap=lr_cap, nb=nb, st=st)


def compress_rows_finish(c: dict):
    """Wait for compress_rows_start's sizes and finish: slices, the rows past the emit
    pass (the later tiers), the block layout."""
    c["ev"].synchronize()
    got = c["got"].numpy().copy()
    probe, nb, st, bcnt, lr = c["probe"], c["nb"], c["st"], c["bcnt"], c["lr"]
    offsets, items, lut, F1 = c["offsets"], c["items"], c["lut"], c["F1"]
    if probe is not None:
        probe["filled"], probe["n"] = int(got[3]), int(got[4])
        hist_h = got[5:]
    else:
        hist_h = got[3:]
    T, nnz, no = int(got[0]), int(got[1]), int(got[2])
    kept, roff, ranks, over, lbase, ovb, lr_cap = (c[k] for k in ("kept", "roff", "ranks", "over", "lbase", "ovb",
                                                                   "lr_cap"))
    kept, roff, ranks = kept[:T], roff[:T + 1], ranks[:nnz]
    if bcnt is not None:
        bcnt = bcnt[:nb * T + PAIR_PAD_BATCHES * 64 + 64]
        bcnt[nb * T:].zero_()
        layout = BlockLayout(bcnt, lr, lbase)
    out = kept, roff, ranks, hist_h, (layout if bcnt is not None else None)
    if no:
        out = _compress_rows_overflow(offsets, items, lut, F1, kept, roff, ranks, over[:no], bcnt, T, nb, st, out)
        if lr is not None:    # the overflow rows' local ranks, after the later tiers sorted them
            _hip_call("fa_hip_lr_rows", _p(roff), _p(ranks), _p(over), no, _p(ovb), nb, _p(lr), lr_cap, st)
    return out


def _compress_rows_overflow(offsets, items, lut, F1, kept, roff, ranks, over, bcnt, T, nb, st, out):
    """The rows of more than 16 tokens compress_rows' emit pass left to the register /
    wave / LDS tiers (and their block counts)."""
    dev = items.device
    no = over.numel()
    if no:
        over = over[:no]
        flag2 = torch.empty(no, dtype=torch.int8, device=dev)
        if bcnt is not None:
            _hip_call("fa_hip_compress_regs_bc", _p(offsets), _p(items), _p(lut), _p(over), no, _p(kept), _p(roff),
                      _p(ranks), _p(flag2), _p(bcnt), T, nb, st)
        else:
            _hip_call("fa_hip_compress_regs", 64, _p(offsets), _p(items), _p(lut), _p(over), no, _p(kept), _p(roff),
                      _p(ranks), _p(flag2), st)
        if F1 <= COMPRESS_WAVE_MAX_F1:
            # rows of > 64 tokens (flag2) through the wave tier and the block counts, by
            # flag: no compaction, no host synchronisation
            _hip_call("fa_hip_compress_wave", _p(offsets), _p(items), _p(lut), _p(over), no, _p(kept), _p(roff),
                      _p(ranks), F1, _p(flag2), st)
            if bcnt is not None:
                _hip_call("fa_hip_block_counts_rows", _p(roff), _p(ranks), _p(over), no, _p(bcnt), T, nb, _p(flag2),
                          st)
            return out
        over2 = over[torch.nonzero(flag2).flatten()].contiguous()
        n2 = over2.numel()
        if n2:
            over3 = torch.empty(n2, dtype=_I32, device=dev)
            n_over3 = torch.zeros(1, dtype=_I32, device=dev)
            _hip_call("fa_hip_compress_lds", _p(offsets), _p(items), _p(lut), _p(over2), n2, _p(kept), _p(roff),
                      _p(ranks), _p(over3), _p(n_over3), st)
            n3 = int(n_over3.item())
            if n3:
                _compress_torch(offsets, items, lut, kept, roff, ranks, over3[:n3])
        if bcnt is not None and n2:       # rows of > 64 tokens, finished by the later tiers
            _hip_call("fa_hip_block_counts_rows", _p(roff), _p(ranks), _p(over2), n2, _p(bcnt), T, nb, None, st)
    return out


def _compress_torch(offsets, items, lut, kept, roff, ranks, rows):
    """Torch implementation: all rows vectorised (rows=None) or the listed rows."""
    if rows is not None:
        for x in rows.tolist():
            t = int(kept[x].item())
            r = lut[items[offsets[t]:offsets[t + 1]].to(_I64)]
            r = torch.sort(r[r >= 0]).values
            ranks[int(roff[x].item()): int(roff[x + 1].item())] = r.to(_I32)
        return ranks
    dev = items.device
    t = kept.to(_I64)
    starts = offsets[t]
    lens = offsets[t + 1] - starts
    total = int(lens.sum().item())
    rowid = torch.repeat_interleave(torch.arange(t.numel(), device=dev), lens)
    seg0 = torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens)
    pos = torch.arange(total, device=dev) - seg0 + torch.repeat_interleave(starts, lens)
    r = lut[items[pos].to(_I64)].to(_I64)
    keep = r >= 0
    base = int(lut.max().item()) + 1
    key, _ = torch.sort(rowid[keep] * base + r[keep])
    ranks[: key.numel()] = (key % base).to(_I32)
    return ranks[: key.numel()]


def row_hash(roff: torch.Tensor, ranks: torch.Tensor):
    T = roff.numel() - 1
    h1 = torch.empty(T, dtype=_I64, device=ranks.device)
    h2 = torch.empty(T, dtype=_I64, device=ranks.device)
    if T <= 0:
        return h1, h2
    if ranks.is_cuda:
        _hip_call("fa_hip_row_hash", _p(roff), _p(ranks), T, _p(h1), _p(h2), _stream(ranks))
    else:
        _native.host().fa_cpu_row_hash(_p(roff), _p(ranks), T, _p(h1), _p(h2), num_threads())
    return h1, h2


def bitmap_geometry(F1: int, ncols: int) -> tuple[int, int, int, int]:
    """(W, Wp, WT, R): valid words, padded row stride, LDS tile words, ranks per pass."""
    W = (ncols + 63) // 64
    WT = 8
    if F1 > 0:
        WT = 1 << max(2, min(5, int(np.floor(np.log2(max(1, 8192 // max(F1, 1)))))))
    R = max(1, min(F1, 8192 // WT)) if F1 > 0 else 1
    Wp = max(64, (W + 63) // 64 * 64)
    return W, Wp, WT, R


def blocked_bitmaps_ok(src, F1: int, ncols: int, item_map=None) -> bool:
    """The 8-word block layout (count.hip BmView) is built by the wave bitmap build
    only: contiguous rows, every item row in one LDS tile."""
    _, Wp, WT, R = bitmap_geometry(F1, ncols)
    return src is None and item_map is None and 0 < F1 <= R and F1 * WT * 8 <= 64 * 1024 and Wp % 8 == 0


def build_bitmaps(roff, ranks, src, ncols: int, F1: int, item_map=None, used=None,
                  blocked: bool = False) -> tuple[torch.Tensor, int]:
    """Item-major bitmaps [F1, Wp] (int64 words) and the valid word count W.

    With ``item_map`` (rank -> row, -1 = skip; device) and ``used`` (sorted ranks of
    the mapped items; device) only those F1 = len(used) rows are built (device only).
    blocked (device, blocked_bitmaps_ok): the Gram's 8-word block layout instead, a
    [Wp / 8, F1, 8] tensor (pair_counts_gram reads either).
    """
    W, Wp, WT, R = bitmap_geometry(F1, ncols)
    dev = ranks.device
    if ranks.is_cuda:
        if blocked:
            if not blocked_bitmaps_ok(src, F1, ncols, item_map):
                raise ValueError("blocked bitmaps need the wave build (contiguous rows, one LDS tile)")
            bm = torch.empty((Wp // 8, F1, 8), dtype=_I64, device=dev)
            _hip_call("fa_hip_build_bitmaps", _p(roff), _p(ranks), None, ncols, F1, Wp, WT, R, _p(bm),
                      None, None, 1, _stream(ranks))
            return bm, W
        bm = torch.empty((max(F1, 1), Wp), dtype=_I64, device=dev)
        if F1 > 0:
            _hip_call("fa_hip_build_bitmaps", _p(roff), _p(ranks), _p(src), ncols, F1, Wp, WT, R, _p(bm),
                      _p(item_map), _p(used), 0, _stream(ranks))
    else:
        bm = torch.zeros((max(F1, 1), Wp), dtype=_I64)
        if F1 > 0:
            _native.host().fa_cpu_build_bitmaps(_p(roff), _p(ranks), _p(src), ncols, Wp, _p(bm), num_threads())
    return bm[:F1], W


def pair_counts_horizontal(roff, ranks, wrow, F1: int, long_rows: bool = True, bcnt=None,
                           raw: bool = False) -> torch.Tensor:
    """Pair supports from the compressed rows -> int64 [F1, F1] (upper triangle);
    raw (device): the kernel's int32 [F1, F1] view as it is (pairs_compact's input).

    Device path: per-row block counts + local-rank bytes (blocked layout), then
    the 256 x 256 packed-u16 tile kernel for unit-weight rows, or 128 x 128 u32
    tiles with row weights.  long_rows: some row may hold >= 256 items, which
    would overflow a u8 count of a 256-item block -> 128-item blocks.  bcnt: the
    256-item block counts of these rows from compression (compress_rows: a
    BlockLayout, or its cnt tensor), which replace the counting pass; a BlockLayout
    with the local ranks and batch bases replaces the scatter pass too.
    """
    T = roff.numel() - 1
    dev = ranks.device
    if ranks.is_cuda:
        if T <= 0 or F1 < 2:
            out = torch.zeros((F1, F1), dtype=_I32, device=dev)
        else:
            st = _stream(ranks)
            pb = 128 if (wrow is not None or long_rows) else 256       # u16 tiles need unit weights
            nb = (F1 + pb - 1) // pb
            nbatch = (T + 63) // 64
            # cnt / base are padded past their ends: the pair kernel's software
            # pipeline loads up to 3 x 16 batches past a chunk unconditionally (those
            # values are never processed; padded bases must be valid lr offsets)
            pad_b = PAIR_PAD_BATCHES
            lay = bcnt if isinstance(bcnt, BlockLayout) else None
            if lay is not None:
                bcnt = lay.cnt
            if (lay is not None and lay.lr is not None and pb == 256 and bcnt.numel() >= nb * T + pad_b * 64
                    and lay.base.numel() >= nb * nbatch + pad_b):
                # the emit pass of compress_rows wrote the whole layout
                cnt, base, lr = bcnt, lay.base, lay.lr
            else:
                bsum = torch.empty(nb * nbatch, dtype=_I64, device=dev)
                if bcnt is not None and pb == 256 and bcnt.numel() >= nb * T + pad_b * 64:
                    cnt = bcnt
                    _hip_call("fa_hip_block_bsum", _p(cnt), T, T, nb, _p(bsum), st)
                else:
                    cnt = torch.empty(nb * T + pad_b * 64, dtype=torch.uint8, device=dev)
                    cnt[nb * T:].zero_()
                    _hip_call("fa_hip_block_counts", _p(roff), _p(ranks), T, F1, _p(cnt), _p(bsum), pb, st)
                base = torch.zeros(nb * nbatch + pad_b, dtype=_I64, device=dev)
                torch.cumsum(bsum, 0, out=base[:nb * nbatch])
                base[:nb * nbatch] -= bsum
                # every rank lands in exactly one block: the layout holds all of them (no readback)
                total = int(ranks.numel())
                lr = torch.empty(total + 1024, dtype=torch.uint8, device=dev)   # pad: aligned dword staging reads
                _hip_call("fa_hip_block_scatter", _p(roff), _p(ranks), T, F1, _p(cnt), _p(base), _p(lr), pb, st)
            if pb == 256:
                # work-queue schedule: persistent workgroups keep their tile across
                # sub-chunks; even row stride -> two counters per 64-bit flush atomic
                ld = F1 + (F1 & 1)
                nbp = nb * (nb + 1) // 2
                zb = torch.zeros(F1 * ld + nbp, dtype=_I32, device=dev)      # counts + queue counters: one fill
                out, qctr = zb[:F1 * ld].view(F1, ld), zb[F1 * ld:]
                _hip_call("fa_hip_pair_queue16", _p(cnt), _p(base), _p(lr), T, F1, ld, _p(qctr), _p(out),
                          TUNING.pair_wg, st)
                out = out[:, :F1]
            else:
                out = torch.zeros((F1, F1), dtype=_I32, device=dev)
                _hip_call("fa_hip_pair_blocked", _p(cnt), _p(base), _p(lr), T, _p(wrow), F1, _p(out),
                          PAIR_CHUNK_ROWS, st)
        return out if raw else out.to(_I64)
    out = torch.zeros((F1, F1), dtype=_I64)
    if T > 0 and F1 >= 2:
        _native.host().fa_cpu_pair_horizontal(_p(roff), _p(ranks), T, _p(wrow), F1, _p(out), num_threads())
    return out


def pairs_compact(pc: torch.Tensor, F1: int, mc: int, flat: bool = False):
    """F_2 on the device (count.hip fa_hip_pairs_compact): pairs with count >= mc in
    triangle order from the raw int32 pair counts (pair_counts_*(raw=True): a matrix
    with any row stride) or, flat=True, from the all-reduced int32 triangle.  Returns
    (rows int32 [C2 + 1, 2], counts int32 [C2 + 1], |F_2| int64 [1]) with no host
    synchronisation."""
    dev = pc.device
    C2 = F1 * (F1 - 1) // 2
    rows = torch.empty((C2 + 1, 2), dtype=_I32, device=dev)
    cnt = torch.empty(C2 + 1, dtype=_I32, device=dev)
    n = torch.empty(1, dtype=_I64, device=dev)
    row_cnt = torch.empty(max(F1, 1), dtype=_I32, device=dev)
    row_off = torch.empty(max(F1, 1), dtype=_I64, device=dev)
    if flat:
        assert pc.is_contiguous() and pc.numel() == C2 and pc.element_size() == 4
    ld = -1 if flat else pc.stride(0)
    _hip_call("fa_hip_pairs_compact", _p(pc), ld, F1, int(mc), _p(row_cnt), _p(row_off), _p(rows), _p(cnt), _p(n),
              _stream(pc))
    return rows, cnt, n


# weight classes shorter than TUNING.gram_mfma_min_class_words words go to the popcount
# Gram (a matrix-core launch per short class would cost more than its work)


def gram_segments(W: int, weighted: bool, wcls=None, force_popc: bool = False) -> list[tuple[int, int, int]]:
    """(word begin, word end, weight) launches of the Gram over words [0, W): one
    matrix-core launch per weight class (weight = its scale; unit weights: one
    class), and the runs of short classes merged into popcount launches (weight 0 =
    per-word weights from wword).  wcls: (weights, words) per class in column order
    (FastApriori._layout_weighted); a weighted layout without it takes the popcount
    Gram throughout."""
    if not weighted:
        return [(0, W, 0 if force_popc else 1)]
    if wcls is None:
        return [(0, W, 0)]
    segs, w0, run0 = [], 0, None
    for wt, nw in zip(*wcls):
        w1 = min(w0 + int(nw), W)
        if w1 > w0:
            if w1 - w0 >= TUNING.gram_mfma_min_class_words and not force_popc:
                if run0 is not None:
                    segs.append((run0, w0, 0))
                    run0 = None
                segs.append((w0, w1, int(wt)))
            elif run0 is None:
                run0 = w0
        w0 = w1
    if run0 is not None and run0 < W:
        segs.append((run0, W, 0))
    return segs


def to_blocked(bm: torch.Tensor) -> torch.Tensor:
    """Row-major bitmaps [F1, Wp] -> the 8-word block layout [Wp / 8, F1, 8]."""
    F1, Wp = bm.shape
    return bm.reshape(F1, Wp // 8, 8).transpose(0, 1).contiguous()


def bitmap_ld(bm) -> int:
    """The slab kernels' bitmap stride argument (count.hip slab_copy_bm): the row
    stride of a row-major bitmap, minus the block stride of a blocked one, 0 for none."""
    if bm is None:
        return 0
    return -bm.stride(0) if bm.dim() == 3 else bm.stride(0)


def _bm_view(bm: torch.Tensor, w0: int):
    """(F1, row stride, block stride, base pointer, in-block offset) of word w0 of a
    row-major [F1, Wp] or blocked [Wp / 8, F1, 8] bitmap (count.hip BmView)."""
    if bm.dim() == 3:
        F1, rs, bs = bm.shape[1], 8, bm.stride(0)
    else:
        F1, rs, bs = bm.shape[0], bm.stride(0), 8
    return F1, rs, bs, bm.data_ptr() + 8 * (w0 >> 3) * bs, w0 & 7


def pair_counts_gram(bm: torch.Tensor, W: int, wword, wcls=None, force_popc: bool = False,
                     fp4: bool = True, raw: bool = False, w0: int = 0) -> torch.Tensor:
    """Pair supports from the item-major bitmaps over words [w0, w0 + W) -> int64
    [F1, F1] (upper triangle).  bm: row-major [F1, Wp] or (device) the 8-word block
    layout [Wp / 8, F1, 8] (build_bitmaps(blocked=True)); wword / wcls cover the W
    words from w0.  Device: the FP4 matrix-core Gram (k_pair_gram_fp4) per weight
    class, scaled by the class weight (FastApriori.scala:233-235's weighted sum), short
    classes by the popcount Gram with per-word weights.  fp4=False: the i8 matrix-core
    form (kept as a test oracle of the FP4 one)."""
    F1 = bm.shape[1] if bm.dim() == 3 else bm.shape[0]
    if bm.is_cuda:
        out = torch.zeros((F1, F1), dtype=_I32, device=bm.device)
        if W > 0 and F1 >= 2:
            st = _stream(bm)
            segs = gram_segments(W, wword is not None, wcls, force_popc)
            for a, b, wt in segs:
                _, rs, bs, ptr, woff = _bm_view(bm, w0 + a)
                if wt > 0:
                    _hip_call("fa_hip_pair_gram_mfma", ptr, F1, rs, bs, woff, b - a, _p(out), 4096, wt, int(fp4), st)
                else:
                    _hip_call("fa_hip_pair_gram_popc", ptr, F1, rs, bs, woff, b - a,
                              wword.data_ptr() + 4 * a if wword is not None else None, _p(out), 4096, st)
        return out if raw else out.to(_I64)
    assert bm.dim() == 2, "the blocked bitmap layout is device-only"
    out = torch.zeros((F1, F1), dtype=_I64)
    if W > 0 and F1 >= 2:
        bm = bm[:, w0:]
        _native.host().fa_cpu_pair_gram(_p(bm), F1, bm.stride(0), W, _p(wword), _p(out), num_threads())
    return out


def _split_groups(ext_off: np.ndarray, per_block: int, max_block_ext: int = 1024):
    """Host-side work split for the candidate kernel.

    Groups with more than ``max_block_ext`` extensions are cut into several
    groups sharing a prefix; then consecutive groups are packed into blocks
    of about ``per_block`` extensions (never more than ``max_block_ext``).
    Returns (group index per new group, new ext_off, block starts).
    """
    G = ext_off.size - 1
    sizes = np.diff(ext_off)
    pieces = np.maximum(1, (sizes + max_block_ext - 1) // max_block_ext)
    gidx = np.repeat(np.arange(G, dtype=np.int64), pieces)
    first = np.repeat(np.cumsum(pieces) - pieces, pieces)
    k = np.arange(gidx.size) - first
    new_off = np.minimum(ext_off[gidx] + k * max_block_ext, ext_off[gidx + 1])
    new_off = np.append(new_off, ext_off[-1]).astype(np.int64)
    # pack consecutive pieces into blocks of <= lim extensions: a piece goes to the
    # block its first extension falls in, with blocks sized lim - max_piece so the
    # straddling piece still fits (vectorised; no Python loop over pieces)
    nsz = np.diff(new_off)
    lim = max(1, min(per_block, max_block_ext))
    step = max(1, lim - int(nsz.max(initial=0)) + 1) if nsz.size and nsz.max() < lim else 1
    before = new_off[:-1] - new_off[0]
    blk = before // step
    starts = np.flatnonzero(np.diff(blk, prepend=-1) > 0) if nsz.size else np.zeros(0, np.int64)
    starts = np.append(starts, nsz.size)
    if starts[0] != 0:
        starts = np.insert(starts, 0, 0)
    return gidx, new_off, np.asarray(starts, dtype=np.int32)


def count_candidates(bm: torch.Tensor, W: int, prefix: torch.Tensor, ext_off: np.ndarray,
                     ext: torch.Tensor, wword) -> torch.Tensor:
    """Support of every candidate prefix[g] + ext[e] (e in group g) -> int64 [C]."""
    C = ext.numel()
    dev = bm.device
    m = prefix.shape[1] if prefix.dim() == 2 else 0
    if C == 0:
        return torch.zeros(0, dtype=_I64, device=dev)
    if bm.is_cuda:
        nsc = max(1, (W + 2047) // 2048)
        per_block = int(np.clip(C * nsc // 4096, 16, 1024))
        gidx, new_off, starts = _split_groups(ext_off, per_block)
        pre = prefix[torch.from_numpy(gidx).to(dev)].contiguous() if gidx.size != prefix.shape[0] else prefix
        off_t = torch.from_numpy(new_off).to(dev)
        st_t = torch.from_numpy(starts).to(dev)
        out = torch.zeros(C, dtype=_I32, device=dev)
        _hip_call("fa_hip_count_candidates", _p(bm), bm.stride(0), W, _p(pre), m, _p(off_t), _p(ext),
                  _p(st_t), starts.size - 1, _p(wword), _p(out), _stream(bm))
        return out.to(_I64)
    out = torch.zeros(C, dtype=_I64)
    off_t = torch.from_numpy(np.ascontiguousarray(ext_off, dtype=np.int64))
    _native.host().fa_cpu_count_candidates(_p(bm), bm.stride(0), W, _p(prefix), m, _p(off_t), _p(ext),
                                           prefix.shape[0], _p(wword), _p(out), num_threads())
    return out


TRIM_HIST_BINS = 256   # csrc/hip/prep.hip kTrimHist


def trim_rows(roff, ranks, alive: torch.Tensor, min_len: int, wrow=None):
    """Keep rows with >= min_len alive items, dropping the dead items.

    alive: int8 [F1] on the rows' device.  Returns (kept row ids int32, new roff,
    new ranks, new wrow, histogram of new row lengths int64 [256], lengths >= 255
    in the last bin) — ranks stay sorted within each row.  Device path: count ->
    scan of 256-row block sums -> emit (csrc/hip/prep.hip k_trim_scan_count /
    k_trim_emit), one host sync for the output sizes.
    """
    T = roff.numel() - 1
    dev = ranks.device
    if T == 0:
        return (torch.zeros(0, dtype=_I32, device=dev), roff, ranks, wrow,
                torch.zeros(TRIM_HIST_BINS, dtype=_I64, device=dev))
    if ranks.is_cuda:
        st = _stream(ranks)
        nb = (T + 255) // 256
        cnt = torch.empty(T, dtype=_I32, device=dev)
        bk = torch.empty(2, nb, dtype=_I32, device=dev)
        F1 = alive.numel()
        _hip_call("fa_hip_trim_scan_count", _p(roff), _p(ranks), T, _p(alive), F1, int(min_len), _p(wrow), _p(cnt),
                  _p(bk[0]), _p(bk[1]), st)
        bases = torch.zeros(2, nb + 1, dtype=_I64, device=dev)
        torch.cumsum(bk[0], 0, dtype=_I64, out=bases[0, 1:])    # two 1-D scans: the [2, nb] scan
        torch.cumsum(bk[1], 0, dtype=_I64, out=bases[1, 1:])    # along dim 1 runs on 2 threads' worth
        K, nnz = (int(v) for v in bases[:, -1].tolist())
        nroff = torch.empty(K + 1, dtype=_I64, device=dev)
        nroff[K:] = nnz
        nranks = torch.empty(max(nnz, 1), dtype=_I32, device=dev)
        kept = torch.empty(max(K, 1), dtype=_I32, device=dev)
        hist = torch.zeros(64, TRIM_HIST_BINS, dtype=_I64, device=dev)
        if K:
            _hip_call("fa_hip_trim_emit", _p(roff), _p(ranks), _p(alive), F1, T, _p(cnt), _p(bases[0]), _p(bases[1]),
                      _p(nroff), _p(nranks), _p(kept), _p(hist), st)
        kept = kept[:K]
        nw = wrow[kept.to(_I64)].contiguous() if wrow is not None else None
        return kept, nroff, nranks[:nnz], nw, hist.sum(0)
    a = alive[ranks.to(_I64)].to(_I64)
    cs = torch.zeros(ranks.numel() + 1, dtype=_I64)
    torch.cumsum(a, 0, out=cs[1:])
    cnt = (cs[roff[1:]] - cs[roff[:-1]]).to(_I32)
    keep = cnt >= min_len
    if wrow is not None:
        keep &= wrow > 0
    kept = torch.nonzero(keep).flatten().to(_I32)
    K = kept.numel()
    nroff = torch.zeros(K + 1, dtype=_I64, device=dev)
    if K:
        torch.cumsum(cnt[kept.to(_I64)].to(_I64), 0, out=nroff[1:])
    nnz = int(nroff[-1].item())
    nranks = torch.empty(max(nnz, 1), dtype=_I32, device=dev)
    if K:
        lens = roff[1:] - roff[:-1]
        rowmask = torch.zeros(T, dtype=torch.bool)
        rowmask[kept.to(_I64)] = True
        em = torch.repeat_interleave(rowmask, lens) & (alive[ranks.to(_I64)] > 0)
        nranks[:nnz] = ranks[em]
    nw = wrow[kept.to(_I64)].contiguous() if wrow is not None else None
    hist = torch.bincount(cnt[kept.to(_I64)].to(_I64).clamp_(max=TRIM_HIST_BINS - 1),
                          minlength=TRIM_HIST_BINS) if K else torch.zeros(TRIM_HIST_BINS, dtype=_I64)
    return kept, nroff, nranks[:nnz], nw, hist


def slab_capacity(n_used: int, C: int) -> int:
    """Accumulator capacity (candidates per pass) of the slab kernel for n_used items
    (csrc/host/plan.cpp slab_width); 0 when no width fits."""
    for sw in (16, 32, 8, 4):     # plan.cpp slab_width order
        cap = int((TUNING.slab_lds_bytes - n_used * (sw + 2) * 8) // 4)
        if cap >= min(C, 8192) or (sw == 4 and cap >= 1024):
            return cap
    return 0


# TUNING.slab_cls: class layout of slab passes (plan.cpp cls_layout, k_count_slab_rec<..,
# kCls>): sibling prefixes share their first m-1 rows in registers; 0 disables it.
# TUNING.dense_min_rows (count_level): expected rows per slab of the rarest frequent prefix
# above which the slab kernel skips its all-zero-prefix test (0 disables).


def _level_plan_bound(F1: int, C: int, G: int, m: int) -> int:
    """int32 entries fa_level_plan may write: maps, gext, gpre, the slab kernel's piece
    tables and 48-B records."""
    return 2 * F1 + C + G * m + 14 * (G + C // 2 + 2) + (m + 16) * (G + C // 8 + 1) + 24


def level_plan_host(prefix: np.ndarray, ext_off: np.ndarray, ext: np.ndarray, F1: int, W: int,
                    lds_bytes: int | None = None, poff: np.ndarray | None = None, cls: int | None = None):
    """fa_level_plan on host arrays (tests / diagnostics): (rc, info, passes, buf)."""
    P, po, G, m = _flat_prefix(prefix, poff)
    C = int(ext.size)
    eo = np.ascontiguousarray(ext_off, dtype=np.int64)
    ex = np.ascontiguousarray(ext, dtype=np.int32)
    params = _plan_params(lds_bytes or TUNING.slab_lds_bytes, W, TUNING.slab_cls if cls is None else cls)
    bound = _level_plan_bound(F1, C, G, m)
    passes = np.zeros((G + C + 2, 3), np.int64)
    info = np.zeros(24, np.int64)
    while True:
        buf = np.zeros(bound, np.int32)
        rc = _native.host().fa_level_plan(P.ctypes.data, po.ctypes.data, G, eo.ctypes.data, ex.ctypes.data, F1,
                                          params.ctypes.data, buf.ctypes.data, bound, passes.ctypes.data,
                                          passes.shape[0], info.ctypes.data)
        if rc != 3:
            break
        bound *= 2    # class layouts pad their passes with idle slots
    return rc, info, passes[:int(info[6])], buf[:int(info[18])]


def _plan_params(lds_bytes: int, W: int, cls: int) -> np.ndarray:
    """fa_level_plan's params (plan.cpp): LDS bytes, bitmap words, accumulator bytes,
    class layout (0: off, 1: by the wave-step read model, 2: always)."""
    return np.array([lds_bytes, W, 4.0, cls], dtype=np.float64)


def emulate_level_plan(bits_by_rank: np.ndarray, info, passes, buf, m: int, C: int) -> np.ndarray:
    """CPU model of the slab kernel over the plan written by fa_level_plan;
    bits_by_rank: bool [F1, ncols]."""
    n_used = int(info[3])
    used = buf[info[13]:info[13] + n_used]
    bits = bits_by_rank[used]
    gext = buf[info[14]:info[14] + C]
    out = np.zeros(C, np.int64)
    npc = int(info[4])
    gpre = buf[info[15]:info[16]]
    loc = buf[info[16]:info[16] + 2 * npc].reshape(-1, 2)
    gpm = buf[info[19]:info[19] + 2 * npc].reshape(-1, 2)
    for a, b, e0 in passes.tolist():
        for pi in range(a, b):
            p = np.logical_and.reduce(bits[gpre[gpm[pi, 0]:gpm[pi, 0] + gpm[pi, 1]]])
            for e in range(loc[pi, 0], loc[pi, 1]):
                out[e0 + e] += int((p & bits[gext[e0 + e]]).sum())
    return out


def emulate_slab_records(bits_by_rank: np.ndarray, info, passes, buf, C: int) -> np.ndarray:
    """CPU model of k_count_slab_rec over the 48-B piece records of a slab plan
    (fa_level_plan info[20]); must equal emulate_level_plan."""
    used = buf[info[13]:info[13] + int(info[3])]
    bits = bits_by_rank[used]
    gpre = buf[info[15]:info[16]]
    rec = buf[info[20]:info[20] + 12 * int(info[4])].view(np.uint32).reshape(-1, 12)
    u16 = np.stack([rec & 0xFFFF, rec >> 16], axis=-1).reshape(-1, 24)   # 24 u16 per record
    out = np.zeros(C, np.int64)
    for a, b, e0 in passes.tolist():
        # slot s = step (s - a) // 1024 of thread (s - a) % 1024; class-layout flags
        # (bit 17: keep q = AND of the first m-1 rows, bit 18: keep p) refer to the
        # thread's previous slot
        for t in range(min(1024, b - a)):
            q = p = None
            for pi in range(a + t, b, 1024):
                r = rec[pi]
                n_ext, m, long_pre = int(r[1] & 0xFF), int((r[1] >> 8) & 0xFF), bool((r[1] >> 16) & 1)
                fl = int((r[1] >> 17) & 3)
                if long_pre:
                    ids = gpre[int(r[8]):int(r[8]) + m]
                else:
                    ids = np.concatenate([u16[pi, 4:8], u16[pi, 16:24]])[:m]
                if not fl & 1:
                    q = np.logical_and.reduce(bits[ids[:m - 1]])
                if not fl & 2:
                    p = q & bits[ids[m - 1]]
                for k in range(n_ext):
                    out[e0 + int(r[0]) + k] += int((p & bits[u16[pi, 8 + k]]).sum())
    return out


LAST_LEVEL_PLAN: dict = {}   # shape of the last count_level call (diagnostics)
CLS_LEVELS = [0]             # count_level calls that ran the class layout (diagnostics, tests)


def _slab_map_lds(F1: int) -> int:
    """LDS bytes of k_count_slab_rec's u16 rank -> slab-row map (plan.cpp fa_slab_map_lds)."""
    return ((F1 * 2 + 15) & ~15) if F1 <= 8192 else 0


def _flat_prefix(prefix: np.ndarray, poff: np.ndarray | None):
    if poff is None:
        P = np.ascontiguousarray(prefix, dtype=np.int32)
        G, m = P.shape
        return P.reshape(-1), np.arange(G + 1, dtype=np.int64) * m, G, m
    poff = np.ascontiguousarray(poff, dtype=np.int64)
    G = poff.size - 1
    return np.ascontiguousarray(prefix, dtype=np.int32).reshape(-1), poff, G, int(np.diff(poff).max(initial=0))


def count_level(roff, ranks, src, ncols: int, F1: int, prefix: np.ndarray, ext_off: np.ndarray, ext: np.ndarray,
                wword, kernel: str = "auto", poff: np.ndarray | None = None, full_bm=None,
                sup_frac: float = 0.0) -> torch.Tensor | None:
    """Support counts of one level on the device: one native planning call
    (csrc/host/plan.cpp fa_level_plan: used items, slab width, pieces, accumulator
    passes, class layout) into one pinned buffer, one host->device copy, then the
    slab kernel (k_count_slab_rec) per pass.

    kernel: accepted for compatibility ("auto" | "slab": both the slab kernel).
    prefix: int32 [G, m], or (poff given) a flat int32 array with group g's
    prefix at poff[g]:poff[g+1] — groups of several levels (k) in one launch.
    full_bm: optional callable(used ranks) returning (bitmap, rank -> bitmap row map
    or None for a rank-indexed bitmap) of the current row layout, holding at least
    the used items' rows (built once, shared by the multi-pass levels until the rows
    change); without it a used-item bitmap is built for each multi-pass level.
    sup_frac: the minimum support as a fraction of the rows; when every frequent prefix
    then expects >= 4 rows per slab (e^-4: ~2 % of a slab's prefixes empty at worst), the
    slab kernel drops its all-zero-prefix test (TUNING.dense_min_rows).
    Returns int64 counts [C] (ext order), or None when no LDS slab fits (the
    caller then uses the bitmap kernel)."""
    dev = ranks.device
    C = int(ext.size)
    if C == 0:
        return torch.zeros(0, dtype=_I64, device=dev)
    P, po, G, m = _flat_prefix(prefix, poff)
    eo = np.ascontiguousarray(ext_off, dtype=np.int64)
    ex = np.ascontiguousarray(ext, dtype=np.int32)
    W = (ncols + 63) // 64
    # the class layout has no weighted (dedup) kernel: unit weights only
    params = _plan_params(TUNING.slab_lds_bytes, W, TUNING.slab_cls if wword is None else 0)
    bound = _level_plan_bound(F1, C, G, m)
    on_gpu = dev.type == "cuda"
    stage = pinned_stage("level_plan") if on_gpu else None
    max_pass = G + C + 2
    passes = np.zeros((max_pass, 3), dtype=np.int64)
    info = np.zeros(24, dtype=np.int64)
    while True:
        buf = stage.get(4 * bound).view(dtype=_I32) if on_gpu else torch.empty(bound, dtype=_I32)
        rc = _native.host().fa_level_plan(P.ctypes.data, po.ctypes.data, G, eo.ctypes.data, ex.ctypes.data, F1,
                                          params.ctypes.data, buf.data_ptr(), bound, passes.ctypes.data, max_pass,
                                          info.ctypes.data)
        if rc != 3:
            break
        bound *= 2    # class layouts pad their passes with idle slots
    if rc == 4:
        return None
    if rc != 0:
        raise RuntimeError(f"fa_level_plan failed ({rc})")
    sw, cap, n_used, npass = int(info[1]), int(info[2]), int(info[3]), int(info[6])
    total = int(info[18])
    dbuf = buf[:total].to(dev, non_blocking=True)
    if on_gpu:
        stage.event = torch.cuda.Event()
        stage.event.record()
    base = dbuf.data_ptr()
    passes = passes[:npass]
    o_im, o_used, o_gpre, o_rec = (int(info[i]) for i in (12, 13, 15, 20))
    out = torch.zeros(C, dtype=_I32, device=dev)
    bm, bm_rows = None, None
    if npass > 1:
        if full_bm is not None:
            bm, bmap = full_bm(buf[o_used:o_used + n_used].numpy().copy())
            if bmap is None:
                bm_rows = base + 4 * o_used         # slab row u -> bitmap row used[u]
            else:
                rows_t = bmap[dbuf[o_used:o_used + n_used].to(_I64)]   # slab row u -> bitmap row of used[u]
                bm_rows = rows_t.data_ptr()
        else:
            bm, _ = build_bitmaps(roff, ranks, src, ncols, n_used, dbuf[o_im:o_im + F1],
                                  dbuf[o_used:o_used + n_used])
    st = _stream(ranks)
    bounds = passes[:, 2].tolist() + [C]
    nslabs = (W + sw - 1) // sw
    dense = wword is None and TUNING.dense_min_rows > 0 and sup_frac * sw * 64 >= TUNING.dense_min_rows
    for q, (a, b, e0) in enumerate(passes.tolist()):
        Cq = bounds[q + 1] - e0
        # piece records (k_count_slab_rec): 48 B per piece, loaded one piece ahead
        lds = n_used * (sw + 2) * 8 + Cq * 4 + _slab_map_lds(F1)
        n_wg = int(max(1, min(nslabs, 256 * min(max(1, TUNING.slab_lds_bytes // lds), 2))))
        _hip_call("fa_hip_count_slab_rec_cls", _p(roff), _p(ranks), _p(src), ncols, base + 4 * o_im, F1,
                  n_used, base + 4 * o_gpre, base + 4 * (o_rec + 12 * a), b - a, Cq, _p(wword),
                  out.data_ptr() + 4 * e0, sw, n_wg, _p(bm), bitmap_ld(bm), st,
                  bm_rows, None, int(info[23]) | (2 if dense else 0))
    CLS_LEVELS[0] += int(info[23])
    LAST_LEVEL_PLAN.clear()
    LAST_LEVEL_PLAN.update(kernel="slab", rows=int(roff.numel() - 1), used=n_used, sw=sw,
                           cap=cap, passes=npass, pieces=int(info[4]), slab_reads=int(info[10]), m=m, C=C,
                           cls=int(info[23]), step_reads=int(info[21]), step_reads_cls=int(info[22]),
                           dense=bool(dense))
    return out.to(_I64)


AG_DEVICE_MAX_F1 = 32768  # device apriori-gen: up to 8 bitset words per lane of a 64-lane wave (gen.hip)


def ag_mark_words(F1: int) -> int:
    """u32 words of the chain's used-item bitset (gen.hip ag_mark_words)."""
    return max(128, (F1 + 31) // 32)

# Device -> host fallbacks taken by the current phase (a mining run or a rules
# phase clears the list when it starts, reset_fallbacks(), and reports what it
# holds when it ends, so a run never re-reports an earlier run's fallbacks).
# Each distinct message is printed on stderr once per process.
FALLBACKS: list = []
_PRINTED: set = set()


def reset_fallbacks() -> None:
    FALLBACKS.clear()


def note_fallback(what: str) -> None:
    if what not in FALLBACKS:
        FALLBACKS.append(what)
    if what not in _PRINTED:
        _PRINTED.add(what)
        import sys
        print(f"fastapriori_amd: {what}", file=sys.stderr, flush=True)


_GEN_WS: dict = {}


def apriori_gen_device(prev: np.ndarray, F1: int, dev, want_rows: bool = False):
    """apriori-gen on the GPU (csrc/hip/gen.hip fa_hip_ag_gen: one native call, two
    stream syncs): (prefix_idx int32 [G], ext_off int64 [G+1], ext int32 [C]) as
    ops.host.apriori_gen, plus the candidate rows int32 [C, m+1] when want_rows."""
    n, m = prev.shape
    P = pinned_stage("gen").h2d(np.ascontiguousarray(prev, dtype=np.int32), dev)
    st = _stream(P)
    sizes = np.zeros(2, dtype=np.int64)
    host_stage = pinned_stage("gen_out")
    need_host = n + 8 * n * (m + 2) + 1024
    for _ in range(4):
        ws = _GEN_WS.get(dev)
        host = host_stage.get(4 * need_host).view(dtype=_I32)
        rc = _native.hip().fa_hip_ag_gen(_p(P), n, m, F1, _p(ws), ws.numel() if ws is not None else 0,
                                         host.data_ptr(), host.numel(), sizes.ctypes.data, st)
        if rc == 5:
            _GEN_WS[dev] = torch.empty(int(sizes[1] * 1.5) + (1 << 20), dtype=torch.uint8, device=dev)
            continue
        if rc == 6:
            need_host = int(sizes[1] * 1.5) + 1024
            continue
        _native.check(rc, "fa_hip_ag_gen")
        break
    else:
        raise RuntimeError("fa_hip_ag_gen: workspace sizing did not converge")
    C = int(sizes[0])
    h = host.numpy()
    cnt_h = h[:n]
    prefix_idx = np.flatnonzero(cnt_h).astype(np.int32)
    ext_off = np.zeros(prefix_idx.size + 1, dtype=np.int64)
    np.cumsum(cnt_h[prefix_idx], out=ext_off[1:])
    ext_h = h[n:n + C].copy()
    if want_rows:
        return prefix_idx, ext_off, ext_h, h[n + C:n + C + C * (m + 1)].reshape(C, m + 1).copy()
    return prefix_idx, ext_off, ext_h


def apriori_gen_chain(rows: np.ndarray, F1: int, dev, max_levels: int, growth: float, total0: int,
                      tmax: int, first_free: bool = False) -> list:
    """Speculative levels for bundling in one native call (csrc/hip/gen.hip fa_hip_ag_chain):
    level m+1 candidates from ``rows`` (int32 [n, m], level k's candidate rows), then
    m+2 from those, ... while each level is non-empty, grows at most ``growth`` x
    and the bundle total stays <= ``tmax``.  Returns [(prefix_idx, ext_off, ext,
    rows), ...] per accepted level, as apriori_gen_device.

    first_free: ``rows`` is F_{k-1}; the first level (level k's candidates) is always
    returned, and the bundle limit comes from its used items on the device (the
    whole of apriori-gen + bundle planning in one call)."""
    n, m = rows.shape
    if n == 0 or max_levels <= 0:
        return []
    P = pinned_stage("gen").h2d(np.ascontiguousarray(rows, dtype=np.int32), dev)
    st = _stream(P)
    sizes = np.zeros(2 + max_levels, dtype=np.int64)
    host_stage = pinned_stage("gen_out")
    need_host = 1 << 20
    for _ in range(32):
        ws = _GEN_WS.get(dev)
        if ws is None or ws.numel() < (64 << 20):
            ws = _GEN_WS[dev] = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
        host = host_stage.get(4 * need_host).view(dtype=_I32)
        rc = _native.hip().fa_hip_ag_chain(_p(P), n, m, F1, _p(ws), ws.numel(), host.data_ptr(), host.numel(),
                                           max_levels, growth, total0, tmax, sizes.ctypes.data, st,
                                           int(first_free), float(TUNING.slab_lds_bytes))
        if rc == 5:
            _GEN_WS[dev] = torch.empty(int(sizes[1]), dtype=torch.uint8, device=dev)
            continue
        if rc == 6:
            need_host = int(sizes[1])
            continue
        _native.check(rc, "fa_hip_ag_chain")
        break
    else:
        raise RuntimeError("fa_hip_ag_chain: buffer sizing did not converge")
    h = host.numpy()
    out, o = [], (ag_mark_words(F1) if first_free else 0)
    for lv in range(int(sizes[0])):
        C = int(sizes[2 + lv])
        cnt_h = h[o:o + n]
        prefix_idx = np.flatnonzero(cnt_h).astype(np.int32)
        ext_off = np.zeros(prefix_idx.size + 1, dtype=np.int64)
        np.cumsum(cnt_h[prefix_idx], out=ext_off[1:])
        ext_h = h[o + n:o + n + C].copy()
        nxt = h[o + n + C:o + n + C + C * (m + 1)].reshape(C, m + 1).copy()
        out.append((prefix_idx, ext_off, ext_h, nxt))
        o += n + C + C * (m + 1)
        n, m = C, m + 1
    return out


def slab_total_limit(n_used: int) -> int:
    """Largest bundle total t with t <= slab_capacity(n_used, t) (monotone in t)."""
    lo, hi = 0, 1 << 31
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if mid <= slab_capacity(n_used, mid):
            lo = mid
        else:
            hi = mid - 1
    return lo


RECOMMEND_INDEX_MIN_RULES = 2048


def recommend_index(ante_off: torch.Tensor, ante: torch.Tensor, F1: int):
    """Rule lists per item for k_recommend_indexed: rule r is listed under the last
    (highest-rank) item of its antecedent, ids ascending.  -> (list_off int64 [F1+1],
    list_rule int32 [R])."""
    key = ante[ante_off[1:] - 1].to(_I64)
    order = torch.argsort(key, stable=True).to(_I32)
    list_off = torch.zeros(F1 + 1, dtype=_I64, device=ante.device)
    torch.cumsum(torch.bincount(key, minlength=F1), 0, out=list_off[1:])
    return list_off, order


def recommend(ante_off, ante, cons, F1: int, boff, bask, index=None) -> torch.Tensor:
    """First-match recommendation per basket -> int32 rank (or -1 for "0").

    ``index``: (list_off, list_rule) from recommend_index — the per-item rule
    lists that let a basket skip rules whose antecedent cannot be inside it."""
    M = boff.numel() - 1
    R = cons.numel()
    dev = bask.device
    out = torch.full((max(M, 0),), -1, dtype=_I32, device=dev)
    if M <= 0 or R == 0:
        return out
    if bask.is_cuda:
        if index is not None:
            rc = _native.hip().fa_hip_recommend_indexed(_p(index[0]), _p(index[1]), _p(ante_off), _p(ante),
                                                        _p(cons), R, F1, _p(boff), _p(bask), M, _p(out),
                                                        _stream(bask))
        else:
            rc = _native.hip().fa_hip_recommend(_p(ante_off), _p(ante), _p(cons), R, F1, _p(boff), _p(bask), M,
                                                _p(out), _stream(bask))
        if rc == 2:  # vocabulary too wide for an LDS bitset: host path
            note_fallback(f"recommendation on the host: F1 = {F1} frequent items exceed the kernel's LDS basket "
                          "bitset (64 KiB)")
            return recommend(ante_off.cpu(), ante.cpu(), cons.cpu(), F1, boff.cpu(), bask.cpu()).to(dev)
        _native.check(rc, "fa_hip_recommend")
        return out
    _native.host().fa_recommend_cpu(_p(ante_off), _p(ante), _p(cons), R, F1, _p(boff), _p(bask), M, _p(out),
                                    num_threads())
    return out


def rules_build_device(levels: list, counts: list, tie_pos: np.ndarray, dev) -> dict:
    """Association rules on the GPU (csrc/hip/rules.hip; AssociationRules.scala:116-182).

    levels[k-1]: int32 [n_k, k] lexicographically sorted itemsets, counts[k-1] their
    supports.  Returns device tensors ante_off int64 [R+1], ante int32, cons int32 [R],
    conf float64 [R] in recommendation order, plus level_stats [(antecedent size,
    before cut, after cut)] — the same table as the host builder (ops.host.rules_build).
    """
    K = len(levels)
    empty = dict(ante_off=torch.zeros(1, dtype=_I64, device=dev), ante=torch.zeros(0, dtype=_I32, device=dev),
                 cons=torch.zeros(0, dtype=_I32, device=dev), conf=torch.zeros(0, dtype=torch.float64, device=dev),
                 level_stats=[], level_ms=[])
    if K < 2 or len(levels[1]) == 0:
        return empty
    lv = [np.ascontiguousarray(l, dtype=np.int32).reshape(-1) for l in levels]
    base = np.zeros(K + 2, dtype=np.int64)            # base[m]: offset of the size-m level
    np.cumsum([l.size for l in lv], out=base[2:K + 2])
    rows_all = torch.from_numpy(np.concatenate(lv)).to(dev)
    cbase = np.zeros(K + 1, dtype=np.int64)
    np.cumsum([len(c) for c in counts], out=cbase[1:])
    cnt_all = torch.from_numpy(np.concatenate([np.asarray(c, dtype=np.int64) for c in counts])).to(dev)
    st = _stream(rows_all)
    lib = _native.hip()

    def rows(m):
        return rows_all.data_ptr() + int(base[m]) * 4

    def cnts(m):
        return cnt_all.data_ptr() + int(cbase[m - 1]) * 8

    kept_prev = conf_prev = None
    parts = []          # per level: (flat rule ids kept, conf, sub)
    stats = []
    level_ms = []       # wall ms of each level's generation + cut (the nonzero readback syncs)
    for k in range(2, K + 1):
        nS, nA = len(levels[k - 1]), len(levels[k - 2])
        if nS == 0:
            break
        t_lv = time.perf_counter()
        sub = torch.empty(nS * k, dtype=_I32, device=dev)
        conf = torch.empty(nS * k, dtype=torch.float64, device=dev)
        _native.check(lib.fa_hip_rule_gen(rows(k), nS, k, rows(k - 1), nA, cnts(k), cnts(k - 1), _p(sub), _p(conf),
                                          st), "fa_hip_rule_gen")
        if k == 2:
            kept = torch.ones(nS * k, dtype=torch.uint8, device=dev)
        else:
            kept = torch.empty(nS * k, dtype=torch.uint8, device=dev)
            _native.check(lib.fa_hip_rule_cut(_p(sub), _p(conf), nS, k, _p(kept_prev), _p(conf_prev), _p(kept), st),
                          "fa_hip_rule_cut")
        ids = torch.nonzero(kept).flatten()
        parts.append((k, ids, conf, sub))
        stats.append((k - 1, nS * k, ids.numel()))
        level_ms.append((time.perf_counter() - t_lv) * 1e3)
        kept_prev, conf_prev = kept, conf
    conf_r = torch.cat([c[i] for _, i, c, _ in parts])
    R = conf_r.numel()
    if R == 0:
        return dict(empty, level_stats=stats, level_ms=level_ms)
    cons_r = torch.cat([rows_all[int(base[k]):int(base[k + 1])][i] for k, i, _, _ in parts])
    ante_idx = torch.cat([s[i] for _, i, _, s in parts])
    msz = torch.cat([torch.full((i.numel(),), k - 1, dtype=_I32, device=dev) for k, i, _, _ in parts])
    tie = torch.from_numpy(np.ascontiguousarray(tie_pos, dtype=np.int64)).to(dev)[cons_r.to(_I64)]
    # total order: conf desc, consequent tie position, antecedent size, antecedent index
    key = (msz.to(_I64) << 32) | ante_idx.to(_I64)
    if len(tie_pos) < (1 << 24) and K < 128:
        key = key | (tie << 39)
        o = torch.argsort(key)
    else:
        o = torch.argsort(key)
        o = o[torch.argsort(tie[o], stable=True)]
    o = o[torch.sort(conf_r[o], descending=True, stable=True)[1]]
    msz_s, idx_s = msz[o].contiguous(), ante_idx[o].contiguous()
    ante_off = torch.zeros(R + 1, dtype=_I64, device=dev)
    torch.cumsum(msz_s.to(_I64), 0, out=ante_off[1:])
    nante = int(ante_off[-1].item())
    ante = torch.empty(nante, dtype=_I32, device=dev)
    base_t = torch.from_numpy(base).to(dev)
    _native.check(lib.fa_hip_rule_emit(_p(rows_all), _p(base_t), _p(msz_s), _p(idx_s), _p(ante_off), R, _p(ante), st),
                  "fa_hip_rule_emit")
    return dict(ante_off=ante_off, ante=ante, cons=cons_r[o].contiguous(), conf=conf_r[o].contiguous(),
                level_stats=stats, level_ms=level_ms)


def _device_lines(buf: torch.Tensor, n: int, last_is_term: bool):
    """Line ends of n file bytes in HBM and per-line upper-bound slots of (len + 1) / 2
    ids: (ends int64 [nl], nl, bound_off int64 [nl + 1], total slots)."""
    dev = buf.device
    st = _stream(buf)
    lib = _native.hip()
    tiles = int(lib.fa_hip_parse_tiles(n))
    tile_cnt = torch.empty(tiles, dtype=_I32, device=dev)
    _native.check(lib.fa_hip_line_count(_p(buf), n, _p(tile_cnt), st), "fa_hip_line_count")
    tile_base = torch.zeros(tiles + 1, dtype=_I64, device=dev)
    torch.cumsum(tile_cnt, 0, out=tile_base[1:])
    n_term = int(tile_base[-1].item())
    nl = n_term + (0 if last_is_term else 1)
    ends = torch.empty(max(nl, 1), dtype=_I64, device=dev)
    _native.check(lib.fa_hip_line_ends(_p(buf), n, _p(tile_base), _p(ends), st), "fa_hip_line_ends")
    if not last_is_term:
        ends[n_term] = n
    ends = ends[:nl]
    starts = torch.empty_like(ends)
    starts[0] = 0
    starts[1:] = ends[:-1] + 1
    bound = torch.clamp((ends - starts + 1) // 2, min=1)
    bound_off = torch.zeros(nl + 1, dtype=_I64, device=dev)
    torch.cumsum(bound, 0, out=bound_off[1:])
    return ends, nl, bound_off, int(bound_off[-1].item())


def _compact_lines(scratch, xscratch, bound_off, dcnt, xcnt, nl, st):
    dev = scratch.device
    off = torch.zeros(nl + 1, dtype=_I64, device=dev)
    torch.cumsum(dcnt, 0, out=off[1:])
    xoff = torch.zeros(nl + 1, dtype=_I64, device=dev)
    torch.cumsum(xcnt, 0, out=xoff[1:])
    n_items, n_extras = (int(v) for v in torch.stack([off[-1], xoff[-1]]).cpu().tolist())
    items = torch.empty(n_items, dtype=_I32, device=dev)
    extras = torch.empty(n_extras, dtype=_I32, device=dev)
    _native.check(_native.hip().fa_hip_compact_lines(_p(scratch), _p(xscratch), _p(bound_off), _p(dcnt), _p(xcnt),
                                                     _p(off), _p(xoff), nl, _p(items), _p(extras), st),
                  "fa_hip_compact_lines")
    return off, items, extras


PARSE_HIST_CAP = None       # kHistCap of the tile parser's fused F1 histogram (parse.hip)


def parse_hist_cap() -> int:
    global PARSE_HIST_CAP
    if PARSE_HIST_CAP is None:
        PARSE_HIST_CAP = int(_native.hip().fa_hip_tparse_hist_cap())
    return PARSE_HIST_CAP


class TileParse:
    """The tile parser's per-region steps (csrc/hip/parse.hip k_tline_count,
    k_tparse, k_tcompact), all queued on one stream.  Line counts come either
    from a device scan with one readback (whole shard) or from the host's count
    of the region's '\n' bytes (streamed regions: no readback at all).  Items of
    every region are written at a device-side running offset into one buffer
    sized by the upper bound (bytes + 1) / 2; the F1 histogram (items and repeats,
    ids < parse_hist_cap()) accumulates per compaction block."""

    GRID = 1024       # compaction workgroups (rows of the histogram partials): 4 per CU

    def __init__(self, buf: torch.Tensor, n: int, dev, scratch_bytes: int, xcap: int | None = None):
        self.buf, self.n, self.dev = buf, n, dev
        self.st = _stream(buf)
        self.lib = _native.hip()
        cap = parse_hist_cap()
        tok_cap = (n + 1) // 2 + 1           # tokens are separated: at most (bytes + 1) / 2
        self.items = torch.empty(tok_cap, dtype=_I32, device=dev)
        # repeated ids are rare: a small buffer, and a second parse in the rare file that overflows it
        self.xcap = max(int(xcap if xcap is not None else n // 64 + 4096), 1)
        self.extras = torch.empty(self.xcap, dtype=_I32, device=dev)
        self.hpart = torch.zeros(self.GRID * cap, dtype=_I64, device=dev)
        self.flags = torch.zeros(4, dtype=_I32, device=dev)
        self.cursor = torch.zeros(2, dtype=_I64, device=dev)     # items, repeats written so far
        self.offs = []                                           # per region: int64 line offsets
        self.scratch_ids = scratch_bytes // 2 + 2
        self.scratch = torch.empty(self.scratch_ids, dtype=_I32, device=dev)
        self.xscratch = torch.empty(self.scratch_ids, dtype=_I32, device=dev)
        self.n_lines = 0

    def region(self, lo: int, hi: int, n_lines: int | None, tail: bool) -> None:
        """Lines of bytes [lo, hi): lo is a line start, hi follows a terminator (or
        is the shard end; tail: its last byte is no terminator, so one more line
        ends at hi).  n_lines: the region's lines when the host knows them (else one
        readback of the device count).  Five launches, no host synchronisation:
        line ends per tile, their scan, the parse, the scan of the tiles' id totals
        (from the running cursor) and the compaction."""
        lib, st, dev = self.lib, self.st, self.dev
        if hi <= lo:
            return
        if (hi - lo) // 2 + 1 > self.scratch_ids:
            # a region past the planned size (long lines carried over, or the final region
            # after a '\r'): larger slots; the old ones are freed in stream order
            self.scratch_ids = (hi - lo) // 2 + 2
            self.scratch = torch.empty(self.scratch_ids, dtype=_I32, device=dev)
            self.xscratch = torch.empty(self.scratch_ids, dtype=_I32, device=dev)
        tiles = int(lib.fa_hip_tparse_tiles(lo, hi))
        tile_cnt = torch.empty(tiles, dtype=_I32, device=dev)
        _native.check(lib.fa_hip_tline_count(_p(self.buf), lo, hi, _p(tile_cnt), st), "fa_hip_tline_count")
        tile_base = torch.empty(tiles + 1, dtype=_I64, device=dev)
        _native.check(lib.fa_hip_scan_small(1, _p(tile_cnt), tiles, _p(tile_base), None, st), "fa_hip_scan_small")
        if n_lines is None:
            n_lines = int(tile_base[-1].item()) + (1 if tail else 0)
        nl = n_lines
        if nl == 0:
            return
        dcnt = torch.empty(nl, dtype=_I32, device=dev)
        xcnt = torch.empty(nl, dtype=_I32, device=dev)
        lbase = torch.empty(nl, dtype=_I64, device=dev)
        tile_dx = torch.empty(2 * tiles, dtype=_I32, device=dev)
        _native.check(lib.fa_hip_tparse(_p(self.buf), self.buf.numel(), lo, hi, int(bool(tail)), lo,
                                        _p(tile_base), _p(dcnt), _p(xcnt), _p(lbase), _p(self.scratch),
                                        _p(self.xscratch), _p(tile_dx), _p(self.flags), st), "fa_hip_tparse")
        tile_xb = torch.empty(2 * (tiles + 1), dtype=_I64, device=dev)
        _native.check(lib.fa_hip_scan_small(2, _p(tile_dx), tiles, _p(tile_xb), _p(self.cursor), st),
                      "fa_hip_scan_small")
        off = torch.empty(nl, dtype=_I64, device=dev)
        grid = max(1, min(self.GRID, tiles))
        _native.check(lib.fa_hip_tcompact(_p(tile_base), _p(tile_xb), tiles, int(bool(tail)), _p(dcnt), _p(xcnt),
                                          _p(lbase),
                                          _p(self.scratch), _p(self.xscratch), _p(self.items), _p(self.extras),
                                          self.xcap, _p(off), grid, _p(self.hpart), _p(self.flags), st),
                      "fa_hip_tcompact")
        self.offs.append(off)
        self.n_lines += nl

    def finish(self):
        """(offsets int64 [nl+1], items, extras, vocab size, hist int64 [V] or None), None
        when a token is not canonical numeric, or the number of repeated ids when they
        overflowed the repeat buffer (parse again with that room).  One readback."""
        dev = self.dev
        tail = torch.cat([self.cursor, self.flags.to(_I64)]).cpu().tolist()
        n_items, n_extras, bad, mx, over, xover = (int(v) for v in tail)
        if bad & 1:
            return None
        if xover:
            return n_extras
        off = torch.cat(self.offs + [self.cursor[:1]]) if self.offs else torch.zeros(1, dtype=_I64, device=dev)
        V = mx + 1 if self.n_lines else 0       # no lines: an empty vocabulary (as the host parser)
        hist = None
        if not over:
            cap = parse_hist_cap()
            hist = torch.empty(cap, dtype=_I64, device=dev)
            _native.check(self.lib.fa_hip_hist_reduce(_p(self.hpart), self.GRID, _p(hist), self.st),
                          "fa_hip_hist_reduce")
            hist = hist[:V]
        return off, self.items[:n_items], self.extras[:n_extras], V, hist


def parse_numeric_device(buf: torch.Tensor, n: int, last_is_term: bool):
    """Parse n file bytes already in HBM (csrc/hip/parse.hip tile parser).  ``buf`` is
    uint8, padded with >= 64 zero bytes past a multiple of 64.  Returns (offsets
    int64 [nl+1], items int32, extras int32, vocab size, F1 histogram int64 [V] or
    None), all on the device except the vocab size, or None when a token is not
    canonical numeric (-> dictionary mode)."""
    dev = buf.device
    if n <= 0:
        return (torch.zeros(1, dtype=_I64, device=dev), torch.zeros(0, dtype=_I32, device=dev),
                torch.zeros(0, dtype=_I32, device=dev), 0, None)
    assert buf.numel() >= (n + 63) // 64 * 64 + 64 and buf.dtype == torch.uint8
    xcap = None
    for _ in range(2):
        tp = TileParse(buf, n, dev, n, xcap)
        tp.region(0, n, None, tail=not last_is_term)
        got = tp.finish()
        if not isinstance(got, int):
            return got
        xcap = got                     # every repeated id, counted by the first pass
    raise RuntimeError("device parser: repeat buffer overflow on the second pass")


def parse_dict_device(buf: torch.Tensor, n: int, last_is_term: bool):
    """Dictionary-mode parse of n file bytes in HBM (k_parse_lines_dict): token ids
    from a device hash table keyed by the parser's 64-bit token hash, then dense ids
    in hash order.  Returns (offsets, items, extras, hashes uint64 np [V], first-
    occurrence byte offsets int64 np [V], lengths int32 np [V]) or None when the
    table overflows or two distinct tokens share a hash (k_dict_verify; -> host parser)."""
    dev = buf.device
    st = _stream(buf)
    lib = _native.hip()
    if n <= 0:
        return None
    ends, nl, bound_off, nb = _device_lines(buf, n, last_is_term)
    # distinct tokens <= tokens <= n / 2; the table holds them at <= 50 % load
    cap = 1 << 20
    while cap < min(n, 1 << 30):
        cap <<= 1
    cap = min(cap, 1 << 28)
    keys = torch.zeros(cap, dtype=_I64, device=dev)
    tpos = torch.empty(cap, dtype=_I64, device=dev)
    tlen = torch.empty(cap, dtype=_I32, device=dev)
    scratch = torch.empty(nb, dtype=_I32, device=dev)
    xscratch = torch.empty(nb, dtype=_I32, device=dev)
    dcnt = torch.empty(nl, dtype=_I32, device=dev)
    xcnt = torch.empty(nl, dtype=_I32, device=dev)
    flags = torch.zeros(2, dtype=_I32, device=dev)
    _native.check(lib.fa_hip_parse_lines_dict(_p(buf), _p(ends), nl, _p(bound_off), _p(scratch), _p(xscratch),
                                              _p(dcnt), _p(xcnt), _p(flags), _p(keys), _p(tpos), _p(tlen), cap, st),
                  "fa_hip_parse_lines_dict")
    # identity check: tokens sharing a 64-bit hash would share an id (flags |= 4)
    _native.check(lib.fa_hip_dict_verify(_p(buf), _p(ends), nl, _p(flags), _p(keys), _p(tpos), _p(tlen), cap, st),
                  "fa_hip_dict_verify")
    if int(flags[0].item()) & 6:
        return None
    off, items, extras = _compact_lines(scratch, xscratch, bound_off, dcnt, xcnt, nl, st)
    occ = keys != 0
    slot_id = (torch.cumsum(occ.to(_I32), 0, dtype=_I32) - 1).contiguous()
    for t in (items, extras):
        _native.check(lib.fa_hip_slot_remap(_p(t), t.numel(), _p(slot_id), st), "fa_hip_slot_remap")
    sel = torch.nonzero(occ).flatten()
    hashes = keys[sel].cpu().numpy().view(np.uint64)
    return off, items, extras, hashes, tpos[sel].cpu().numpy(), tlen[sel].cpu().numpy()


# ---------------------------------------------------------------------------
# Device-resident level bundles (csrc/hip/gen.hip fa_hip_dl_level0 / fa_hip_dl_more,
# csrc/hip/levels.hip fa_hip_dl_plan / fa_hip_dl_threshold; driven by
# models.apriori.FastApriori._mine_device)
# ---------------------------------------------------------------------------
DL_CTL = 1024           # gen.hip kDlCtl
DL_BITS = 512           # gen.hip kDlBits: the control block's used-item bitset (ctl[512:1024])
DL_EMPTY = 104          # gen.hip kDlEmpty: the chain stopped on a level without candidates
DL_MAX_F1 = 32768       # its bits (and the generator's 8 bitset words per lane)
DL_MAX_M = 40           # levels.hip kDlMaxM (prefixes past 12 ids go through gpre)
DL_MAX_LEVELS = 31


class DlPostC(ctypes.Structure):
    """gen.hip DlPost: what fa_hip_dl_more queues right after its synchronisation
    (device plan, trimming decision, slab count) without returning to Python first."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("item_map", "rec", "part", "out")] + \
               [(n, ctypes.c_int64) for n in ("rec_cap", "part_cap", "out_cap")] + \
               [(n, ctypes.c_void_p) for n in ("roff", "ranks", "src", "wword")] + \
               [("ncols", ctypes.c_int64), ("lds_kernel", ctypes.c_double), ("lds_budget", ctypes.c_double)] + \
               [(n, ctypes.c_void_p) for n in ("c1", "alive", "len_hist")] + \
               [(n, ctypes.c_int64) for n in ("T", "nnz", "trim_min_rows", "trim_ok", "k",
                                               "done", "sw", "cap", "n_wg", "C", "trim")] + \
               [("gpre", ctypes.c_void_p), ("gpre_cap", ctypes.c_int64), ("accb", ctypes.c_double)] + \
               [("trim_rows_frac", ctypes.c_double), ("trim_nnz_frac", ctypes.c_double)]


class DeviceLevelState:
    """Per-device buffers of the device bundle loop, reused across mining runs:
    the generator workspace, the control block (+ its pinned host mirror), the
    per-level F sizes (fsz[k] = |F_k| on the device) and the post-step's plan and
    count buffers (DlPostC; sized for one accumulator pass)."""

    def __init__(self, dev):
        self.dev = dev
        self.ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
        self.ctl = torch.zeros(DL_CTL, dtype=_I64, device=dev)
        self.ctl_h = torch.zeros(DL_CTL, dtype=_I64, pin_memory=True)
        self.fsz = torch.zeros(128, dtype=_I64, device=dev)
        self.desc = np.zeros((32, 8), dtype=np.int64)
        self.info = np.zeros(4, dtype=np.int64)
        self.post = DlPostC()
        self.post_bufs = None
        self.post_keep = ()
        self.rows_hint = 0          # rows (columns) the next bundle's count runs over (lane_deal)

    def grow(self, nbytes: int) -> None:
        self.ws = torch.empty(int(nbytes * 1.25) + (1 << 20), dtype=torch.uint8, device=self.dev)

    def post_buffers(self, F1: int, c_cap: int, rows_cap: int, gpre_n: int = 0):
        """Grow-only plan / count buffers of the post step: item_map [F1], piece
        records [c_cap], planner scratch for rows_cap parent rows, counts [c_cap],
        long-prefix slab rows [gpre_n]."""
        part_n = 8 * ((rows_cap + 255) // 256 + 2)
        b = self.post_bufs
        if (b is None or b["F1"] < F1 or b["c_cap"] < c_cap or b["part"].numel() < part_n
                or b["gpre"].numel() < gpre_n):
            F1, c_cap = max(F1, b["F1"] if b else 0), max(c_cap, b["c_cap"] if b else 0)
            part_n = max(part_n, b["part"].numel() if b else 0)
            gpre_n = max(gpre_n, b["gpre"].numel() if b else 1)
            b = self.post_bufs = dict(F1=F1, c_cap=c_cap,
                                      item_map=torch.empty(max(F1, 1), dtype=_I32, device=self.dev),
                                      rec=torch.empty(12 * c_cap + 12, dtype=_I32, device=self.dev),
                                      part=torch.empty(part_n, dtype=_I32, device=self.dev),
                                      out=torch.empty(c_cap, dtype=_I32, device=self.dev),
                                      gpre=torch.empty(max(gpre_n, 1), dtype=_I32, device=self.dev))
        return b


_DL_STATE: dict = {}


def device_level_state(dev) -> DeviceLevelState:
    st = _DL_STATE.get(dev)
    if st is None:
        st = _DL_STATE[dev] = DeviceLevelState(dev)
    return st


def dl_lds_budget(F1: int) -> int:
    """LDS bytes left to slab + accumulators in k_count_slab_rec (the rank map's copy
    subtracted, as plan.cpp slab_width does)."""
    return TUNING.slab_lds_bytes - _slab_map_lds(F1)


# TUNING.dl_acc16: window-by-window device levels count into two u16 counters per
# accumulator word when the rows have unit weights: twice the candidates per pass, half
# the passes.  One-pass bundles keep u32 accumulators: with u16 ones the larger capacity
# made the generator pick 16-word slabs for level 3 alone and cut the later bundles
# differently, T10I4D100M 43.2 vs 42.3 ms (docs/PERF_HISTORY.md; that arm was removed)


def dl_slab_width(n_used: int, C: int, lds: int, accb: int = 4, cap_max: bool = False) -> tuple[int, int]:
    """plan.cpp slab_width: (SW, accumulator capacity) for n_used items and C candidates
    (accb: LDS bytes per accumulator).  cap_max (TUNING.slab_cap_max, gen.hip
    d_slab_cap): the first width whose capacity holds all C candidates."""
    for sw in (16, 32, 8, 4):
        cap = int((lds - n_used * (sw + 2) * 8) // accb)
        if cap_max:
            if cap >= C and (sw != 4 or cap >= 1024):
                return sw, cap
        elif cap >= min(C, 8192) or (sw == 4 and cap >= 1024):
            return sw, cap
    return 0, 0


def dl_bundle_gen(S: DeviceLevelState, P0: int, n_src: int | None, n_const: int, n_bound: int, m0: int, F1: int,
                  c_bound: int, lds: int, growth: float, max_levels: int, stream: int, post: bool = False,
                  accb: float = 4.0) -> np.ndarray:
    """Candidates of a device bundle: level 0 from F_{k-1} rows P0 and the speculative
    levels 1 .. max_levels-1 (accepted on the device), all queued before ONE
    synchronisation (accb: LDS bytes per slab accumulator, 2 = packed u16 counters).  Returns the control block (host int64 [DL_CTL]); S.desc[:L]
    describes the accepted levels (L = ctl[1])."""
    lib = _native.hip()
    info = np.zeros(2, dtype=np.int64)
    lib.fa_hip_set_cap_max(int(TUNING.slab_cap_max))
    for _ in range(6):
        S.desc[:] = 0
        rc = lib.fa_hip_dl_level0(P0, n_src, n_const, n_bound, m0, F1, _p(S.ws), S.ws.numel(), _p(S.ctl),
                                  _p(S.ctl_h), c_bound, float(lds), float(accb), S.info.ctypes.data,
                                  int(max_levels <= 1), stream)
        if rc == 5:
            S.grow(int(S.info[0]))
            continue
        _native.check(rc, "fa_hip_dl_level0")
        S.desc[0, :5] = [P0, S.info[1], S.info[2], S.info[3], m0]
        if max_levels <= 1:
            c = S.ctl_h.numpy()
            S.desc[0, 5:8] = [c[8], c[40], 0]
            return c.copy()
        S.post.done = 0
        lane_deal(lib, S.rows_hint)    # (the post step's plan)
        rc = lib.fa_hip_dl_more(F1, _p(S.ws), S.ws.numel(), int(S.info[0]), _p(S.ctl), _p(S.ctl_h), float(growth),
                                int(max_levels), float(lds), float(accb), int(c_bound), S.desc.ctypes.data,
                                info.ctypes.data,
                                stream, ctypes.addressof(S.post) if post else None)
        if rc == 5:
            S.grow(int(info[0]))
            continue
        _native.check(rc, "fa_hip_dl_more")
        return S.ctl_h.numpy().copy()
    raise RuntimeError("device bundle generation: workspace sizing did not converge")


def set_piece_part(part: int, nparts: int) -> None:
    """The share of the piece records the slab counts launched from now on count
    (count.hip fa_hip_set_piece_part: 64-piece chunks part, part + nparts, ...); (0, 1): all."""
    _native.check(_native.hip().fa_hip_set_piece_part(int(part), int(nparts)), "fa_hip_set_piece_part")


def lane_deal(lib, rows: int) -> None:
    """Bank-aware lane deal of the next device plans (levels.hip k_dl_lane_assign) for a
    count over this many rows: on from TUNING.lane_deal_min_rows (its fixed cost is
    repaid by the slabs it speeds up)."""
    lib.fa_hip_set_lane_deal(int(0 <= TUNING.lane_deal_min_rows <= rows))


def dl_plan(S: DeviceLevelState, L: int, F1: int, n_used: int, C: int, lds: int, dev, accb: float = 4.0) -> dict:
    """Device piece plan of a bundle's C candidates (levels.hip fa_hip_dl_plan), queued
    on the stream right after the generator's synchronisation: it depends on the
    candidates only, not on the row layout, so the host's trimming decision runs
    while it executes.  Returns the plan for dl_count."""
    st = torch.cuda.current_stream(dev).cuda_stream
    sw, cap = dl_slab_width(n_used, C, lds, accb, TUNING.slab_cap_max)
    if sw == 0 or C > cap:
        raise RuntimeError(f"device bundle of {C} candidates over {n_used} items does not fit one pass")
    item_map = torch.empty(max(F1, 1), dtype=_I32, device=dev)
    rec = torch.empty(12 * C + 12, dtype=_I32, device=dev)
    R = int(S.desc[:L, 5].sum())                     # parent rows of the bundle
    part = torch.empty(8 * max(1, (R + 255) // 256), dtype=_I32, device=dev)
    lib = _native.hip()
    gn = int(lib.fa_hip_dl_gpre_need(S.desc.ctypes.data, L))
    gpre = torch.empty(max(gn, 1), dtype=_I32, device=dev)
    lane_deal(lib, S.rows_hint)
    _native.check(lib.fa_hip_dl_plan(S.desc.ctypes.data, L, _p(S.ctl), F1, _p(item_map), _p(rec), C,
                                     _p(part), part.numel(), _p(gpre), gpre.numel(), sw, st), "fa_hip_dl_plan")
    out = torch.zeros(C, dtype=_I32, device=dev)
    return dict(sw=sw, cap=cap, item_map=item_map, rec=rec, out=out, n_used=n_used, C=C, gpre=gpre, accb=accb)


def dl_count_multipass(S: DeviceLevelState, F1: int, n_used: int, C: int, lds: int, roff, ranks, src, ncols: int,
                       wword, bm, bm_rows, sup_frac: float, dev, bmap=None, window_rows=None) -> torch.Tensor | None:
    """Counts of a device bundle's single level whose C candidates exceed one
    accumulator pass: per window of candidates, a device plan of that window
    (levels.hip fa_hip_dl_plan_window[_bits]) and a slab count from the used items'
    bitmap (bm [n_used or more][Wp]; bm_rows: slab row -> bitmap row, device int32, or
    None when bitmap row u is slab row u).  sup_frac: minimum support / rows
    (count_level's dense test).  Returns int32 [C] (not reduced across ranks), or None
    when no slab width fits the used items.

    TUNING.mp_window_items: every window's slab holds only the items ITS candidates
    use (bmap: device rank -> bitmap row, None = rank-indexed bitmap), and windows grow
    chunk by chunk (dl_window_plan) while their candidates fit what those rows leave
    of the LDS: deep T40I10 levels use 2-3x fewer items per window than per level, so
    every pass copies fewer slab rows and fewer passes are needed.

    window_rows (optional, with per-window items): (used_w, candidates), used_w the
    sorted ranks of a window's items -> None, or (ncols_w, bm_w): the bitmap of exactly those items over the rows
    that hold >= k of them (FastApriori._window_rows: a row with fewer holds none of the
    window's k-candidates), counted instead of the level's bitmap."""
    acc16 = TUNING.dl_acc16 and wword is None
    accb = 2 if acc16 else 4
    sw, cap = dl_slab_width(n_used, min(C, 8192), lds, accb)
    if sw == 0:
        return None
    st = _stream(ranks)
    lib = _native.hip()
    wins = None
    if TUNING.mp_window_items:
        wins = dl_window_plan(S, F1, C, lds, accb, st, dev)
    if not wins:
        cap = min(cap, C)
        cap = -(-C // -(-C // cap))                      # equal windows
        wins = [(w0, min(C, w0 + cap), sw, None) for w0 in range(0, C, cap)]
    cap = max(w1 - w0 for w0, w1, _, _ in wins)
    item_map = torch.empty(max(F1, 1), dtype=_I32, device=dev)
    rec = torch.empty(12 * cap + 12, dtype=_I32, device=dev)
    R = int(S.desc[0, 5])
    part = torch.empty(8 * max(1, (R + 255) // 256) + 16, dtype=_I32, device=dev)
    gn = int(lib.fa_hip_dl_gpre_need(S.desc.ctypes.data, 1))
    gpre = torch.empty(max(gn, 1), dtype=_I32, device=dev)
    out = torch.zeros(C, dtype=_I32, device=dev)
    npass, used_sum, rows_sum, trimmed = 0, 0, 0, 0
    lane_deal(lib, ncols)
    for w0, w1, wsw, bits in wins:
        nu, rows_w, bits_p, bm_w, ncols_w = n_used, bm_rows, None, bm, ncols
        if bits is not None:
            used_w = np.flatnonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[:F1])
            nu = int(used_w.size)
            bits_t = torch.from_numpy(bits.view(np.int64).copy()).to(dev, non_blocking=False)
            bits_p = bits_t
            got = window_rows(used_w, w1 - w0) if window_rows is not None else None
            if got is not None:
                # the window's own rows: its items' bitmap, bitmap row u = slab row u
                ncols_w, bm_w = got
                rows_w = None
                trimmed += 1
            else:
                used_t = torch.from_numpy(used_w.astype(np.int64)).to(dev)
                rows_w = (bmap[used_t] if bmap is not None else used_t).to(_I32).contiguous()
        if ncols_w == 0:
            continue                                     # no row holds k of the window's items
        W = (ncols_w + 63) // 64
        dense = wword is None and TUNING.dense_min_rows > 0 and sup_frac * wsw * 64 >= TUNING.dense_min_rows
        nslabs = (W + wsw - 1) // wsw
        _native.check(lib.fa_hip_dl_plan_window_bits(S.desc.ctypes.data, 1, _p(S.ctl), F1, _p(bits_p), _p(item_map),
                                                     _p(rec), cap, _p(part), part.numel(), _p(gpre), gpre.numel(),
                                                     w0, w1, wsw, st), "fa_hip_dl_plan_window_bits")
        nacc = (w1 - w0 + 1) // 2 if acc16 else w1 - w0
        lds_k = nu * (wsw + 2) * 8 + ((nacc + 3) & ~3) * 4
        n_wg = int(max(1, min(nslabs, 256 * min(max(1, TUNING.slab_lds_bytes // lds_k), 2))))
        _hip_call("fa_hip_count_slab_rec_cls", _p(roff), _p(ranks), _p(src), ncols_w, _p(item_map), F1, nu,
                  _p(gpre), _p(rec), 0, w1 - w0, _p(wword), out.data_ptr() + 4 * w0, wsw, n_wg, _p(bm_w),
                  bitmap_ld(bm_w), st, _p(rows_w), _p(S.ctl) + 8 * 221, (2 if dense else 0) | (4 if acc16 else 0))
        npass += 1
        used_sum += nu
        rows_sum += ncols_w
    LAST_LEVEL_PLAN.clear()
    LAST_LEVEL_PLAN.update(kernel="slab_dev_multi", rows=int(roff.numel() - 1), used=n_used, sw=sw, cap=cap,
                           passes=npass, pieces=-1, slab_reads=0, m=int(S.desc[0, 4]), C=C,
                           window_used_avg=round(used_sum / max(npass, 1), 1),
                           window_rows_avg=round(rows_sum / max(npass, 1)), windows_trimmed=trimmed)
    return out


WINDOW_SAMPLE = 16   # window_bitmap: the share of the words (1 / this) that decides max_keep
WINDOW_MAX_ITEMS = 2047   # count.hip k_win_alive: bit-sliced counts of up to 11 planes


def window_bitmap(bm: torch.Tensor, rows_w: torch.Tensor, W: int, k: int, max_keep: int | None = None,
                  blocked: bool = True):
    """The bitmap of a window's items over only the rows holding >= k of them, from the
    level's bitmap (count.hip k_win_alive / k_win_compact; FastApriori._window_rows).
    bm: the level's bitmap (row-major or 8-word blocked), rows_w: device int32 [n] its
    rows of the window's items (sorted by rank), W: its valid words.  Returns (K rows,
    bitmap of the window's items over them, row u = item u: the 8-word blocked layout
    [Wp' / 8, n, 8] (blocked; what slab_copy_bm streams best: a row-major one measured
    slower at T40I10D100M's levels 3-8) or row-major [n, Wp']), (0, None) when no row qualifies,
    or None when more than max_keep rows do -- judged on the first 1/WINDOW_SAMPLE of the
    words, then on all of them (a host synchronisation each)."""
    n = int(rows_w.numel())
    dev = bm.device
    st = _stream(bm)
    ld = bitmap_ld(bm)
    alive = torch.empty(max(W, 1), dtype=_I64, device=dev)
    cnt = torch.empty(max(W, 1), dtype=_I32, device=dev)
    if max_keep is not None and W >= 64 * WINDOW_SAMPLE:
        # the first 1/WINDOW_SAMPLE of the words first (rows are in no particular order):
        # a window that would keep too many rows costs that much of a pass, not a pass
        ws = W // WINDOW_SAMPLE
        _hip_call("fa_hip_win_alive", _p(bm), ld, _p(rows_w), n, ws, int(k), _p(alive), _p(cnt), st)
        if int(cnt[:ws].sum().item()) * (W / ws) > max_keep:
            return None
    _hip_call("fa_hip_win_alive", _p(bm), ld, _p(rows_w), n, W, int(k), _p(alive), _p(cnt), st)
    off = torch.zeros(W + 1, dtype=_I64, device=dev)
    torch.cumsum(cnt[:W], 0, out=off[1:])
    K = int(off[W].item())
    if max_keep is not None and K > max_keep:
        return None
    if K == 0:
        return 0, None
    wp = -(-((K + 63) // 64) // 64) * 64
    if blocked:
        out = torch.zeros((wp // 8, n, 8), dtype=_I64, device=dev)
        ldo = -out.stride(0)
    else:
        out = torch.zeros((n, wp), dtype=_I64, device=dev)
        ldo = out.stride(0)
    _hip_call("fa_hip_win_compact", _p(bm), ld, _p(rows_w), n, W, _p(alive), _p(off), _p(out), ldo, st)
    return K, out


def dl_window_plan(S: DeviceLevelState, F1: int, C: int, lds: int, accb: int, st: int, dev,
                   chunk: int = 1024) -> list | None:
    """Windows of a multi-pass level's C candidates (device bundle level 0) sized by their
    own used items: the used-item bitset of every chunk of candidates
    (levels.hip fa_hip_dl_chunk_bits, one small readback), then, greedily, the longest run
    of chunks whose item union leaves accumulators for all of its candidates at the
    widest slab holding min(candidates, 8192) (dl_slab_width).  Returns [(w0, w1, sw,
    uint64 bitset [nwd])], or None when F1 is too wide for the bitsets."""
    nwd = (F1 + 63) // 64
    if nwd > 512 or C < 1:
        return None
    nch = -(-C // chunk)
    bits_d = torch.empty(nch * nwd, dtype=_I64, device=dev)
    _native.check(_native.hip().fa_hip_dl_chunk_bits(S.desc.ctypes.data, F1, chunk, _p(bits_d), st),
                  "fa_hip_dl_chunk_bits")
    bits = bits_d.cpu().numpy().view(np.uint64).reshape(nch, nwd)
    pop8 = np.array([bin(i).count("1") for i in range(256)], dtype=np.int64)
    wins = []
    j = 0
    while j < nch:
        acc = np.zeros(nwd, dtype=np.uint64)
        k, best = j, None
        while k < nch:
            a2 = acc | bits[k]
            n = int(pop8[a2.view(np.uint8)].sum())
            cand = min((k + 1) * chunk, C) - j * chunk
            sw, cap = dl_slab_width(n, min(cand, 8192), lds, accb)
            if sw == 0 or cap < cand:
                break
            acc, best = a2, sw
            k += 1
        if best is None:
            return None                              # one chunk does not fit: the level-wide windows
        wins.append((j * chunk, min(k * chunk, C), best, acc))
        j = k
    return wins


def dl_plan_from_post(S: DeviceLevelState, n_used: int) -> dict:
    """The plan the post step queued (S.post.done >= 1), in dl_plan's form."""
    P, b = S.post, S.post_bufs
    C = int(P.C)
    out = b["out"][:C]
    return dict(sw=int(P.sw), cap=int(P.cap), item_map=b["item_map"], rec=b["rec"], out=out, n_used=n_used, C=C,
                gpre=b["gpre"], accb=float(P.accb))


def dl_count(S: DeviceLevelState, plan: dict, roff, ranks, src, ncols: int, F1: int, wword) -> torch.Tensor:
    """Slab count of a planned bundle (dl_plan) over the current rows -> int32 [C] on
    the device, bundle order (not yet reduced across ranks)."""
    st = _stream(ranks)
    sw, cap, n_used, C = plan["sw"], plan["cap"], plan["n_used"], plan["C"]
    item_map, rec, out = plan["item_map"], plan["rec"], plan["out"]
    W = (ncols + 63) // 64
    nslabs = (W + sw - 1) // sw
    acc16 = plan.get("accb", 4.0) == 2.0 and wword is None
    nacc = (C + 1) // 2 if acc16 else C
    lds_k = n_used * (sw + 2) * 8 + ((nacc + 3) & ~3) * 4 + _slab_map_lds(F1)
    n_wg = int(max(1, min(nslabs, 256 * min(max(1, TUNING.slab_lds_bytes // lds_k), 2))))
    _hip_call("fa_hip_count_slab_rec_cls", _p(roff), _p(ranks), _p(src), ncols, _p(item_map), F1, n_used,
              _p(plan.get("gpre")), _p(rec), 0, C, _p(wword), _p(out), sw, n_wg, None, 0, st, None,
              _p(S.ctl) + 8 * 221, 4 if acc16 else 0)
    LAST_LEVEL_PLAN.clear()
    LAST_LEVEL_PLAN.update(kernel="slab_dev", rows=int(roff.numel() - 1), used=n_used, sw=sw, cap=cap, passes=1,
                           pieces=-1, slab_reads=0, m=-1, C=C)
    # (item_map and rec may be freed now: the caching allocator hands their blocks only
    # to work queued later on this stream)
    return out


def dl_threshold(S: DeviceLevelState, L: int, counts: torch.Tensor, mc: int, k0: int):
    """Keep counts >= mc per level of a device bundle.  Returns (rows int32 arena,
    cnt int32 arena, rows_off int64 [L], cnt_off int64 [L]); |F_{k0+l}| lands in
    S.fsz[k0 + l] on the device."""
    dev = counts.device
    C = S.desc[:L, 6]
    w = S.desc[:L, 4] + 1
    rows_off = np.zeros(L, dtype=np.int64)
    cnt_off = np.zeros(L, dtype=np.int64)
    if L > 1:
        rows_off[1:] = np.cumsum(C * w)[:-1]
        cnt_off[1:] = np.cumsum(C)[:-1]
    rows = torch.empty(max(int((C * w).sum()), 1), dtype=_I32, device=dev)
    # the kept counts + the multi-workgroup threshold's block counts (levels.hip) in one allocation
    nblk = int(((C + 1023) // 1024).sum())
    cnt = torch.empty(max(int(C.sum()), 1) + nblk, dtype=_I32, device=dev)
    scratch = cnt[cnt.numel() - nblk:]
    _native.check(_native.hip().fa_hip_dl_threshold(S.desc.ctypes.data, L, _p(counts), int(mc), _p(rows),
                                                    rows_off.ctypes.data, _p(cnt), cnt_off.ctypes.data,
                                                    _p(S.fsz) + 8 * k0, _p(scratch), nblk, _stream(counts)),
                  "fa_hip_dl_threshold")
    cnt = cnt[:cnt.numel() - nblk]
    return rows, cnt, rows_off, cnt_off
