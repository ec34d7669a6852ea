"""Input shards and output files (reference formats).

Reading (Utils.scala:19-27): each rank parses the lines that start inside its
byte range [size*r/W, size*(r+1)/W) of the file with the native mmap parser.
Writing (Utils.scala:29-49): rank 0 writes Spark-style output directories with
a single ``part-00000`` plus an empty ``_SUCCESS`` marker.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from ..models.data import MiningResult, TransactionShard, Vocabulary
from ..ops import _native
from ..tuning import TUNING
from .env import num_threads


def _pinned(n: int, dtype, pin: bool) -> torch.Tensor:
    n = max(n, 1)
    if pin:
        try:
            return torch.empty(n, dtype=dtype, pin_memory=True)
        except RuntimeError:
            pass
    return torch.empty(n, dtype=dtype)


def txndb_to_shard(h, device: torch.device, line_base: int = 0) -> TransactionShard:
    """Export a native TxnDB handle into torch tensors (frees the handle)."""
    lib = _native.host()
    info = np.zeros(6, dtype=np.int64)
    lib.fa_txndb_info(h, info.ctypes.data)
    n, nnz, nx, numeric, vocab, dbytes = (int(v) for v in info)
    pin = device.type == "cuda"
    off = _pinned(n + 1, torch.int64, pin)
    items = _pinned(nnz, torch.int32, pin)
    extras = np.zeros(max(nx, 1), dtype=np.int32)
    lib.fa_txndb_export(h, off.data_ptr(), items.data_ptr(), extras.ctypes.data, num_threads())
    buf = soff = hashes = None
    if not numeric:
        # the dictionary stays a byte blob + offsets (Vocabulary.decode on demand)
        buf = np.zeros(max(dbytes, 1), dtype=np.uint8)
        soff = np.zeros(vocab + 1, dtype=np.int64)
        hashes = np.zeros(max(vocab, 1), dtype=np.uint64)
        lib.fa_txndb_export_dict(h, buf.ctypes.data, soff.ctypes.data, hashes.ctypes.data, num_threads())
        hashes = hashes[:vocab]
    lib.fa_txndb_free(h)
    off = off[: n + 1]
    if n == 0:
        off.zero_()
    items = items[:nnz]
    shard = TransactionShard(off.to(device, non_blocking=True), items.to(device, non_blocking=True),
                             extras[:nx], Vocabulary(bool(numeric), vocab, None, hashes, buf, soff), line_base)
    return shard


def parse_file(path: str, byte_begin: int = 0, byte_end: int = -1, mode: int = 0,
               device: torch.device | str = "cpu", line_base: int = 0) -> TransactionShard:
    err = C.c_int(0)
    h = _native.host().fa_parse_file(path.encode(), byte_begin, byte_end, mode, num_threads(), C.byref(err))
    if not h:
        if err.value == 7:
            raise RuntimeError(f"{path}: two distinct tokens share a 64-bit hash (dictionary mode)")
        raise FileNotFoundError(f"cannot read {path} (error {err.value})")
    return txndb_to_shard(h, torch.device(device), line_base)


# ---------------------------------------------------------------------------
# Device parser path: the shard's bytes go to HBM (pread by host threads into a
# ring of pinned slots, overlapped with the H2D copies) and are tokenised by
# csrc/hip/parse.hip.  Numeric vocabularies only; anything else returns None and
# the caller uses the host parser.
# (TUNING.gpu_parse / gpu_parse_dict switch it off.)
_RING_SLOT = 32 << 20
# pinned slots in flight (TUNING.ring_slots; one reader thread each, up to the host
# thread count): one thread's pread out of the page cache runs at ~4-6 GB/s, so 8
# readers held the 3.9 GB T10I4D100M file at ~35 GB/s, below the ~57 GB/s of the H2D copies
_ring: list = []


def ring_slots() -> int:
    """Pinned ring slots in use (allocated on first use, grown when the knob grows)."""
    ns = max(1, int(TUNING.ring_slots))
    if len(_ring) < ns:
        _ring.extend(torch.empty(_RING_SLOT, dtype=torch.uint8, pin_memory=True) for _ in range(ns - len(_ring)))
    return ns


def _next_line_start(fd: int, size: int, pos: int) -> int:
    """First line start >= pos (parse.cpp next_line_start): the byte after the first
    terminator at or after pos - 1 ('\r\n' counts as one)."""
    if pos <= 0:
        return 0
    i = pos - 1
    while i < size:
        blk = os.pread(fd, 1 << 16, i)
        if not blk:
            break
        for k, c in enumerate(blk):
            if c == 10:
                return i + k + 1
            if c == 13:
                if i + k + 1 < size and os.pread(fd, 1, i + k + 1) == b"\n":
                    return i + k + 2
                return i + k + 1
        i += len(blk)
    return size


_copy_streams: dict = {}


def _file_to_device(fd: int, first: int, n: int, dev, parse: bool = False, last_is_term: bool = True):
    r"""Bytes [first, first + n) of the file -> uint8 device tensor padded with zeros
    to a multiple of 64 plus 64.  Host threads pread _RING_SLOT chunks into a ring
    of pinned slots; each lands in HBM by an asynchronous copy on a copy stream.

    parse=True also parses while the bytes stream in (csrc/hip/parse.hip tile
    parser, ops.primitives.TileParse): every chunk's reader thread counts its '\n'
    bytes and finds the last one (fa_chunk_scan), and as soon as a chunk's copy
    lands, the lines it completes -- from the previous region's end to just past its
    last '\n' -- are parsed on the compute stream (it waits for that copy only)
    while the next chunks are still being read and copied.  The partial last line
    carries into the next region.  From the first chunk holding a '\r' on (lone
    '\r' ends lines too), the rest is one final region parsed after the last copy.
    Returns the buffer, and with parse=True the parser's result
    (TileParse.finish) as a second value."""
    from concurrent.futures import ThreadPoolExecutor

    out = torch.empty((n + 63) // 64 * 64 + 64, dtype=torch.uint8, device=dev)
    out[n:].zero_()
    tp = None
    if parse:
        from ..ops import primitives as prim
        tp = prim.TileParse(out, n, dev, scratch_bytes=min(n, 2 * _RING_SLOT))
    if n == 0:
        return (out, tp.finish()) if parse else out
    NS = ring_slots()
    cs = _copy_streams.get(dev)
    if cs is None:
        cs = _copy_streams[dev] = torch.cuda.Stream(dev)
    compute = torch.cuda.current_stream(dev)
    cs.wait_stream(compute)             # the buffer's allocation and zero fill come first
    nch = (n + _RING_SLOT - 1) // _RING_SLOT
    events: list = [None] * NS
    lib = _native.host()

    def read_chunk(c: int):
        ev = events[c % NS]
        if ev is not None:
            ev.synchronize()          # the slot's previous H2D copy has finished
        off = c * _RING_SLOT
        m = min(_RING_SLOT, n - off)
        slot = _ring[c % NS]
        mv = memoryview(slot.numpy())
        got = 0
        while got < m:
            r = os.preadv(fd, [mv[got:m]], first + off + got)
            if r <= 0:
                raise OSError(f"short read at {first + off + got}")
            got += r
        if not parse:
            return None
        info = np.zeros(3, dtype=np.int64)
        lib.fa_chunk_scan(slot.data_ptr(), m, info.ctypes.data)
        return info

    streaming = parse and TUNING.stream_parse
    rend = 0                            # parsed up to here (a line start)
    with ThreadPoolExecutor(min(num_threads(), NS)) as ex:
        fut = {c: ex.submit(read_chunk, c) for c in range(min(NS, nch))}
        for c in range(nch):
            info = fut.pop(c).result()
            s, off = c % NS, c * _RING_SLOT
            m = min(_RING_SLOT, n - off)
            with torch.cuda.stream(cs):
                out[off:off + m].copy_(_ring[s][:m], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(cs)
            events[s] = ev
            if c + NS < nch:
                fut[c + NS] = ex.submit(read_chunk, c + NS)
            if streaming and c + 1 < nch:
                if info[2]:
                    streaming = False   # a '\r': the rest is the final region
                elif info[1] >= 0:
                    compute.wait_event(ev)
                    end = off + int(info[1]) + 1
                    tp.region(rend, end, int(info[0]), tail=False)
                    rend = end
    compute.wait_event(events[(nch - 1) % NS])
    if not parse:
        return out
    tp.region(rend, n, None, tail=not last_is_term)
    return out, tp.finish()


def parse_file_device(path: str, byte_begin: int, byte_end: int, device, line_base: int = 0,
                      force_dict: bool = False):
    """Lines starting in [byte_begin, byte_end) parsed on the GPU, or None (a CPU device,
    or a dictionary table overflow).  Numeric tokens take the numeric id space; any
    other token the device dictionary path (hash-table ids, strings read back from the
    file only for the ids decoded later)."""
    from ..ops import primitives as prim

    device = torch.device(device)
    if device.type != "cuda":
        return None
    fd = os.open(path, os.O_RDONLY)
    try:
        size = os.fstat(fd).st_size
        b = max(0, min(byte_begin, size))
        e = size if byte_end < 0 else max(b, min(byte_end, size))
        first = _next_line_start(fd, size, b)
        last = _next_line_start(fd, size, e) if e < size else size
        last = max(last, first)
        n = last - first
        last_is_term = n == 0 or os.pread(fd, 1, last - 1) in (b"\n", b"\r")
        if force_dict:
            buf, got = _file_to_device(fd, first, n, device), None
        else:
            buf, got = _file_to_device(fd, first, n, device, parse=True, last_is_term=last_is_term)
            if isinstance(got, int):
                # more repeated ids than the streamed parse's repeat buffer: again, with room
                got = prim.parse_numeric_device(buf, n, last_is_term)
    finally:
        os.close(fd)
    if got is not None:
        del buf
        off, items, extras, vocab, hist = got
        return TransactionShard(off, items, extras.cpu().numpy(), Vocabulary(True, vocab), line_base, hist)
    got = prim.parse_dict_device(buf, n, last_is_term) if TUNING.gpu_parse_dict else None
    del buf
    if got is None:
        return None
    off, items, extras, hashes, pos, lens = got
    voc = Vocabulary(False, int(hashes.size), hashes=hashes, file_src=(path, first, pos, lens))
    return TransactionShard(off, items, extras.cpu().numpy(), voc, line_base)


def parse_bytes(data: bytes, mode: int = 0, device="cpu") -> TransactionShard:
    h = _native.host().fa_parse_buffer(data, len(data), mode, num_threads())
    if not h:
        raise RuntimeError("two distinct tokens share a 64-bit hash (dictionary mode)")
    return txndb_to_shard(h, torch.device(device))


def read_shard(path: str, comm, device: torch.device | str | None = None) -> TransactionShard:
    """This rank's shard of ``path``; all ranks agree on numeric vs dict ids."""
    device = torch.device(device or comm.device)
    size = _native.host().fa_file_size(path.encode())
    if size < 0:
        raise FileNotFoundError(path)
    b = size * comm.rank // comm.world_size
    e = size * (comm.rank + 1) // comm.world_size
    shard = parse_file_device(path, b, e, device) if (TUNING.gpu_parse and device.type == "cuda") else None
    if shard is None:
        # host parser, straight into pinned buffers when the shard goes to a GPU
        shard = parse_file(path, b, e, 0, device)
    need_dict = comm.allreduce_int(0 if shard.vocab.numeric else 1, "max")
    if need_dict and shard.vocab.numeric:
        # another rank saw non-numeric tokens: every rank takes dictionary ids
        shard = (parse_file_device(path, b, e, device, force_dict=True)
                 if (TUNING.gpu_parse and TUNING.gpu_parse_dict and device.type == "cuda") else None) or parse_file(path, b, e, 1,
                                                                                                  device)
    counts = comm.all_gather_int(shard.n_lines)
    shard.line_base = int(sum(counts[: comm.rank]))
    return shard.to(device)


def generate_shard(n_txn: int, comm, device=None, avg_len: float = 10.0, avg_pat: float = 4.0,
                   n_patterns: int = 2000, n_items: int = 1000, seed: int = 1, users: bool = False
                   ) -> TransactionShard:
    """This rank's slice of a synthetic Quest database (see csrc/host/quest.cpp)."""
    device = torch.device(device or comm.device)
    b = n_txn * comm.rank // comm.world_size
    e = n_txn * (comm.rank + 1) // comm.world_size
    h = _native.host().fa_quest_generate(b, e, avg_len, avg_pat, n_patterns, n_items, seed,
                                         1 if users else 0, num_threads())
    return txndb_to_shard(h, device, b)


def generate_zipf_shard(n_txn: int, comm, device=None, mean_len: float = 177.0, sigma: float = 0.5,
                        n_items: int = 5_267_656, s: float = 1.05, q: float = 50.0, n_topics: int = 2000,
                        seed: int = 1) -> TransactionShard:
    """This rank's slice of a wide-vocabulary (webdocs-like) synthetic database
    (Zipf-Mandelbrot background words + topic cores, see csrc/host/quest.cpp)."""
    device = torch.device(device or comm.device)
    b = n_txn * comm.rank // comm.world_size
    e = n_txn * (comm.rank + 1) // comm.world_size
    h = _native.host().fa_zipf_generate(b, e, mean_len, sigma, n_items, s, q, n_topics, seed, num_threads())
    return txndb_to_shard(h, device, b)


def write_zipf_file(path: str, n_txn: int, mean_len: float = 177.0, sigma: float = 0.5, n_items: int = 5_267_656,
                    s: float = 1.05, q: float = 50.0, n_topics: int = 2000, seed: int = 1,
                    string_tokens: bool = False) -> None:
    """Wide-vocabulary documents (generate_zipf_shard's model) as a text file; with
    ``string_tokens`` every word is a letter string ("w" + base-26), so the file
    takes the dictionary path of the parser and the miner."""
    rc = _native.host().fa_zipf_write(path.encode(), n_txn, mean_len, sigma, n_items, s, q, n_topics, seed,
                                      1 if string_tokens else 0, num_threads())
    if rc:
        raise OSError(f"failed to write {path}")


def write_quest_file(path: str, n_txn: int, avg_len=10.0, avg_pat=4.0, n_patterns=2000, n_items=1000,
                     seed=1, users=False) -> None:
    rc = _native.host().fa_quest_write(path.encode(), n_txn, avg_len, avg_pat, n_patterns, n_items, seed,
                                       1 if users else 0, num_threads())
    if rc:
        raise OSError(f"failed to write {path}")


# ---------------------------------------------------------------------------
# Writers
# ---------------------------------------------------------------------------
class OutputExistsError(FileExistsError):
    pass


def _prepare_dir(path: str, overwrite: bool) -> None:
    if os.path.exists(path):
        if not overwrite:
            # Spark's saveAsTextFile refuses an existing output directory.
            raise OutputExistsError(f"Output directory {path} already exists")
        for f in os.listdir(path):
            os.remove(os.path.join(path, f))
    else:
        os.makedirs(path, exist_ok=True)


def _tokens_blob(items: list[str]):
    enc = [t.encode("utf-8") for t in items]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        off[1:] = np.cumsum([len(e) for e in enc])
    blob = b"".join(enc) or b"\0"
    return blob, off


def write_freq_itemsets(result: MiningResult, out_dir: str, with_counts: bool = False,
                        overwrite: bool = False) -> str:
    """``<output>freqItemset/part-00000`` (or ``freqItems`` with counts, Utils.scala:61)."""
    _prepare_dir(out_dir, overwrite)
    blob, off = _tokens_blob(result.items)
    levels = [np.ascontiguousarray(l, dtype=np.int32) for l in result.levels]
    counts = [np.ascontiguousarray(c, dtype=np.int64) for c in result.counts]
    K = len(levels)
    rows_p = (C.c_void_p * max(K, 1))(*[l.ctypes.data for l in levels])
    cnt_p = (C.c_void_p * max(K, 1))(*[c.ctypes.data for c in counts])
    sizes = np.array([l.shape[0] for l in levels] or [0], dtype=np.int64)
    part = os.path.join(out_dir, "part-00000")
    rc = _native.host().fa_write_freq_itemsets(part.encode(), blob, off.ctypes.data, len(result.items),
                                               C.cast(rows_p, C.c_void_p), C.cast(cnt_p, C.c_void_p),
                                               sizes.ctypes.data, K, 1 if with_counts else 0, num_threads())
    if rc:
        raise OSError(f"failed to write {part}")
    open(os.path.join(out_dir, "_SUCCESS"), "wb").close()
    return part


def write_lines(lines: list[str], out_dir: str, overwrite: bool = False) -> str:
    """``<output>recommends/part-00000``: one token per U.dat line (Utils.scala:43-49)."""
    _prepare_dir(out_dir, overwrite)
    part = os.path.join(out_dir, "part-00000")
    with open(part, "wb") as f:
        if lines:
            f.write(("\n".join(lines) + "\n").encode("utf-8"))
    open(os.path.join(out_dir, "_SUCCESS"), "wb").close()
    return part


def write_items_to_rank(result: MiningResult, path: str) -> None:
    """``ItemsToRank`` ("item rank" lines) and ``FreqItems`` companions read by getAll (Utils.scala:65-81)."""
    with open(path, "w", encoding="utf-8") as f:
        for r, t in enumerate(result.items):
            f.write(f"{t} {r}\n")


def write_freq_items(result: MiningResult, path: str) -> None:
    with open(path, "w", encoding="utf-8") as f:
        for t in result.items:
            f.write(t + "\n")


def load_saved_results(freq_with_counts: str, items_to_rank: str, min_count: int = 0,
                       n_lines: int = 0) -> MiningResult:
    """Rebuild a MiningResult from saved files — the reference's ``Utils.getAll``
    (Utils.scala:65-81): "item rank" lines + "a b c[cnt]" itemset lines."""
    rank: dict[str, int] = {}
    with open(items_to_rank, encoding="utf-8") as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            tok, r = line.rsplit(" ", 1)
            rank[tok] = int(r)
    items = [None] * len(rank)
    for t, r in rank.items():
        items[r] = t
    by_k: dict[int, list[tuple[list[int], int]]] = {}
    part = freq_with_counts
    if os.path.isdir(part):
        part = os.path.join(part, "part-00000")
    with open(part, encoding="utf-8") as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            body, cnt = line[:-1].rsplit("[", 1)
            ranks = sorted(rank[t] for t in body.split(" "))
            by_k.setdefault(len(ranks), []).append((ranks, int(cnt)))
    K = max(by_k) if by_k else 0
    levels, counts = [], []
    for k in range(1, K + 1):
        rows = sorted(by_k.get(k, []))
        levels.append(np.array([r for r, _ in rows], dtype=np.int32).reshape(-1, k))
        counts.append(np.array([c for _, c in rows], dtype=np.int64))
    return MiningResult(items=items, levels=levels, counts=counts, min_count=min_count, n_lines=n_lines)
