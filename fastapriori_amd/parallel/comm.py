"""Collective communication for count distribution (one process per GPU).

Every rank owns a contiguous shard of the transactions; all ranks hold the
identical candidate lists and only count vectors move (SURVEY §2.4 plan):

  X3/X8   line / transaction totals          -> all_reduce(int64[1])
  X4      F1 token histogram                  -> all_reduce(int64[V])
  X12     pair supports                       -> reduce_scatter + local threshold + all_gather of the
                                                 survivors (big triangles), else all_reduce
  X15     level-k candidate supports          -> all_reduce(int64[C_k])
  X17     U.dat line offsets                  -> all_gather(int64[1])
  X24     recommendations                     -> gather to rank 0

On ROCm the ``nccl`` backend is RCCL, riding xGMI between the GPUs of a node;
``gloo`` serves CPU-only runs and tests.  What matters on xGMI is how many bytes
each collective moves, not how they are cut: a mining run issues six collectives
and the largest payload is the k = 2 triangle (T10I4D100M: 1.9 MB, one ring
all-reduce of ~22 us on one ~153 GB/s link).  Triangles from
``TUNING.pair_rs_min`` pairs on go as a reduce-scatter + local threshold +
all-gather of the survivors instead (``reduce_scatter_select``).  Vectors longer
than ``TUNING.bucket_mb`` (64 MiB: F1 past ~5800 items) are reduced in buckets of
that size, a multiple of world_size elements, so that no single call pins a huge
staging buffer; below it there is exactly one call per vector.
"""
from __future__ import annotations

import functools
import os
import pickle
import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist


def _timed(fn):
    """Host wall time spent inside the collectives (comm_ms; nested calls count once).
    RCCL collectives are asynchronous: this is the time the host is held, including
    the readbacks the small decision collectives need (bench.py per-rank record)."""
    @functools.wraps(fn)
    def wrap(self, *a, **kw):
        if self._depth:
            return fn(self, *a, **kw)
        self._depth += 1
        t0 = time.perf_counter()
        b0 = self.bytes_reduced + self.bytes_gathered
        try:
            return fn(self, *a, **kw)
        finally:
            self._depth -= 1
            dt = (time.perf_counter() - t0) * 1e3
            self.comm_ms += dt
            self.comm_calls += 1
            if self.trace is not None:
                # (collective, payload bytes it moved per rank, host ms)
                self.trace.append((fn.__name__, self.bytes_reduced + self.bytes_gathered - b0, round(dt, 3)))
    return wrap


@dataclass
class Comm:
    rank: int = 0
    world_size: int = 1
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    bytes_reduced: int = 0
    bytes_gathered: int = 0   # payload bytes received by the all-gathers (Comm.trace)
    force: bool = False     # run the collective code paths even at world size 1 (FA_FORCE_PG)
    comm_ms: float = 0.0    # host time inside collectives (see _timed)
    comm_calls: int = 0
    _depth: int = 0
    trace: list | None = None   # set to [] to record every top-level collective (_timed)

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 or self.force

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    # -- tensors ------------------------------------------------------------
    def _comm_device(self) -> torch.device:
        return self.device if self.backend == "nccl" else torch.device("cpu")

    @_timed
    def all_reduce_(self, t: torch.Tensor, op=None, bound: int | None = None) -> torch.Tensor:
        """In-place sum (or ``op``) across ranks; returns the tensor on its own device.

        ``bound``: an upper bound of every reduced value (support counts never exceed
        the global number of lines).  Below 2**31 an int64 vector travels as int32,
        halving the bytes on the xGMI links."""
        if not self.distributed:
            return t
        op = op or dist.ReduceOp.SUM
        dev = self._comm_device()
        if bound is not None and t.dtype == torch.int64 and 0 <= bound < (1 << 31):
            x = t.to(device=dev, dtype=torch.int32)
        else:
            x = t if t.device == dev else t.to(dev)
        flat = x.view(-1)
        nbytes = flat.numel() * flat.element_size()
        self.bytes_reduced += nbytes
        bucket = self.bucket_elems(flat.element_size())
        if flat.numel() <= bucket:
            dist.all_reduce(flat, op=op)
        else:
            for s in range(0, flat.numel(), bucket):
                dist.all_reduce(flat[s:s + bucket], op=op)
        if x is not t:
            t.copy_(x)
        return t

    @_timed
    def reduce_scatter_select(self, t: torch.Tensor, thr: int, bound: int | None = None):
        """Entries of the cross-rank sum of ``t`` that are >= ``thr``: (indices, values),
        identical on every rank and in index order.

        reduce-scatter (each rank receives the sum of its 1/world slice) + a local
        threshold + an all-gather of the survivors only.  An all-reduce moves
        2(W-1)/W of the vector per rank; this moves (W-1)/W plus the survivors, which
        for the k = 2 triangle are a few percent of it (the
        FastApriori.scala:236-238 collect of F_2 without shipping C_2)."""
        dev = self._comm_device()
        narrow = bound is not None and t.dtype == torch.int64 and 0 <= bound < (1 << 31)
        x = t.to(device=dev, dtype=torch.int32 if narrow else t.dtype).reshape(-1)
        n, W = x.numel(), self.world_size
        chunk = (n + W - 1) // W
        if chunk * W != n:
            x = torch.cat([x, torch.zeros(chunk * W - n, dtype=x.dtype, device=dev)])
        part = torch.empty(chunk, dtype=x.dtype, device=dev)
        dist.reduce_scatter_tensor(part, x)
        self.bytes_reduced += chunk * (W - 1) * x.element_size()
        loc = torch.nonzero(part >= thr).flatten()
        # the zero padding past n is never an entry (min_support 0 would select it)
        loc = loc[loc + self.rank * chunk < n]
        mine = torch.stack([loc + self.rank * chunk, part[loc].to(torch.int64)]) if loc.numel() else \
            torch.zeros((2, 0), dtype=torch.int64, device=dev)
        sizes = self.all_gather_ints([int(mine.shape[1])])[:, 0]
        mx = int(sizes.max())
        buf = torch.zeros((2, max(mx, 1)), dtype=torch.int64, device=dev)
        buf[:, :mine.shape[1]] = mine
        # flat buffers: gloo's all_gather_into_tensor takes only the concatenated form
        out = torch.empty(W * buf.numel(), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, buf.view(-1))
        out = out.view(W, 2, max(mx, 1))
        self.bytes_reduced += int(sizes.sum()) * 16
        got = torch.cat([out[r, :, :int(sizes[r])] for r in range(W)], dim=1)
        return got[0], got[1]

    def bucket_elems(self, elem_size: int) -> int:
        """Elements per all-reduce call: TUNING.bucket_mb MiB, rounded down to a multiple
        of world_size (every bucket splits evenly into RCCL's per-rank chunks)."""
        from ..tuning import TUNING
        n = int(float(TUNING.bucket_mb) * (1 << 20)) // elem_size
        q = max(1, self.world_size)
        return max(q, n // q * q)

    @_timed
    def allreduce_int(self, v: int, op: str = "sum") -> int:
        if not self.distributed:
            return int(v)
        t = torch.tensor([int(v)], dtype=torch.int64, device=self._comm_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return int(t.item())

    @_timed
    def allreduce_float_max(self, v: float) -> float:
        if not self.distributed:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self._comm_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    @_timed
    def all_gather_int(self, v: int) -> list[int]:
        if not self.distributed:
            return [int(v)]
        t = torch.tensor([int(v)], dtype=torch.int64, device=self._comm_device())
        out = [torch.zeros_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    @_timed
    def all_gather_ints(self, values) -> np.ndarray:
        """One collective for several small integers: int64 [world, len(values)]."""
        v = np.asarray(values, dtype=np.int64).reshape(1, -1)
        if not self.distributed:
            return v
        t = torch.from_numpy(v.ravel().copy()).to(self._comm_device())
        out = torch.empty(self.world_size * t.numel(), dtype=torch.int64, device=t.device)
        dist.all_gather_into_tensor(out, t)
        self.bytes_gathered += out.numel() * 8
        return out.cpu().numpy().reshape(self.world_size, -1)

    @_timed
    def all_gather_varlen_np(self, a: np.ndarray) -> list[np.ndarray]:
        """All-gather 1-D int64 arrays of different lengths (sizes, then one padded
        all_gather_into_tensor): rank order, on every rank."""
        a = np.ascontiguousarray(a, dtype=np.int64).ravel()
        if not self.distributed:
            return [a]
        sizes = self.all_gather_ints([a.size])[:, 0]
        mx = max(int(sizes.max()), 1)
        dev = self._comm_device()
        buf = torch.zeros(mx, dtype=torch.int64, device=dev)
        if a.size:
            buf[:a.size] = torch.from_numpy(a).to(dev)
        out = torch.empty(self.world_size * mx, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, buf)
        self.bytes_gathered += out.numel() * 8
        o = out.cpu().numpy().reshape(self.world_size, mx)
        return [o[r, :int(sizes[r])] for r in range(self.world_size)]

    @_timed
    def all_gather_object(self, obj) -> list:
        if not self.distributed:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    @_timed
    def broadcast_object(self, obj, src: int = 0):
        if not self.distributed:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src)
        return box[0]

    @_timed
    def gather_varlen(self, t: torch.Tensor) -> list[torch.Tensor] | None:
        """Gather 1-D tensors of different lengths to rank 0 (None elsewhere)."""
        if not self.distributed:
            return [t.cpu()]
        dev = self._comm_device()
        sizes = self.all_gather_int(t.numel())
        mx = max(sizes) if sizes else 0
        buf = torch.zeros(max(mx, 1), dtype=t.dtype, device=dev)
        buf[: t.numel()] = t.to(dev)
        outs = [torch.zeros_like(buf) for _ in range(self.world_size)]
        dist.all_gather(outs, buf)
        if not self.is_root:
            return None
        return [o[:s].cpu() for o, s in zip(outs, sizes)]

    @_timed
    def all_to_all_varlen(self, parts: list[np.ndarray], dtype=np.int64) -> list[np.ndarray]:
        """Exchange variable-length int arrays: parts[r] goes to rank r."""
        if not self.distributed:
            return [parts[0]]
        dev = self._comm_device()
        send_sizes = torch.tensor([p.size for p in parts], dtype=torch.int64, device=dev)
        recv_sizes = torch.empty_like(send_sizes)
        dist.all_to_all_single(recv_sizes, send_sizes)
        rs = recv_sizes.cpu().tolist()
        send = torch.from_numpy(np.concatenate(parts).astype(dtype)).to(dev) if sum(p.size for p in parts) \
            else torch.zeros(0, dtype=torch.int64, device=dev)
        recv = torch.empty(sum(rs), dtype=send.dtype, device=dev)
        dist.all_to_all_single(recv, send, output_split_sizes=rs,
                               input_split_sizes=[p.size for p in parts])
        out = recv.cpu().numpy()
        res, o = [], 0
        for s in rs:
            res.append(out[o:o + s])
            o += s
        return res

    @_timed
    def barrier(self) -> None:
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


def init_comm(device: str | None = None, backend: str | None = None, timeout_s: float = 1800) -> Comm:
    """Create the communicator from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).

    ``device``: "cuda", "cpu" or None (cuda when available).  The backend is
    RCCL ("nccl") for GPU runs, gloo for CPU runs.
    """
    from datetime import timedelta

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    if device == "cuda":
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            # NUMA-local CPUs of this rank's GPU, before anything pins host memory
            from .affinity import bind_local_rank
            bind_local_rank(dev, int(os.environ.get("LOCAL_RANK", str(rank))),
                            int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
    else:
        dev = torch.device("cpu")
    # FA_FORCE_PG=1 keeps a process group (and every collective) at world size 1, so a
    # one-GPU box exercises the RCCL code paths of the multi-GPU run
    force = world <= 1 and os.environ.get("FA_FORCE_PG") == "1"
    if world <= 1 and not force:
        return Comm(0, 1, dev, "none")
    if force:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            from .launch import free_port
            os.environ["MASTER_PORT"] = str(free_port())
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    # FA_DIST_BACKEND=gloo lets several ranks share one GPU (tests on a 1-GPU box);
    # production GPU runs use RCCL ("nccl"), one process per GPU.
    be = backend or os.environ.get("FA_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
    if be == "nccl":
        # one process per GPU: RCCL cannot run two ranks of one communicator on one device
        # (a launcher that gives every rank exactly one visible GPU through
        # HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES shows device_count() == 1: no check)
        n_local = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
        n_dev = torch.cuda.device_count()
        # one visible GPU is fine when the launcher narrowed each rank's view to its own
        # GPU; without such a per-rank variable the ranks would share the device
        narrowed = any(os.environ.get(v) for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                   "CUDA_VISIBLE_DEVICES"))
        if n_local > n_dev and not (n_dev == 1 and narrowed):
            raise RuntimeError(f"{n_local} local ranks but {n_dev} visible GPUs: RCCL needs one GPU per rank "
                               "(FA_DIST_BACKEND=gloo lets ranks share a GPU for tests)")
    if not dist.is_initialized():
        kw = dict(backend=be, timeout=timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
        if be == "nccl" and dist.get_world_size() > 1:
            _check_one_gpu_per_rank(dev)
        elif dev.type == "cuda" and dist.get_world_size() > 1:
            # gloo ranks sharing a GPU split its CPU slice (parallel.affinity)
            from .affinity import refine_for_shared_gpu
            try:
                refine_for_shared_gpu(_gpu_key(dev), dist.distributed_c10d._get_default_store(),   # noqa: SLF001
                                      dist.barrier)
            except (RuntimeError, AttributeError, ValueError):
                pass
    return Comm(dist.get_rank(), dist.get_world_size(), dev, be, force=force)


def _gpu_key(dev, props=None, host: str | None = None) -> str:
    """This host's identity of the rank's GPU, which a launcher that narrows every rank's
    view to "device 0" does not hide: its PCI address (domain:bus:device, unique on a
    host), else its UUID unless that is blank or all zeros (a build reporting
    one UUID for every device would fail every rank after the first), else the visible-
    devices variable and index."""
    import socket
    from .affinity import gpu_bdf
    props = props if props is not None else torch.cuda.get_device_properties(dev)
    host = host if host is not None else socket.gethostname()
    ident = None
    try:
        if int(props.pci_bus_id) or int(props.pci_device_id) or int(props.pci_domain_id):
            ident = "pci:" + gpu_bdf(props)
    except (AttributeError, TypeError, ValueError):
        ident = None
    if ident is None:
        u = str(getattr(props, "uuid", "") or "")
        if u.strip("0-{}").strip() and u.lower() not in ("none", "null"):
            ident = "uuid:" + u
    if ident is None:
        vis = next((os.environ.get(v) for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                "CUDA_VISIBLE_DEVICES") if os.environ.get(v)), "")
        ident = f"vis:{vis}/{getattr(dev, 'index', dev)}"
    return f"fa_gpu/{host}/{ident}"


def _check_one_gpu_per_rank(dev, store=None, key: str | None = None, rank: int | None = None) -> None:
    """RCCL ranks of one communicator must not share a GPU, also when each rank's
    *_VISIBLE_DEVICES shows it a single device (the same value exported to
    every local rank).  Every rank counts itself under its GPU's key in the rendezvous
    store: a second rank on the same GPU sees 2 and fails fast."""
    store = store if store is not None else dist.distributed_c10d._get_default_store()     # noqa: SLF001
    n = store.add(key if key is not None else _gpu_key(dev), 1)
    if n > 1:
        r = dist.get_rank() if rank is None else rank
        raise RuntimeError(f"rank {r} shares its GPU with another rank: RCCL needs one GPU per rank "
                           "(FA_DIST_BACKEND=gloo lets ranks share a GPU for tests)")


def shutdown_comm(comm: Comm) -> None:
    """Leave the process group.  The closing barrier is skipped while an exception
    propagates (called from a ``finally``): the peers may be blocked in another
    collective, and a failed rank must exit rather than wait for them (fail fast)."""
    import sys
    if comm.distributed and dist.is_initialized():
        failing = sys.exc_info()[0] is not None
        try:
            if not failing:
                comm.barrier()
        finally:
            if failing and comm.backend == "nccl":
                # a clean destroy would wait for the peers' pending collectives
                try:
                    dist.distributed_c10d._abort_process_group()   # noqa: SLF001
                    return
                except Exception:
                    pass
            dist.destroy_process_group()


__all__ = ["Comm", "init_comm", "shutdown_comm", "pickle"]
