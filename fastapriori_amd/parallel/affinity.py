"""Per-rank CPU / NUMA placement on a multi-GPU node.

One process per GPU (torchrun).  Each rank's host work -- the 16-slot pread ring
into pinned memory, the host-to-device copies, the C++ parser and writer threads --
belongs on the CPUs of its GPU's NUMA node: a pinned buffer on the far socket
crosses the inter-socket link on every H2D copy, and the per-rank end-to-end read
is bound by exactly those copies (docs/PERF.md, the reference's window).  SURVEY
X1: every rank reads its own byte range of D.dat.

The plan: the GPU's PCI address (torch device properties) names its sysfs node
``/sys/bus/pci/devices/<bdf>/{numa_node,local_cpulist}``; the node's CPUs that this
process may use are split evenly among the local ranks whose GPUs sit on the same
node, and the rank binds to its slice (``os.sched_setaffinity``) before anything
pins host memory.  Its host thread count becomes the slice size.
"""
from __future__ import annotations

import os


def parse_cpulist(text: str) -> list[int]:
    """sysfs cpulist ("0-3,8,10-11") -> sorted CPU ids."""
    out: set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return sorted(out)


def gpu_bdf(props) -> str:
    """PCI address domain:bus:device.function of a torch device's properties."""
    return f"{int(props.pci_domain_id):04x}:{int(props.pci_bus_id):02x}:{int(props.pci_device_id):02x}.0"


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def gpu_node(bdf: str, sysfs: str = "/sys") -> tuple[int, list[int]]:
    """(NUMA node, local CPUs) of the PCI device bdf; (-1, []) when sysfs does not say."""
    base = os.path.join(sysfs, "bus", "pci", "devices", bdf)
    node = _read(os.path.join(base, "numa_node"))
    cpus = _read(os.path.join(base, "local_cpulist"))
    return (int(node) if node not in (None, "") else -1), (parse_cpulist(cpus) if cpus else [])


def plan_affinity(local_rank: int, bdfs: list[str], allowed: list[int], sysfs: str = "/sys",
                  local_world: int | None = None) -> dict:
    """CPU set and thread count of local rank ``local_rank``.

    bdfs: the PCI address of every local rank's GPU when the process sees all of them
    (one entry per local rank), or only its own (a launcher narrowed the view: then the
    rank's peers on the node are unknown and ``local_world`` ranks are assumed spread
    evenly over the nodes that have GPUs).  allowed: the CPUs this process may run on.
    Returns {"node", "cpus", "threads", "peers"}; cpus is empty when sysfs gives no
    locality (no binding then)."""
    allowed_set = set(allowed)
    mine = bdfs[local_rank] if len(bdfs) > local_rank else bdfs[0]
    node, local = gpu_node(mine, sysfs)
    cpus = [c for c in local if c in allowed_set]
    if not cpus:
        return {"node": node, "cpus": [], "threads": 0, "peers": 1}
    if len(bdfs) > 1:
        peers = [r for r, b in enumerate(bdfs) if gpu_node(b, sysfs)[0] == node]
        j, n = peers.index(local_rank), len(peers)
    else:
        # narrowed view: the rank's peers are unknown, but its GPU's position
        # among the node's GPUs in sysfs (PCI order) gives every GPU of the node its own
        # slice, whatever order the launcher hands GPUs to local ranks in
        same = [b for b, nd in _gpu_devices(sysfs) if nd == node]
        if mine.lower() in same:
            j, n = same.index(mine.lower()), len(same)
        else:
            # not listed: an even spread of the local ranks over the GPUs' nodes (>= 1)
            lw = max(1, local_world or 1)
            nodes = max(1, len({nd for _, nd in _gpu_devices(sysfs) if nd >= 0}) or 1)
            n = max(1, -(-lw // nodes))
            j = (local_rank // nodes) % n
    part = cpus[j * len(cpus) // n:(j + 1) * len(cpus) // n] or cpus
    return {"node": node, "cpus": part, "threads": len(part), "peers": n}


def _gpu_devices(sysfs: str) -> list[tuple[str, int]]:
    """(bdf, NUMA node) of the AMD display / processing-accelerator PCI devices (class
    0x03 / 0x12, vendor 0x1002 when sysfs names one: a board's management VGA is not a
    peer), in PCI address order."""
    base = os.path.join(sysfs, "bus", "pci", "devices")
    out = []
    try:
        names = sorted(os.listdir(base))
    except OSError:
        return out
    for b in names:
        cls = _read(os.path.join(base, b, "class")) or ""
        vendor = _read(os.path.join(base, b, "vendor"))
        if cls.startswith(("0x03", "0x12")) and vendor in (None, "0x1002"):
            node = _read(os.path.join(base, b, "numa_node"))
            out.append((b.lower(), int(node) if node not in (None, "") else -1))
    return out


PLACEMENT: dict = {}          # this process's binding (recorded by bench.py per rank)


def bind_local_rank(dev, local_rank: int, local_world: int, sysfs: str = "/sys") -> dict:
    """Bind this process to its GPU's share of NUMA-local CPUs (before any pinned
    allocation) and size its host threads to it.  A no-op without sysfs locality, on the
    CPU device, or with FA_NUM_THREADS set (an explicit host thread count wins)."""
    from ..utils import env
    PLACEMENT.clear()
    if dev.type != "cuda" or not hasattr(os, "sched_setaffinity"):
        return PLACEMENT
    import torch
    n = torch.cuda.device_count()
    narrowed = any(os.environ.get(v) for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                               "CUDA_VISIBLE_DEVICES"))
    try:
        if n == local_world:
            bdfs = [gpu_bdf(torch.cuda.get_device_properties(i)) for i in range(n)]
            idx = local_rank
        elif n == 1 and local_world > 1 and not narrowed:
            # every local rank on the one visible GPU (gloo ranks sharing a card: tests, the
            # multi-rank rehearsal): the node's CPUs split among all of them
            bdfs = [gpu_bdf(torch.cuda.get_device_properties(dev))] * local_world
            idx = local_rank
        else:
            bdfs = [gpu_bdf(torch.cuda.get_device_properties(dev))]
            idx = 0
        plan = plan_affinity(idx, bdfs, sorted(os.sched_getaffinity(0)), sysfs, local_world)
    except (RuntimeError, AttributeError, ValueError, OSError):
        return PLACEMENT
    if plan["cpus"]:
        try:
            os.sched_setaffinity(0, plan["cpus"])
        except OSError:
            return PLACEMENT
        if not os.environ.get("FA_NUM_THREADS"):
            env.set_num_threads(plan["threads"])
    PLACEMENT.update(plan)
    return PLACEMENT


def shared_slice(cpus: list[int], idx: int, n: int) -> list[int]:
    """Sharer idx of n's part of a GPU's CPU slice (at least one CPU each)."""
    part = cpus[idx * len(cpus) // n:(idx + 1) * len(cpus) // n]
    return part or [cpus[idx % len(cpus)]]


def refine_for_shared_gpu(key: str, store, barrier) -> dict:
    """Ranks sharing one GPU (gloo ranks on a one-GPU box: tests, the 8-rank rehearsal)
    were each bound to that GPU's whole CPU slice by bind_local_rank, which cannot tell
    them apart before the process group exists.  After it does: every rank counts itself
    under its GPU's key in the rendezvous store, and the k ranks on one GPU split its
    slice k ways (disjoint CPU sets, host threads sized to them).  No-op without a
    binding or when the GPU is the rank's own."""
    from ..utils import env
    if not PLACEMENT.get("cpus"):
        return PLACEMENT
    idx = int(store.add(f"fa_place/{key}", 1)) - 1
    barrier()
    n = int(store.add(f"fa_place/{key}", 0))
    if n <= 1:
        return PLACEMENT
    part = shared_slice(list(PLACEMENT["cpus"]), idx, n)
    try:
        os.sched_setaffinity(0, part)
    except OSError:
        return PLACEMENT
    if not os.environ.get("FA_NUM_THREADS"):
        env.set_num_threads(len(part))
    PLACEMENT.update(cpus=part, threads=len(part), gpu_sharers=n)
    return PLACEMENT

