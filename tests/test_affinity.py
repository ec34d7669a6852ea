"""Per-rank NUMA / CPU placement (parallel.affinity) on a fake sysfs tree: 8 GPUs on two
NUMA nodes of 64 CPUs each; every local rank binds to its GPU's node, the node's CPUs
split evenly among the ranks whose GPUs sit there (each rank reads its own
byte range, through its own pinned ring and H2D copies)."""
import os

import pytest

from fastapriori_amd.parallel.affinity import parse_cpulist, plan_affinity


def _fake_sysfs(root, gpus):
    for bdf, node, cpus in gpus:
        d = os.path.join(root, "bus", "pci", "devices", bdf)
        os.makedirs(d)
        with open(os.path.join(d, "numa_node"), "w") as f:
            f.write(f"{node}\n")
        with open(os.path.join(d, "local_cpulist"), "w") as f:
            f.write(cpus + "\n")
        with open(os.path.join(d, "class"), "w") as f:
            f.write("0x120000\n")


GPUS = [(f"0000:{0x05 + 0x10 * i:02x}:00.0", 0 if i < 4 else 1, "0-63" if i < 4 else "64-127") for i in range(8)]


def test_parse_cpulist():
    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []


@pytest.mark.parametrize("lr", range(8))
def test_each_rank_gets_its_nodes_share(tmp_path, lr):
    _fake_sysfs(str(tmp_path), GPUS)
    bdfs = [g[0] for g in GPUS]
    p = plan_affinity(lr, bdfs, list(range(128)), str(tmp_path))
    node = 0 if lr < 4 else 1
    j = lr % 4
    assert p["node"] == node and p["peers"] == 4
    assert p["cpus"] == list(range(64 * node + 16 * j, 64 * node + 16 * (j + 1)))
    assert p["threads"] == 16


def test_allowed_cpus_restrict_the_share(tmp_path):
    # a cgroup that leaves this process CPUs 0-31 and 64-95 only
    _fake_sysfs(str(tmp_path), GPUS)
    allowed = list(range(0, 32)) + list(range(64, 96))
    bdfs = [g[0] for g in GPUS]
    shares = [plan_affinity(lr, bdfs, allowed, str(tmp_path))["cpus"] for lr in range(8)]
    assert shares[0] == list(range(0, 8)) and shares[3] == list(range(24, 32))
    assert shares[4] == list(range(64, 72)) and shares[7] == list(range(88, 96))
    assert len({c for s in shares for c in s}) == 64          # disjoint, all used


def test_narrowed_view_spreads_ranks_over_nodes(tmp_path):
    # every rank sees only its own GPU (HIP_VISIBLE_DEVICES=<its gpu>): its node's CPUs,
    # shared by local_world / nodes = 4 ranks
    _fake_sysfs(str(tmp_path), GPUS)
    p = plan_affinity(0, [GPUS[5][0]], list(range(128)), str(tmp_path), local_world=8)
    assert p["node"] == 1 and p["peers"] == 4 and p["threads"] == 16
    assert set(p["cpus"]) <= set(range(64, 128))


def test_no_locality_means_no_binding(tmp_path):
    p = plan_affinity(0, ["0000:99:00.0"], list(range(16)), str(tmp_path))
    assert p["cpus"] == [] and p["threads"] == 0


def test_narrowed_view_blocked_gpu_order_gets_disjoint_slices(tmp_path):
    # GPUs 0-3 on node 0 and 4-7 on node 1 handed to local ranks 0-7 in order,
    # each rank seeing only its own GPU: the slice comes from the GPU's position among its
    # node's GPUs, so the four ranks of a node get four disjoint slices
    _fake_sysfs(str(tmp_path), GPUS)
    shares = [plan_affinity(lr, [GPUS[lr][0]], list(range(128)), str(tmp_path), local_world=8)["cpus"]
              for lr in range(8)]
    assert all(len(s) == 16 for s in shares)
    assert len({c for s in shares for c in s}) == 128


def test_narrowed_view_ignores_non_amd_display_devices(tmp_path):
    # a management VGA on node 0 (vendor 0x1a03) is no peer of the GPUs there
    _fake_sysfs(str(tmp_path), GPUS)
    d = os.path.join(str(tmp_path), "bus", "pci", "devices", "0000:01:00.0")
    os.makedirs(d)
    for name, val in (("numa_node", "0"), ("local_cpulist", "0-63"), ("class", "0x030000"), ("vendor", "0x1a03")):
        with open(os.path.join(d, name), "w") as f:
            f.write(val + "\n")
    p = plan_affinity(0, [GPUS[0][0]], list(range(128)), str(tmp_path), local_world=8)
    assert p["peers"] == 4 and p["cpus"] == list(range(0, 16))


class _Props:
    def __init__(self, bus, dev=0, dom=0, uuid=""):
        self.pci_bus_id, self.pci_device_id, self.pci_domain_id, self.uuid = bus, dev, dom, uuid


def test_gpu_key_uses_pci_address_not_a_shared_uuid():
    # a ROCm build reporting the same (or an all-zero) UUID for every GPU must
    # not make distinct GPUs collide; the PCI address keys them
    from fastapriori_amd.parallel.comm import _gpu_key
    same = "00000000-0000-0000-0000-000000000000"
    a = _gpu_key(0, _Props(0x05, uuid=same), host="h")
    b = _gpu_key(0, _Props(0x15, uuid=same), host="h")
    assert a != b and a.startswith("fa_gpu/h/pci:0000:05:00.0")
    # no PCI address: a real UUID keys it; an all-zero one does not
    assert _gpu_key(0, _Props(0, uuid="GPU-1234abcd"), host="h").endswith("uuid:GPU-1234abcd")
    assert "uuid" not in _gpu_key(0, _Props(0, uuid=same), host="h")


def test_one_gpu_per_rank_check_on_a_store():
    from datetime import timedelta

    import torch.distributed as dist

    from fastapriori_amd.parallel.comm import _check_one_gpu_per_rank, _gpu_key
    store = dist.HashStore()
    store.set_timeout(timedelta(seconds=5))
    k0 = _gpu_key(0, _Props(0x05), host="h")
    k1 = _gpu_key(1, _Props(0x15), host="h")
    _check_one_gpu_per_rank(None, store, k0, rank=0)
    _check_one_gpu_per_rank(None, store, k1, rank=1)          # another GPU: fine
    with pytest.raises(RuntimeError, match="shares its GPU"):
        _check_one_gpu_per_rank(None, store, k0, rank=2)      # a second rank on GPU 0


def test_ranks_sharing_one_gpu_split_its_node(tmp_path):
    # gloo ranks sharing the one visible GPU (the multi-rank rehearsal): bind_local_rank
    # plans with that GPU repeated per local rank, so the node's CPUs split 8 ways
    _fake_sysfs(str(tmp_path), GPUS)
    bdfs = [GPUS[5][0]] * 8
    shares = [plan_affinity(lr, bdfs, list(range(128)), str(tmp_path))["cpus"] for lr in range(8)]
    assert all(len(s) == 8 for s in shares)
    assert len({c for s in shares for c in s}) == 64 and set().union(*shares) == set(range(64, 128))


def test_ranks_sharing_a_gpu_split_its_slice_after_rendezvous():
    # gloo ranks on one GPU were bound to the GPU's whole slice (a narrowed view cannot tell
    # them apart); after the rendezvous the k sharers split it k ways, disjoint
    from fastapriori_amd.parallel.affinity import shared_slice
    slice_ = list(range(160, 192))
    parts = [shared_slice(slice_, i, 8) for i in range(8)]
    assert all(len(p) == 4 for p in parts) and sorted(c for p in parts for c in p) == slice_
    # more sharers than CPUs: one CPU each (shared, but never empty)
    assert [shared_slice([3, 4], i, 3) for i in range(3)] == [[3], [3], [4]]


def test_refine_binds_through_the_store(monkeypatch):
    from fastapriori_amd.parallel import affinity
    calls = {}
    monkeypatch.setattr(affinity.os, "sched_setaffinity", lambda pid, cpus: calls.setdefault("cpus", list(cpus)))

    class Store:
        def __init__(self):
            self.v = {}

        def add(self, k, d):
            self.v[k] = self.v.get(k, 0) + d
            return self.v[k]
    st = Store()
    st.add("fa_place/g", 3)                     # three other sharers arrived first
    affinity.PLACEMENT.clear()
    affinity.PLACEMENT.update(node=0, cpus=list(range(32)), threads=32, peers=4)
    monkeypatch.setenv("FA_NUM_THREADS", "2")
    p = affinity.refine_for_shared_gpu("g", st, lambda: None)
    assert p["gpu_sharers"] == 4 and p["cpus"] == list(range(24, 32)) and calls["cpus"] == list(range(24, 32))
    affinity.PLACEMENT.clear()
