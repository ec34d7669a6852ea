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
