"""GPU correctness at scale: the default device path (fused compression, queue-
scheduled pair kernel, device level bundles, the slab kernel's class layout,
transaction trimming) against the C++ CPU miner on the same synthetic databases.

* 2M Quest rows (T10I4 shape), default MinerConfig: trimming is live
  (trim_min_rows = 1 << 20) and the device level bundles run.
* 400K T40I10 rows at min_sup 0.5 %: >= 8 levels (the deep-k path; trimming forced
  on so every level's trim + re-layout runs).
Both compare the complete itemset -> count maps (exact integers).
Reference semantics: FastApriori.scala:46-160.
"""
import pytest
import torch

from fastapriori_amd.models.apriori import FastApriori, MinerConfig
from fastapriori_amd.parallel.comm import Comm
from fastapriori_amd.utils.io import generate_shard
from fastapriori_amd.utils.metrics import Logger

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _mine(shard, ms, **kw):
    cfg = MinerConfig(min_support=ms, **kw)
    return FastApriori(ms, config=cfg, logger=Logger(0, enabled=False)).run(shard)


def test_t10_2m_rows_default_config_matches_cpu():
    cpu = generate_shard(2_000_000, Comm(), "cpu", 10.0, 4.0, 2000, 1000, 3)
    ref = _mine(cpu, 0.001)
    m = FastApriori(0.001, config=MinerConfig(min_support=0.001), logger=Logger(0, enabled=False))
    got = m.run(cpu.to(DEV))
    assert len(ref.levels) >= 10
    assert [len(x) for x in got.levels] == [len(x) for x in ref.levels]
    assert got.as_dict() == ref.as_dict()
    assert got.items == ref.items


def test_t40_deep_levels_match_cpu():
    cpu = generate_shard(400_000, Comm(), "cpu", 40.0, 10.0, 2000, 1000, 3)
    ref = _mine(cpu, 0.005, trim_min_rows=0)
    got = _mine(cpu.to(DEV), 0.005, trim_min_rows=0)
    assert len(ref.levels) >= 8
    assert [len(x) for x in got.levels] == [len(x) for x in ref.levels]
    assert got.as_dict() == ref.as_dict()


@pytest.mark.parametrize("frac", [0.7, 1.01])
def test_t40_window_trim_matches_cpu(frac):
    """Window-by-window levels counted over each window's own rows (FastApriori._window_rows:
    rows holding >= k of the window's items, trimmed + a bitmap of those items): every
    window trimmed (frac 1.01) and the cost model's choice (0.7) both give the CPU miner's
    exact counts, and the trimmed windows really ran."""
    from fastapriori_amd.tuning import override
    cpu = generate_shard(400_000, Comm(), "cpu", 40.0, 10.0, 2000, 1000, 5)
    ref = _mine(cpu, 0.005, trim_min_rows=0)
    with override(window_trim=True, window_trim_est_frac=frac, window_trim_rows_frac=max(frac, 0.97),
                  window_trim_cost=0.0 if frac > 1 else 100.0, window_trim_min_rows=0):
        m = FastApriori(0.005, config=MinerConfig(min_support=0.005, trim_min_rows=0), logger=Logger(0, enabled=False))
        got = m.run(cpu.to(DEV))
    assert m.stats.get("device_multipass", 0) >= 1, m.stats
    if frac > 1:
        assert m.stats.get("window_trims", 0) >= m.stats["device_multipass"], m.stats
    assert [len(x) for x in got.levels] == [len(x) for x in ref.levels]
    assert got.as_dict() == ref.as_dict()
