"""Device-resident level bundles (FastApriori._mine_device; csrc/hip/gen.hip
fa_hip_dl_*, csrc/hip/levels.hip) against the host-driven level loop and the C++
CPU miner: identical itemsets, counts and level order (rows lexicographic).

Covers unit and weighted (dedup) layouts, transaction trimming inside a device
bundle, max_level, levels that need several accumulator passes (T40I10 shape,
counted on the device window by window), wide vocabularies (F1 > 4096), prefixes
past the records' 12 inline ids, and an empty F_2.
Reference semantics: FastApriori.scala:110-160.
"""
import re

import numpy as np
import pytest
import torch

import fastapriori_amd.models.apriori as ap
from fastapriori_amd.tuning import TUNING
from fastapriori_amd.models.apriori import FastApriori, MinerConfig
from fastapriori_amd.models.oracle import mining_log_lines
from fastapriori_amd.parallel.comm import Comm
from fastapriori_amd.utils.io import generate_shard
from fastapriori_amd.utils.metrics import Logger

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _mine(shard, ms, **kw):
    cfg = MinerConfig(min_support=ms, **kw)
    m = FastApriori(ms, config=cfg, logger=Logger(0, enabled=False))
    return m.run(shard), m.stats


def _same(a, b):
    assert [len(x) for x in a.levels] == [len(x) for x in b.levels]
    for x, y in zip(a.levels, b.levels):
        assert np.array_equal(x, y)
    for x, y in zip(a.counts, b.counts):
        assert np.array_equal(x, y)
    assert a.items == b.items


@pytest.mark.parametrize("n,ms,kw", [
    (300_000, 0.002, {}),
    (300_000, 0.002, {"dedup": "on"}),
    (1_200_000, 0.002, {"trim_min_rows": 0}),
    (200_000, 0.003, {"max_level": 5}),
    (50_000, 0.004, {"pair_strategy": "gram"}),
])
def test_device_levels_match_host_loop(tune, n, ms, kw):
    cpu = generate_shard(n, Comm(), "cpu", 10.0, 4.0, 2000, 1000, 5)
    g = cpu.to(DEV)
    got, st = _mine(g, ms, **kw)
    tune(device_levels=False)
    ref, st2 = _mine(g, ms, **kw)
    assert "device_bundles" not in st2
    if len(ref.levels) >= 3:
        assert st.get("device_bundles", 0) >= 1
    _same(got, ref)
    if n <= 300_000:
        cref, _ = _mine(cpu, ms, **kw)
        assert got.as_dict() == cref.as_dict()


def test_multipass_level_stays_on_device(tune):
    # T40I10 at a lower support: levels whose candidates need several accumulator passes
    # are counted on the device window by window (FastApriori._dl_multipass);
    # dl_multi=False hands them to the host loop instead
    cpu = generate_shard(150_000, Comm(), "cpu", 40.0, 10.0, 2000, 1000, 3)
    ref, _ = _mine(cpu, 0.006)
    assert len(ref.levels) >= 6
    got, st = _mine(cpu.to(DEV), 0.006)
    assert st.get("device_multipass", 0) >= 1 and st.get("host_levels", 0) == 0, st
    assert st["device_levels"] >= len(ref.levels) - 2 and "fallbacks" not in st
    assert got.as_dict() == ref.as_dict()
    _same(got, ref)
    tune(dl_multi=False)
    got2, st2 = _mine(cpu.to(DEV), 0.006)
    assert st2.get("host_levels", 0) >= 1
    _same(got2, ref)


def test_blocked_gram_bitmap_feeds_multipass_levels(tune):
    # the Gram's full bitmap in 8-word blocks (count.hip BmView) is reused by the
    # window-by-window levels' slab copies (slab_copy_bm, negative stride): same
    # results as with the row-major bitmap and the host loop
    cpu = generate_shard(150_000, Comm(), "cpu", 40.0, 10.0, 2000, 1000, 3)
    ref, _ = _mine(cpu, 0.006)
    got, st = _mine(cpu.to(DEV), 0.006, pair_strategy="gram")
    assert st.get("bm_blocked") and st.get("device_multipass", 0) >= 1, st
    _same(got, ref)
    tune(bitmap_blocked=False)
    got2, st2 = _mine(cpu.to(DEV), 0.006, pair_strategy="gram")
    assert not st2.get("bm_blocked")
    _same(got2, ref)


def _multipass_lds(ref, accb: int = 4) -> int:
    """An LDS budget in which level 3's used items (at most the items of F_2) fit 4-word
    slabs (slab rows 48 B) with room for ~|F_3| / 4 accumulators of accb bytes: level 3
    then needs several passes."""
    F1, F3 = len(ref.levels[0]), len(ref.levels[2])
    U = int(np.unique(np.asarray(ref.levels[1])).size)
    return U * 48 + accb * max(1024, F3 // 4) + 2 * F1 + 256


def test_small_lds_forces_device_multipass(tune):
    # a shrunk LDS budget turns T10I4 levels into multi-pass ones: windows, trimming and
    # the used items' bitmap on the unit and the weighted (dedup) layout
    import fastapriori_amd.ops.primitives as prim
    cpu = generate_shard(200_000, Comm(), "cpu", 10.0, 4.0, 2000, 1000, 4)
    ref, _ = _mine(cpu, 0.002)
    for dd in ("off", "on"):
        # unit weights count into packed u16 accumulators (2 B each)
        tune(slab_lds_bytes=_multipass_lds(ref, 2 if dd == "off" and TUNING.dl_acc16 else 4))
        got, st = _mine(cpu.to(DEV), 0.002, dedup=dd, trim_min_rows=0)
        assert st.get("device_multipass", 0) >= 1, st
        _same(got, ref)


def test_deep_database_all_levels_on_device():
    # >= 14 levels (prefixes past the 12 ids a piece record holds inline: levels.hip gpre)
    cpu = generate_shard(120_000, Comm(), "cpu", 40.0, 10.0, 2000, 1000, 3)
    ref, _ = _mine(cpu, 0.005)
    assert len(ref.levels) >= 14
    got, st = _mine(cpu.to(DEV), 0.005)
    assert st.get("host_levels", 0) == 0 and st["device_levels"] >= len(ref.levels) - 2, st
    assert "fallbacks" not in st
    _same(got, ref)


def test_device_levels_no_frequent_pairs():
    cpu = generate_shard(20_000, Comm(), "cpu", 10.0, 4.0, 2000, 1000, 2)
    got, _ = _mine(cpu.to(DEV), 0.2)
    ref, _ = _mine(cpu, 0.2)
    assert got.as_dict() == ref.as_dict()


def test_device_levels_repeat_runs_identical():
    # buffers (workspace, control block, F sizes) are reused across runs
    cpu = generate_shard(100_000, Comm(), "cpu", 10.0, 4.0, 2000, 1000, 7)
    g = cpu.to(DEV)
    m = FastApriori(0.003, config=MinerConfig(min_support=0.003), logger=Logger(0, enabled=False))
    a = m.run(g)
    b = m.run(g)
    c = FastApriori(0.002, config=MinerConfig(min_support=0.002), logger=Logger(0, enabled=False)).run(g)
    _same(a, b)
    cref, _ = _mine(cpu, 0.002)
    assert c.as_dict() == cref.as_dict()


def test_wide_f1_generates_on_device_without_fallbacks():
    # F1 = 6319 > 4096: the generator's lanes hold two bitset words each
    # (gen.hip ag_row_bits<2>); no level may fall back to the host generator
    cpu = generate_shard(300_000, Comm(), "cpu", 10.0, 4.0, 6000, 12000, 3)
    got, st = _mine(cpu.to(DEV), 0.0004)
    ref, _ = _mine(cpu, 0.0004)
    assert len(got.items) > 4096 and len(ref.levels) >= 8
    # every level >= 3 in device bundles (gen.hip: 2 bitset words per lane, ctl bitset of F1 bits)
    assert st.get("host_levels", 0) == 0 and st["device_levels"] >= len(ref.levels) - 2, st
    assert "fallbacks" not in st
    assert got.as_dict() == ref.as_dict()
    _same(got, ref)


def test_f2_stays_on_device_until_the_flush(tune):
    # F_2 compacted on the device (no readback between the pair kernel and the first
    # bundle): same itemsets, and the reference's log lines in level order
    import io
    cpu = generate_shard(200_000, Comm(), "cpu", 10.0, 4.0, 2000, 1000, 9)
    g = cpu.to(DEV)
    logs = {}
    for dl in (True, False):
        tune(device_levels=dl)
        buf = io.StringIO()
        lg = Logger(0, enabled=True)
        lg.stream = buf
        m = FastApriori(0.002, config=MinerConfig(min_support=0.002), logger=lg)
        res = m.run(g)
        if dl:
            assert m._f2_defer and m.stats.get("device_bundles", 0) >= 1
            got = res
        else:
            ref = res
        logs[dl] = [re.sub(r"(Use Time \d+ items )\d+$", r"\g<1>#", l[5:]) for l in buf.getvalue().splitlines()
                    if l.startswith("==== ")]
    _same(got, ref)
    assert got.as_dict() == _mine(cpu, 0.002)[0].as_dict()
    # both loops print exactly the reference's lines (FastApriori.scala:107-127), replayed
    # from the itemsets by the oracle's loop
    want = mining_log_lines(len(got.items), got.as_dict().keys())
    assert logs[True] == want and logs[False] == want


def test_u16_window_accumulators_drain_mid_run(tune):
    # packed-u16 window accumulators drain into the u32 counts every
    # 65535 / (SW * 64) slabs.  One workgroup walks every slab (fa_hip_debug_slab_max_wg),
    # and items 0-3 sit in every row, so their level-3 and level-4 counters pass 65535
    # several times: a broken mid-run drain would wrap them.
    import fastapriori_amd.ops.primitives as prim
    from fastapriori_amd.ops import _native
    from fastapriori_amd.utils.io import parse_bytes
    rng = np.random.default_rng(11)
    n = 300_000
    extra = np.argsort(rng.random((n, 37)), axis=1)[:, :5] + 4
    text = "\n".join("0 1 2 3 " + " ".join(map(str, r)) for r in extra.tolist()) + "\n"
    cpu = parse_bytes(text.encode(), device=torch.device("cpu"))
    ref, _ = _mine(cpu, 0.002)
    assert max(ref.counts[2]) > 4 * 65535
    tune(slab_lds_bytes=_multipass_lds(ref, 2))
    hip = _native.hip()
    hip.fa_hip_debug_slab_max_wg(1)
    try:
        got, st = _mine(parse_bytes(text.encode(), device=DEV), 0.002, dedup="off", trim_min_rows=1 << 40)
    finally:
        hip.fa_hip_debug_slab_max_wg(0)
    assert st.get("device_multipass", 0) >= 1, st
    _same(got, ref)


def test_lane_deal_keeps_counts(tune):
    # the bank-aware lane deal (levels.hip k_dl_lane_assign) moves piece records between
    # lanes only: every level identical to the undealt plan, one-pass bundles and
    # window-by-window levels (T40 shape) alike
    for args, ms in (((10.0, 4.0, 2000, 1000), 0.002), ((40.0, 10.0, 2000, 1000), 0.006)):
        cpu = generate_shard(150_000, Comm(), "cpu", *args, 3)
        g = cpu.to(DEV)
        tune(lane_deal_min_rows=-1)
        ref, _ = _mine(g, ms)
        tune(lane_deal_min_rows=0)
        got, st = _mine(g, ms)
        assert st.get("device_bundles", 0) >= 1
        _same(got, ref)


def test_window_items_keep_counts(tune):
    # window-by-window levels whose windows hold only their own used items
    # (TUNING.mp_window_items, ops.primitives.dl_window_plan): every level identical to
    # the level-wide windows, on the T40 shape
    cpu = generate_shard(150_000, Comm(), "cpu", 40.0, 10.0, 2000, 1000, 3)
    g = cpu.to(DEV)
    tune(mp_window_items=False)
    ref, _ = _mine(g, 0.006)
    tune(mp_window_items=True)
    got, st = _mine(g, 0.006)
    assert st.get("device_multipass", 0) >= 1 and "fallbacks" not in st, st
    assert len(ref.levels) >= 6
    _same(got, ref)
