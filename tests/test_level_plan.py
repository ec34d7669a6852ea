"""Planner of the slab level kernel (csrc/host/plan.cpp fa_level_plan), checked on
CPU: ops.primitives.emulate_level_plan executes a plan's pieces and
emulate_slab_records the 48-B records with k_count_slab_rec's exact semantics
(class-layout keep flags, pass-local extension offsets) over a bool bitmap; both
must equal brute-force support counts for every accumulator capacity (many passes
included), prefix length and layout.
"""
import numpy as np
import pytest

from fastapriori_amd.ops.host import apriori_gen


def _level(rng, n_items=14, n_rows=400, k=4, dens=0.45):
    bits = rng.random((n_items, n_rows)) < dens
    # frequent (k-1)-itemsets of this bitmap at a low threshold -> realistic sharing
    from itertools import combinations
    m = k - 1
    prev = []
    for c in combinations(range(n_items), m):
        if np.logical_and.reduce(bits[list(c)]).sum() >= 6:
            prev.append(c)
    return bits, np.array(prev, dtype=np.int32).reshape(-1, m)


@pytest.mark.parametrize("lds_kb", [160, 6, 3])
@pytest.mark.parametrize("k", [3, 5])
def test_level_plan_counts(lds_kb, k):
    # fa_level_plan (one-call planner feeding the GPU level kernel), single- and
    # multi-pass, must reproduce brute-force supports
    from fastapriori_amd.ops.primitives import emulate_level_plan, emulate_slab_records, level_plan_host
    rng = np.random.default_rng(k)
    bits, prev = _level(rng, n_items=16, k=k)
    pidx, eoff, ext = apriori_gen(prev)
    if ext.size == 0:
        pytest.skip("no candidates")
    P = prev[pidx]
    rc, info, passes, buf = level_plan_host(P, eoff, ext, bits.shape[0], (bits.shape[1] + 63) // 64,
                                            lds_bytes=lds_kb * 1024)
    if rc == 4:                      # no slab fits this LDS budget: the caller uses the bitmap kernel
        assert lds_kb < 8
        return
    assert rc == 0
    assert info[6] >= 1 and (info[6] > 1) == (ext.size > info[2])
    g_of_e = np.repeat(np.arange(pidx.size), np.diff(eoff))
    want = np.array([np.logical_and.reduce(bits[list(P[g]) + [e]]).sum() for g, e in zip(g_of_e, ext)])
    got = emulate_level_plan(bits, info, passes, buf, P.shape[1], ext.size)
    assert np.array_equal(got, want)
    assert np.array_equal(emulate_slab_records(bits, info, passes, buf, ext.size), want)


@pytest.mark.parametrize("k", [7, 11, 15])
def test_slab_records_long_prefixes(k):
    # k_count_slab_rec records hold prefixes of <= 12 ids inline (ids 4-11 in the
    # third int4) and point into gpre beyond that
    from fastapriori_amd.ops.primitives import emulate_slab_records, level_plan_host
    rng = np.random.default_rng(k)
    bits, prev = _level(rng, n_items=16, n_rows=300, k=k, dens=0.88)
    pidx, eoff, ext = apriori_gen(prev)
    if ext.size == 0:
        pytest.skip("no candidates")
    P = prev[pidx]
    rc, info, passes, buf = level_plan_host(P, eoff, ext, bits.shape[0], 5)
    assert rc == 0
    g_of_e = np.repeat(np.arange(pidx.size), np.diff(eoff))
    want = np.array([np.logical_and.reduce(bits[list(P[g]) + [e]]).sum() for g, e in zip(g_of_e, ext)])
    assert np.array_equal(emulate_slab_records(bits, info, passes, buf, ext.size), want)


def test_level_plan_mixed_prefix_lengths():
    # groups of several levels (different k) in one slab launch: flat prefixes + poff
    from fastapriori_amd.ops.primitives import emulate_level_plan, emulate_slab_records, level_plan_host
    rng = np.random.default_rng(11)
    bits, prev3 = _level(rng, n_items=16, k=4)
    _, prev2 = _level(rng, n_items=16, k=3)
    groups = []
    for prev in (prev2, prev3):
        pidx, eoff, ext = apriori_gen(prev)
        groups.append((prev[pidx], eoff, ext))
    flat = np.concatenate([g[0].ravel() for g in groups]).astype(np.int32)
    poff = np.concatenate([[0], np.cumsum(np.concatenate([np.full(g[0].shape[0], g[0].shape[1]) for g in groups]))])
    eoff = np.concatenate([[0], np.cumsum(np.concatenate([np.diff(g[1]) for g in groups]))])
    ext = np.concatenate([g[2] for g in groups]).astype(np.int32)
    rc, info, passes, buf = level_plan_host(flat, eoff, ext, bits.shape[0], 8, poff=poff)
    assert rc == 0
    want = []
    for P, eo, ex in groups:
        g_of_e = np.repeat(np.arange(P.shape[0]), np.diff(eo))
        want += [np.logical_and.reduce(bits[list(P[g]) + [e]]).sum() for g, e in zip(g_of_e, ex)]
    got = emulate_level_plan(bits, info, passes, buf, 0, ext.size)
    assert np.array_equal(got, np.array(want))
    assert np.array_equal(emulate_slab_records(bits, info, passes, buf, ext.size), np.array(want))


def test_bundled_levels_match_unbundled(monkeypatch, tune):
    # counting later levels from the previous level's candidates must not change results
    import torch
    from fastapriori_amd.models import apriori as ap
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils.io import generate_shard
    sh = generate_shard(20000, Comm(), torch.device("cpu"), 10.0, 4.0, 200, 100, seed=3)
    seen = []
    orig = FastApriori._plan_bundle

    def spy(self, *a):
        b = orig(self, *a)
        seen.append(len(b))
        return b
    monkeypatch.setattr(FastApriori, "_plan_bundle", spy)
    on = FastApriori(0.003, config=MinerConfig(min_support=0.003)).run(sh)
    assert max(seen) > 1 and len(on.levels) >= 5
    tune(bundle_levels=False)
    off = FastApriori(0.003, config=MinerConfig(min_support=0.003)).run(sh)
    assert on.as_dict() == off.as_dict() and on.items == off.items


@pytest.mark.parametrize("k", [3, 5, 7])
@pytest.mark.parametrize("lds_kb", [160, 6])
def test_slab_class_layout_counts(k, lds_kb):
    # plan.cpp cls_layout: sibling pieces in one thread's slots with keep-q / keep-p
    # flags, idle slots padding the wave rows; the record emulation follows the flags
    # slot by slot (k_count_slab_rec<.., kCls>) and must reproduce brute-force supports
    from fastapriori_amd.ops.primitives import emulate_level_plan, emulate_slab_records, level_plan_host
    rng = np.random.default_rng(k + lds_kb)
    bits, prev = _level(rng, n_items=16, n_rows=300, k=k, dens=0.6 if k < 7 else 0.8)
    pidx, eoff, ext = apriori_gen(prev)
    if ext.size == 0:
        pytest.skip("no candidates")
    P = prev[pidx]
    rc, info, passes, buf = level_plan_host(P, eoff, ext, bits.shape[0], 5, lds_bytes=lds_kb * 1024, cls=2)
    assert rc == 0 and info[23] == 1
    g_of_e = np.repeat(np.arange(pidx.size), np.diff(eoff))
    want = np.array([np.logical_and.reduce(bits[list(P[g]) + [e]]).sum() for g, e in zip(g_of_e, ext)])
    assert np.array_equal(emulate_level_plan(bits, info, passes, buf, P.shape[1], ext.size), want)
    assert np.array_equal(emulate_slab_records(bits, info, passes, buf, ext.size), want)
    # every pass's slots are whole steps of the 1024-thread workgroup
    assert all((b - a) % 1024 == 0 for a, b, _ in passes.tolist())


def test_slab_class_layout_chosen_on_deep_levels():
    # a deep downward-closed level has long sibling runs: the class layout's wave-step
    # reads are well below the size-sorted layout's, so the planner takes it (cls=1)
    from itertools import combinations
    from fastapriori_amd.ops.primitives import level_plan_host
    rng = np.random.default_rng(2)
    rows = set()
    for _ in range(40):
        big = np.sort(rng.choice(40, 11, replace=False))
        rows.update(combinations(big.tolist(), 6))
    prev = np.array(sorted(rows), np.int32)
    pidx, eoff, ext = apriori_gen(prev)
    rc, info, passes, buf = level_plan_host(prev[pidx], eoff, ext, 40, 1 << 14, cls=1)
    assert rc == 0
    assert info[22] < 0.85 * info[21] and info[23] == (info[22] < 0.8 * info[21])
    rc0, info0, _, _ = level_plan_host(prev[pidx], eoff, ext, 40, 1 << 14, cls=0)
    assert rc0 == 0 and info0[23] == 0 and info0[22] == 0
