"""HIP kernel numerics: every device op against its CPU reference on the same inputs.

All counts are integers, so the comparison is exact.  Shapes deliberately hit
the edges: T not a multiple of 64, W not a multiple of the kernel tiles,
F1 not a multiple of the 64/128 item tiles, long transactions (>64 items,
which take the LDS-sort tier), and dedup weight classes.
"""
import numpy as np
import pytest
import torch

from fastapriori_amd import ops
from fastapriori_amd.models.apriori import FastApriori, MinerConfig
from fastapriori_amd.ops import _native
from fastapriori_amd.ops.host import apriori_gen
from fastapriori_amd.parallel.comm import Comm
from fastapriori_amd.utils.io import generate_shard, parse_bytes

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_native_library_is_loaded():
    lib = _native.hip()
    assert lib is not None
    import os
    maps = open(f"/proc/{os.getpid()}/maps").read()
    assert "libfa_hip.so" in maps


def _random_db(n, V, max_len, seed, long_rows=0):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len + 1, n)
    if long_rows:
        lens[rng.choice(n, long_rows, replace=False)] = rng.integers(65, 300, long_rows)
    rows = [rng.choice(V, size=min(l, V), replace=False).astype(np.int32) for l in lens]
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum([r.size for r in rows])
    items = np.concatenate(rows) if rows else np.zeros(0, np.int32)
    return torch.from_numpy(off), torch.from_numpy(items.astype(np.int32))


@pytest.mark.parametrize("V", [37, 1000, 20000])
def test_histogram(V):
    _, items = _random_db(5000, V, 30, 1)
    ref = ops.histogram(items, V)
    got = ops.histogram(items.to(DEV), V).cpu()
    assert torch.equal(ref, got)
    # unaligned view
    got2 = ops.histogram(items[1:].contiguous().to(DEV)[0:], V).cpu()
    assert torch.equal(ops.histogram(items[1:].contiguous(), V), got2)


def _prep(n=3000, V=400, max_len=25, seed=0, long_rows=5, F1_frac=0.6):
    off, items = _random_db(n, V, max_len, seed, long_rows)
    rng = np.random.default_rng(seed + 1)
    F1 = int(V * F1_frac)
    perm = rng.permutation(V)
    lut = np.full(V, -1, np.int32)
    lut[perm[:F1]] = np.arange(F1, dtype=np.int32)
    return off, items, torch.from_numpy(lut), F1


def _compress_inputs(off, items, lut):
    cnt = ops.txn_freq_count(off, items, lut)
    kept = torch.nonzero(cnt >= 2).flatten().to(torch.int32)
    roff = torch.zeros(kept.numel() + 1, dtype=torch.int64)
    roff[1:] = torch.cumsum(cnt[kept.long()].long(), 0)
    return cnt, kept, roff


def test_txn_count_and_compress():
    off, items, lut, F1 = _prep()
    cnt, kept, roff = _compress_inputs(off, items, lut)
    gcnt = ops.txn_freq_count(off.to(DEV), items.to(DEV), lut.to(DEV)).cpu()
    assert torch.equal(cnt, gcnt)
    ref = ops.compress(off, items, lut, kept, roff)
    got = ops.compress(off.to(DEV), items.to(DEV), lut.to(DEV), kept.to(DEV), roff.to(DEV)).cpu()
    assert torch.equal(ref, got)
    # long-row tier: wave-per-row rank bitmap instead of the LDS sort
    got = ops.compress(off.to(DEV), items.to(DEV), lut.to(DEV), kept.to(DEV), roff.to(DEV), F1).cpu()
    assert torch.equal(ref, got)


@pytest.mark.parametrize("V,frac", [(900, 0.5), (9000, 0.7)])
def test_compress_long_documents(V, frac):
    # mean row length > 48 -> every row through the wave kernel (F1 > 4096 -> 2 words per lane)
    off, items, lut, F1 = _prep(n=1500, V=V, max_len=400, seed=3, long_rows=0, F1_frac=frac)
    cnt, kept, roff = _compress_inputs(off, items, lut)
    assert torch.equal(cnt, ops.txn_freq_count(off.to(DEV), items.to(DEV), lut.to(DEV)).cpu())
    ref = ops.compress(off, items, lut, kept, roff)
    got = ops.compress(off.to(DEV), items.to(DEV), lut.to(DEV), kept.to(DEV), roff.to(DEV), F1).cpu()
    assert torch.equal(ref, got)


@pytest.mark.parametrize("max_len, long_rows, n", [(80, 0, 4000), (70, 40, 3000), (90, 0, 600)])
def test_compress_staged64(max_len, long_rows, n):
    # mean row length > 16: span-staged counts and the 64-token staged tier (64 KB input span per
    # workgroup; rows of > 64 tokens to the wave tier; wide spans through the unstaged path)
    off, items, lut, F1 = _prep(n=n, V=900, max_len=max_len, seed=max_len + n, long_rows=long_rows)
    assert items.numel() > 16 * n
    cnt, kept, roff = _compress_inputs(off, items, lut)
    assert torch.equal(cnt, ops.txn_freq_count(off.to(DEV), items.to(DEV), lut.to(DEV)).cpu())
    ref = ops.compress(off, items, lut, kept, roff)
    got = ops.compress(off.to(DEV), items.to(DEV), lut.to(DEV), kept.to(DEV), roff.to(DEV), F1).cpu()
    assert torch.equal(ref, got)


def test_row_hash_matches_host():
    off, items, lut, F1 = _prep(seed=3)
    _, kept, roff = _compress_inputs(off, items, lut)
    ranks = ops.compress(off, items, lut, kept, roff)
    h1, h2 = ops.row_hash(roff, ranks)
    g1, g2 = ops.row_hash(roff.to(DEV), ranks.to(DEV))
    assert torch.equal(h1, g1.cpu()) and torch.equal(h2, g2.cpu())


@pytest.mark.parametrize("F1_frac", [0.05, 0.6, 1.0])
def test_bitmaps_pairs_candidates(F1_frac):
    off, items, lut, F1 = _prep(n=5000, V=700, seed=5, F1_frac=F1_frac)
    _, kept, roff = _compress_inputs(off, items, lut)
    ranks = ops.compress(off, items, lut, kept, roff)
    T = kept.numel()
    bm, W = ops.build_bitmaps(roff, ranks, None, T, F1)
    gbm, gW = ops.build_bitmaps(roff.to(DEV), ranks.to(DEV), None, T, F1)
    assert W == gW
    assert torch.equal(bm[:, :W], gbm[:, :W].cpu())
    # horizontal vs gram vs host
    ph = ops.pair_counts_horizontal(roff, ranks, None, F1)
    gph = ops.pair_counts_horizontal(roff.to(DEV), ranks.to(DEV), None, F1, long_rows=False).cpu()
    gpg = ops.pair_counts_gram(gbm, gW, None).cpu()
    assert torch.equal(ph, gph)
    assert torch.equal(torch.triu(ph, 1), torch.triu(gpg, 1))
    if ops.primitives.blocked_bitmaps_ok(None, F1, T):
        # the Gram's 8-word block layout from the wave build, and the Gram on it
        bbm, bW = ops.build_bitmaps(roff.to(DEV), ranks.to(DEV), None, T, F1, blocked=True)
        assert bW == W and torch.equal(bbm.cpu(), ops.primitives.to_blocked(bm))
        assert torch.equal(torch.triu(ph, 1), torch.triu(ops.pair_counts_gram(bbm, bW, None).cpu(), 1))
        # a word window off the block boundary (candidate-mode column slices)
        w0 = min(13, W - 1)
        part = ops.pair_counts_gram(bbm, W - w0, None, w0=w0).cpu()
        assert torch.equal(torch.triu(part, 1), torch.triu(ops.pair_counts_gram(bm, W - w0, None, w0=w0), 1))
    # level-3 candidates from the frequent pairs
    iu = torch.triu_indices(F1, F1, 1)
    pc = ph[iu[0], iu[1]]
    sel = torch.nonzero(pc >= max(1, int(pc.float().quantile(0.7).item()))).flatten()
    prev = torch.stack([iu[0][sel], iu[1][sel]], 1).numpy().astype(np.int32)
    if prev.shape[0] < 3:
        return
    pidx, eoff, ext = apriori_gen(prev)
    if ext.size == 0:
        return
    prefix = torch.from_numpy(prev[pidx].copy())
    ext_t = torch.from_numpy(ext.copy())
    ref = ops.count_candidates(bm, W, prefix, eoff, ext_t, None)
    got = ops.count_candidates(gbm, gW, prefix.to(DEV), eoff, ext_t.to(DEV), None).cpu()
    assert torch.equal(ref, got)
    slab = ops.count_level(roff.to(DEV), ranks.to(DEV), None, T, F1, prev[pidx], eoff, ext, None, kernel="slab")
    assert slab is not None and torch.equal(ref, slab.cpu())


def test_slab_many_passes_and_levels():
    # a deep-level database: many candidates force several accumulator passes
    sh = generate_shard(60000, Comm(), "cpu", 14.0, 6.0, 300, 120, seed=11)
    cfg = dict(min_support=0.004, dedup="off")
    ref = FastApriori(0.004, config=MinerConfig(trim_min_rows=0, level_kernel="bitmap", **cfg)).run(sh)
    got = FastApriori(0.004, config=MinerConfig(trim_min_rows=0, level_kernel="slab", **cfg)).run(sh.to(DEV))
    assert len(ref.levels) >= 4
    assert ref.as_dict() == got.as_dict()


def test_weighted_dedup_paths_match():
    # many duplicate rows -> dedup on; compare full mining cuda vs cpu, both strategies
    sh = generate_shard(20000, Comm(), "cpu", 6.0, 3.0, 50, 60, seed=7)
    res_cpu = FastApriori(0.01, config=MinerConfig(min_support=0.01, dedup="off")).run(sh)
    shg = sh.to(DEV)
    for strat in ("horizontal", "gram"):
        for dd in ("on", "off"):
            r = FastApriori(0.01, config=MinerConfig(min_support=0.01, dedup=dd, pair_strategy=strat)).run(shg)
            assert r.as_dict() == res_cpu.as_dict(), (strat, dd)


def test_recommend_kernel():
    sh = generate_shard(20000, Comm(), "cpu", 8.0, 3.0, 80, 100, seed=9)
    res = FastApriori(0.01, config=MinerConfig(min_support=0.01)).run(sh)
    from fastapriori_amd.models.rules import AssociationRules
    users = generate_shard(3000, Comm(), "cpu", 8.0, 3.0, 80, 100, seed=9, users=True)
    ar = AssociationRules(res)
    ref = ar.recommend_shard(users)
    got = ar.recommend_shard(users.to(DEV)).cpu()
    assert torch.equal(ref, got)


@pytest.mark.parametrize("seed,min_sup", [(9, 0.01), (11, 0.004)])
def test_rules_device_matches_host(seed, min_sup):
    # subset index, level-wise cut, ordering and antecedent emission on the GPU
    # against the C++ builder, on a mined result with several levels
    from fastapriori_amd.models.rules import AssociationRules
    sh = generate_shard(30000, Comm(), "cpu", 10.0, 4.0, 60, 80, seed=seed)
    res = FastApriori(min_sup, config=MinerConfig(min_support=min_sup)).run(sh)
    assert len(res.levels) >= 4
    host = AssociationRules(res).rules()
    dev = AssociationRules(res, device=DEV)
    got = dev.rules()
    assert got.n_rules == host.n_rules > 0
    assert np.array_equal(got.ante_off, host.ante_off)
    assert np.array_equal(got.ante, host.ante)
    assert np.array_equal(got.cons, host.cons)
    assert np.array_equal(got.conf, host.conf)
    assert got.level_stats == host.level_stats
    users = generate_shard(3000, Comm(), "cpu", 8.0, 3.0, 60, 80, seed=seed, users=True)
    ref = AssociationRules(res).recommend_shard(users)
    assert torch.equal(dev.recommend_shard(users.to(DEV)).cpu(), ref)
    # indexed (per-item rule lists) and plain ordered scans agree
    import fastapriori_amd.ops.primitives as prim
    ud = users.to(DEV)
    old_min = prim.RECOMMEND_INDEX_MIN_RULES
    try:
        prim.RECOMMEND_INDEX_MIN_RULES = 1
        dev.use_index = True
        a = dev.recommend_shard(ud).cpu()
        dev.use_index = False
        b = dev.recommend_shard(ud).cpu()
    finally:
        prim.RECOMMEND_INDEX_MIN_RULES = old_min
    assert torch.equal(a, ref) and torch.equal(b, ref)
    assert (ref >= 0).any() and (ref < 0).any()


def test_gen_chain_matches_iterated_gen():
    # fa_hip_ag_chain == apriori_gen applied level after level (no growth / capacity stop)
    sh = generate_shard(20000, Comm(), "cpu", 10.0, 4.0, 60, 80, seed=5)
    res = FastApriori(0.004, config=MinerConfig(min_support=0.004)).run(sh)
    prev = res.levels[2]
    pi, eo, ex = apriori_gen(prev)
    g = np.repeat(np.arange(pi.size), np.diff(eo))
    cand = np.ascontiguousarray(np.concatenate([prev[pi[g]], ex[:, None]], axis=1), dtype=np.int32)
    F1 = len(res.items)
    # speculative chains from candidates can grow fast: cap the depth at 4 levels
    got = ops.primitives.apriori_gen_chain(cand, F1, DEV, 4, 1e9, 0, 1 << 40)
    assert len(got) >= 2
    cur = cand
    for gpi, geo, gex, grows in got:
        pi, eo, ex = apriori_gen(cur)
        assert np.array_equal(gpi, pi) and np.array_equal(geo, eo) and np.array_equal(gex, ex)
        g = np.repeat(np.arange(pi.size), np.diff(eo))
        cur = np.ascontiguousarray(np.concatenate([cur[pi[g]], ex[:, None]], axis=1), dtype=np.int32)
        assert np.array_equal(grows, cur)
    assert len(got) == 4 or apriori_gen(cur)[2].size == 0
    # depth / capacity / growth stops
    two = ops.primitives.apriori_gen_chain(cand, F1, DEV, 2, 1e9, 0, 1 << 40)
    assert len(two) == min(2, len(got))
    cap = ops.primitives.apriori_gen_chain(cand, F1, DEV, 4, 1e9, 0, got[0][2].size)
    assert len(cap) == 1
    # first_free: level k itself from F_{k-1} in the same call, limit from its used items
    ff = ops.primitives.apriori_gen_chain(prev, F1, DEV, 4, 1e9, 0, 0, first_free=True)
    pi, eo, ex = apriori_gen(prev)
    assert np.array_equal(ff[0][0], pi) and np.array_equal(ff[0][1], eo) and np.array_equal(ff[0][2], ex)
    assert np.array_equal(ff[0][3], cand)
    for a, b in zip(ff[1:], got):
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
    used = np.unique(cand)
    lim = ops.primitives.slab_total_limit(used.size)
    assert sum(l[2].size for l in ff) <= max(lim, ff[0][2].size)
    c0 = got[0][2].size      # growth is measured against the previous level (the input for level 0)
    assert len(ops.primitives.apriori_gen_chain(cand, F1, DEV, 4, (c0 - 0.5) / cand.shape[0], 0, 1 << 40)) == 0


def test_bundling_chain_matches_python_loop(tune):
    import fastapriori_amd.models.apriori as ap
    sh = generate_shard(200000, Comm(), "cpu", 10.0, 4.0, 60, 80, seed=8).to(DEV)
    cfg = MinerConfig(min_support=0.003)
    a = FastApriori(0.003, config=cfg).run(sh)
    tune(gen_chain=False)
    b = FastApriori(0.003, config=MinerConfig(min_support=0.003)).run(sh)
    assert a.as_dict() == b.as_dict()


def test_parse_to_device_roundtrip():
    sh = parse_bytes(b"1 2 3\n\n4 4 5\n", device=DEV)
    assert sh.items.is_cuda and sh.n_lines == 3


def test_slab_multipass_from_bitmap(tune):
    # shrink the LDS budget so the accumulator needs several passes -> bitmap-tile path
    import fastapriori_amd.ops.primitives as prim
    sh = generate_shard(30000, Comm(), "cpu", 12.0, 5.0, 200, 100, seed=13)
    cfg = dict(min_support=0.005, dedup="off")
    ref = FastApriori(0.005, config=MinerConfig(trim_min_rows=0, level_kernel="bitmap", **cfg)).run(sh)
    tune(slab_lds_bytes=24 * 1024)
    got = FastApriori(0.005, config=MinerConfig(trim_min_rows=0, level_kernel="slab", **cfg)).run(sh.to(DEV))
    assert ref.as_dict() == got.as_dict()
    got_w = FastApriori(0.005, config=MinerConfig(trim_min_rows=0, level_kernel="slab", min_support=0.005, dedup="on")).run(sh.to(DEV))
    assert ref.as_dict() == got_w.as_dict()


@pytest.mark.parametrize("lds_kb,dense", [(160, 0), (24, 0), (24, 1e-9)])
def test_slab_class_layout_on_gpu(tune, lds_kb, dense):
    # every slab pass in the class layout (plan.cpp cls_layout, slab_cls=2), so
    # k_count_slab_rec<.., kCls> runs single-pass (contiguous build) and multi-pass
    # (bitmap copy) levels; counts must equal the bitmap kernel's
    import fastapriori_amd.ops.primitives as prim
    sh = generate_shard(60000, Comm(), "cpu", 14.0, 6.0, 300, 120, seed=11)
    cfg = dict(min_support=0.004, dedup="off")
    ref = FastApriori(0.004, config=MinerConfig(trim_min_rows=0, level_kernel="bitmap", **cfg)).run(sh)
    import fastapriori_amd.models.apriori as ap
    tune(device_levels=False)    # the host plans (device plans: test_gpu_device_levels)
    tune(slab_cls=2)
    tune(slab_lds_bytes=lds_kb * 1024 - 512)
    if dense:   # every level "dense": the slab kernel runs without its all-zero-prefix test
        tune(dense_min_rows=dense)
    n0 = prim.CLS_LEVELS[0]
    got = FastApriori(0.004, config=MinerConfig(trim_min_rows=0, level_kernel="slab", **cfg)).run(sh.to(DEV))
    assert len(ref.levels) >= 5
    assert prim.CLS_LEVELS[0] > n0
    assert ref.as_dict() == got.as_dict()


@pytest.mark.parametrize("long_rows", [False, True])
def test_pair_kernels_agree(long_rows):
    # unit weights: 256-rank blocks + k_pair_queue16 (long_rows: 128-rank blocks +
    # k_pair_blocked); row weights: k_pair_blocked
    off, items, lut, F1 = _prep(n=20000, V=900, seed=21, long_rows=30, F1_frac=0.9)
    _, kept, roff = _compress_inputs(off, items, lut)
    ranks = ops.compress(off, items, lut, kept, roff)
    ref = ops.pair_counts_horizontal(roff, ranks, None, F1)
    got = ops.pair_counts_horizontal(roff.to(DEV), ranks.to(DEV), None, F1, long_rows).cpu()
    assert torch.equal(ref, got)
    w = torch.randint(0, 4, (kept.numel(),), dtype=torch.int32)
    refw = ops.pair_counts_horizontal(roff, ranks, w, F1)
    gotw = ops.pair_counts_horizontal(roff.to(DEV), ranks.to(DEV), w.to(DEV), F1).cpu()
    assert torch.equal(refw, gotw)


@pytest.mark.parametrize("F1,n_wg", [(600, 0), (601, 3), (257, 1)])
def test_pair_queue_drain_and_stealing(tune, F1, n_wg):
    """k_pair_queue16 over many sub-chunks: pair counts far above 2^16 (the u16 LDS
    counters drain bit 15 into the global count), odd F1 (u32 flush path), and few
    workgroups for many tiles (tile switches and stealing)."""
    tune(pair_wg=n_wg)
    rng = np.random.default_rng(F1)
    n = 150_000
    lens = rng.integers(2, 9, n)
    roff = np.zeros(n + 1, np.int64)
    roff[1:] = np.cumsum(lens)
    rows = []
    for L in lens:
        # ranks 0 and 1 in ~90 % of rows (counts ~135K: drained several times)
        head = [r for r in (0, 1) if rng.random() < 0.9]
        rest = rng.choice(np.arange(2, F1), size=max(int(L) - len(head), 0), replace=False)
        rows.append(np.sort(np.concatenate([np.array(head, np.int64), rest]).astype(np.int32)))
    lens = np.array([r.size for r in rows])
    roff[1:] = np.cumsum(lens)
    ranks = torch.from_numpy(np.concatenate(rows))
    roff = torch.from_numpy(roff)
    ref = ops.pair_counts_horizontal(roff, ranks, None, F1)
    got = ops.pair_counts_horizontal(roff.to(DEV), ranks.to(DEV), None, F1, False).cpu()
    assert int(ref[0, 1]) > 100_000
    assert torch.equal(ref, got)


@pytest.mark.parametrize("offset", [0, 1])
def test_f1_sketch_and_exact(offset):
    rng = np.random.default_rng(7)
    ids = (rng.zipf(1.3, 2_000_003) % 3_000_000).astype(np.int32)
    items = torch.from_numpy(ids)[offset:]
    sk_cpu = ops.f1_sketch(items)
    sk_gpu = ops.f1_sketch(items.to(DEV)).cpu()
    assert torch.equal(sk_cpu, sk_gpu)
    cand = torch.from_numpy(np.unique(ids[:5000])[:3000].astype(np.int64))
    assert torch.equal(ops.f1_exact(items, cand), ops.f1_exact(items.to(DEV), cand.to(DEV)).cpu())


def test_wide_vocab_miner_matches_cpu():
    from fastapriori_amd.utils.io import generate_zipf_shard
    sh = generate_zipf_shard(20000, Comm(), "cpu", mean_len=80.0, n_items=3_000_000, n_topics=100)
    cfg = MinerConfig(min_support=0.02)
    ref = FastApriori(0.02, config=MinerConfig(min_support=0.02, f1="histogram")).run(sh)
    got = FastApriori(0.02, config=cfg).run(sh.to(DEV))
    assert got.items == ref.items and got.as_dict() == ref.as_dict() and ref.n_itemsets > 100


@pytest.mark.parametrize("weighted", [False, True])
def test_trim_rows_matches_cpu(weighted):
    off, items, lut, F1 = _prep(n=5000, V=300, max_len=40, seed=11, long_rows=20)
    cnt, kept, roff = _compress_inputs(off, items, lut)
    ranks = ops.compress(off, items, lut, kept, roff)
    rng = np.random.default_rng(3)
    alive = torch.from_numpy((rng.random(F1) < 0.6).astype(np.int8))
    wrow = torch.from_numpy(rng.integers(0, 3, kept.numel()).astype(np.int32)) if weighted else None
    ref = ops.trim_rows(roff, ranks, alive, 3, wrow)
    got = ops.trim_rows(roff.to(DEV), ranks.to(DEV), alive.to(DEV), 3, wrow.to(DEV) if weighted else None)
    for a, b in zip(ref, got):
        if a is None:
            assert b is None
        else:
            assert torch.equal(a, b.cpu())


@pytest.mark.parametrize("lds_kb", [0, 24, 12])
def test_slab_kernel_budgets_and_weights(tune, lds_kb):
    # single- and multi-pass slab plans (smaller LDS budgets: narrower slabs, more
    # passes from the bitmap tiles), unit and dedup weights: whole-miner results must
    # equal the CPU reference through the deep levels
    import fastapriori_amd.ops.primitives as prim
    sh = generate_shard(30000, Comm(), "cpu", 14.0, 6.0, 200, 120, seed=17)
    cfg = dict(min_support=0.004)
    ref = FastApriori(0.004, config=MinerConfig(trim_min_rows=0, level_kernel="bitmap", dedup="off", **cfg)).run(sh)
    assert len(ref.levels) >= 5
    if lds_kb:
        tune(slab_lds_bytes=lds_kb * 1024)
    for dd in ("off", "on"):
        got = FastApriori(0.004, config=MinerConfig(trim_min_rows=0, level_kernel="slab", dedup=dd, **cfg)).run(
            sh.to(DEV))
        assert ref.as_dict() == got.as_dict(), (lds_kb, dd)


def test_bundled_levels_on_gpu(tune):
    # several levels of different k counted in one slab launch (per-piece prefix lengths)
    from fastapriori_amd.models import apriori as ap
    sh = generate_shard(40000, Comm(), "cpu", 10.0, 4.0, 200, 100, seed=23)
    ref = FastApriori(0.003, config=MinerConfig(min_support=0.003, level_kernel="bitmap")).run(sh)
    got = FastApriori(0.003, config=MinerConfig(min_support=0.003)).run(sh.to(DEV))
    assert ref.as_dict() == got.as_dict() and len(ref.levels) >= 5
    tune(bundle_levels=False)
    got2 = FastApriori(0.003, config=MinerConfig(min_support=0.003)).run(sh.to(DEV))
    assert ref.as_dict() == got2.as_dict()


@pytest.mark.parametrize("n,max_len,long_rows", [(5000, 25, 5), (70000, 14, 40), (3000, 60, 300)])
def test_compress_rows_fused(n, max_len, long_rows):
    # two-pass fused compression (kept rows, offsets, sorted ranks, length histogram) vs the CPU path;
    # long rows go through the overflow tiers, wide spans through the unstaged path
    off, items, lut, F1 = _prep(n=n, V=700, max_len=max_len, seed=n, long_rows=long_rows)
    cnt, kept, roff = _compress_inputs(off, items, lut)
    ref = ops.compress(off, items, lut, kept, roff)
    gk, groff, granks, ghist, bcnt = ops.compress_rows(off.to(DEV), items.to(DEV), lut.to(DEV), F1)
    assert torch.equal(kept, gk.cpu()) and torch.equal(roff, groff.cpu()) and torch.equal(ref, granks.cpu())
    h = torch.bincount(torch.clamp(cnt[cnt >= 2], max=255).long(), minlength=256)
    assert torch.equal(h, torch.as_tensor(ghist))
    # 256-rank block counts written by the emit pass (+ the overflow-row fixup) vs the ranks
    T, nb = gk.numel(), (F1 + 255) // 256
    r = ref.long()
    row = torch.repeat_interleave(torch.arange(T), (roff[1:] - roff[:-1]).long())
    want = torch.zeros(nb, T, dtype=torch.long)
    want.index_put_((r >> 8, row), torch.ones_like(r), accumulate=True)
    got = bcnt.cnt.cpu()[:nb * T].view(nb, T).long()
    assert torch.equal(got, want.clamp(max=255))


def _dmix64(z):
    # prep.hip dmix64 on uint64 arrays (wrapping arithmetic)
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


@pytest.mark.parametrize("n,dups", [(60000, 0), (300000, 40)])
def test_dedup_probe_counts(n, dups):
    # the dedup estimate's probe (prep.hip k_dedup_probe + k_probe_count): hashed rows and
    # occupied slots of the first min(T, 2^18) kept rows vs the same hash in numpy; dups > 0
    # repeats a few row patterns (occupied slots < hashed rows)
    import fastapriori_amd.ops.primitives as prim
    off, items, lut, F1 = _prep(n=n, V=300, max_len=16, seed=n + dups, long_rows=0, F1_frac=0.9)
    if dups:
        o, it = off.numpy(), items.numpy()
        pat = [it[o[i]:o[i + 1]] for i in range(dups)]
        rows = [pat[i % dups] if i % 3 == 0 else it[o[i]:o[i + 1]] for i in range(n)]
        off = torch.zeros(n + 1, dtype=torch.int64)
        off[1:] = torch.from_numpy(np.cumsum([r.size for r in rows]))
        items = torch.from_numpy(np.concatenate(rows).astype(np.int32))
    probe = {}
    kept, roff, ranks, _, _ = ops.compress_rows(off.to(DEV), items.to(DEV), lut.to(DEV), F1, probe=probe)
    nmax = min(kept.numel(), prim.DEDUP_PROBE_ROWS)
    ro, rk = roff.cpu().numpy(), ranks.cpu().numpy().astype(np.uint64)
    lens = ro[1:nmax + 1] - ro[:nmax]
    sel = np.flatnonzero(lens <= 16)
    a = np.full(sel.size, 0x243F6A8885A308D3, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in range(16):
            live = lens[sel] > j
            idx = np.where(live, ro[sel] + j, 0)
            a = np.where(live, _dmix64(a ^ rk[idx]), a)
        a = _dmix64(a ^ lens[sel].astype(np.uint64))
    slots = (a >> np.uint64(1)) & np.uint64((1 << 22) - 1)
    assert probe["n"] == sel.size
    assert probe["filled"] == np.unique(slots).size
    if dups:
        assert probe["filled"] < probe["n"]


@pytest.mark.parametrize("long_rows", [0, 12])
def test_pair_counts_with_compress_block_counts(long_rows):
    # the pair layout built from the emit pass's block counts == the counting pass
    off, items, lut, F1 = _prep(n=90000, V=900, max_len=22, seed=5, long_rows=long_rows)
    kept, roff, ranks, _, bcnt = ops.compress_rows(off.to(DEV), items.to(DEV), lut.to(DEV), F1)
    assert bcnt is not None and bcnt.lr is not None      # the emit pass wrote the whole layout
    a = ops.pair_counts_horizontal(roff, ranks, None, F1, long_rows=False, bcnt=bcnt)
    a2 = ops.pair_counts_horizontal(roff, ranks, None, F1, long_rows=False, bcnt=bcnt.cnt)   # + scatter pass
    b = ops.pair_counts_horizontal(roff, ranks, None, F1, long_rows=False)
    assert torch.equal(a.cpu(), b.cpu()) and torch.equal(a2.cpu(), b.cpu()) and int(a.sum()) > 0
    # the fused local ranks and batch bases == the block-scatter pass's
    import fastapriori_amd.ops.primitives as prim
    T, nb = roff.numel() - 1, (F1 + 255) // 256
    nbatch, nnz = (T + 63) // 64, int(ranks.numel())
    bsum = torch.empty(nb * nbatch, dtype=torch.int64, device=DEV)
    cnt = bcnt.cnt
    prim._hip_call("fa_hip_block_bsum", prim._p(cnt), T, T, nb, prim._p(bsum), prim._stream(ranks))
    base = torch.cumsum(bsum, 0) - bsum
    lr = torch.zeros(nnz + 1024, dtype=torch.uint8, device=DEV)
    prim._hip_call("fa_hip_block_scatter", prim._p(roff), prim._p(ranks), T, F1, prim._p(cnt), prim._p(base), prim._p(lr),
                  256, prim._stream(ranks))
    assert torch.equal(bcnt.base[:nb * nbatch].cpu(), base.cpu())
    assert torch.equal(bcnt.lr[:nnz].cpu(), lr[:nnz].cpu())


@pytest.mark.parametrize("k", [3, 4, 6])
def test_apriori_gen_device_matches_host(k):
    # GPU bitset apriori-gen == host apriori-gen on real levels (and speculative candidate levels)
    sh = generate_shard(30000, Comm(), "cpu", 12.0, 5.0, 150, 300, seed=29)
    res = FastApriori(0.003, config=MinerConfig(min_support=0.003)).run(sh)
    assert len(res.levels) >= k
    prev = res.levels[k - 2]
    want = apriori_gen(prev)
    got = ops.apriori_gen_device(prev, len(res.items), DEV)
    for a, b in zip(want, got):
        assert np.array_equal(a, b)
    pidx, eoff, ext = want
    g = np.repeat(np.arange(pidx.size), np.diff(eoff))
    cand = np.ascontiguousarray(np.concatenate([prev[pidx[g]], ext[:, None]], 1), np.int32)
    got = ops.apriori_gen_device(cand, len(res.items), DEV, want_rows=True)
    want = apriori_gen(cand)
    for a, b in zip(want, got[:3]):
        assert np.array_equal(a, b)
    g2 = np.repeat(np.arange(want[0].size), np.diff(want[1]))
    assert np.array_equal(got[3], np.concatenate([cand[want[0][g2]], want[2][:, None]], 1))


@pytest.mark.parametrize("blocked", [False, True])
@pytest.mark.parametrize("fp4", [False, True])
@pytest.mark.parametrize("F1,T", [(37, 5000), (300, 70001), (1000, 9000)])
def test_pair_gram_mfma_matches_popcount(F1, T, fp4, blocked):
    # i8 MFMA Gram (v_mfma_i32_32x32x32_i8, the test oracle), and its FP4 form (the
    # product path: v_mfma_scale_f32_32x32x64_f8f6f4 on e2m1 0/1 operands), vs the popcount
    # Gram and a numpy Gram on asymmetric random bitmaps (F1 not a multiple of the 128
    # tile, W of the 8-word step)
    rng = np.random.default_rng(F1)
    dens = rng.random(F1) * 0.6
    bits = rng.random((F1, T)) < dens[:, None]
    W = (T + 63) // 64
    Wp = (W + 63) // 64 * 64
    words = np.zeros((F1, Wp), dtype=np.uint64)
    packed = np.packbits(bits, axis=1, bitorder="little")
    pad = np.zeros((F1, W * 8), np.uint8)
    pad[:, :packed.shape[1]] = packed
    words[:, :W] = pad.view(np.uint64)
    bm = torch.from_numpy(words.view(np.int64)).to(DEV)
    if blocked:   # the 8-word block layout (count.hip BmView)
        bm = ops.primitives.to_blocked(bm)
    got = ops.pair_counts_gram(bm, W, None, fp4=fp4).cpu()
    ref = ops.pair_counts_gram(bm, W, None, force_popc=True).cpu()
    want = torch.from_numpy(bits.astype(np.int64) @ bits.astype(np.int64).T)
    iu = torch.triu_indices(F1, F1, 1)
    assert torch.equal(got[iu[0], iu[1]], want[iu[0], iu[1]])
    assert torch.equal(ref[iu[0], iu[1]], want[iu[0], iu[1]])


@pytest.mark.parametrize("blocked", [False, True])
@pytest.mark.parametrize("fp4", [False, True])
@pytest.mark.parametrize("F1,classes", [(300, [(1, 700), (2, 40), (3, 600), (7, 3), (9, 520)]),
                                        (37, [(1, 9), (4, 530)])])
def test_weighted_gram_mfma_matches_popcount(F1, classes, fp4, blocked):
    # deduplicated layouts: one scaled matrix-core launch per weight class of >= 512
    # words, the short classes by the popcount Gram -- exact against the weighted
    # popcount Gram and a numpy reference (FastApriori.scala:233-235)
    rng = np.random.default_rng(F1 + len(classes))
    W = sum(n for _, n in classes)
    Wp = (W + 63) // 64 * 64
    words = rng.integers(0, 1 << 63, size=(F1, Wp), dtype=np.int64) & rng.integers(0, 1 << 63, size=(F1, Wp),
                                                                                     dtype=np.int64)
    words[:, W:] = 0
    wword = np.concatenate([np.full(n, wt, np.int32) for wt, n in classes])
    wcls = (np.array([wt for wt, _ in classes], np.int64), np.array([n for _, n in classes], np.int64))
    segs = ops.primitives.gram_segments(W, True, wcls)
    assert any(w > 1 for _, _, w in segs) and any(w == 0 for _, _, w in segs)
    bm = torch.from_numpy(words).to(DEV)
    if blocked:   # classes start off the 8-word blocks (700, 740, ...): the view's woff
        bm = ops.primitives.to_blocked(bm)
    ww = torch.from_numpy(wword).to(DEV)
    got = ops.pair_counts_gram(bm, W, ww, wcls, fp4=fp4).cpu()
    ref = ops.pair_counts_gram(bm, W, ww, wcls, force_popc=True).cpu()
    bits = np.unpackbits(words[:, :W].view(np.uint8), axis=1, bitorder="little").astype(np.int64)
    wcol = np.repeat(wword.astype(np.int64), 64)
    want = torch.from_numpy((bits * wcol) @ bits.T)
    iu = torch.triu_indices(F1, F1, 1)
    assert torch.equal(got[iu[0], iu[1]], want[iu[0], iu[1]])
    assert torch.equal(ref[iu[0], iu[1]], want[iu[0], iu[1]])


def _unpack_rows(words: np.ndarray, ncols: int) -> np.ndarray:
    """uint64 words [n, W] -> bool [n, ncols] (column c = bit c & 63 of word c >> 6)."""
    b = np.unpackbits(words.astype(np.uint64).view(np.uint8).reshape(words.shape[0], -1), axis=1, bitorder="little")
    return b[:, :ncols].astype(bool)


@pytest.mark.parametrize("out_blocked", [False, True])
@pytest.mark.parametrize("blocked", [False, True])
@pytest.mark.parametrize("ncols,n_items,k,dens", [(64 * 37 + 5, 9, 3, 0.3), (64 * 300, 70, 9, 0.12),
                                                  (64 * 5 + 63, 3, 2, 0.5), (64 * 80, 40, 39, 0.9),
                                                  (1000, 12, 13, 0.5)])
def test_window_bitmap_matches_numpy(blocked, out_blocked, ncols, n_items, k, dens):
    """count.hip k_win_alive / k_win_compact (ops.primitives.window_bitmap) against numpy:
    the rows holding >= k of the window's items, each item's bits compressed to them
    (window rows gathered from a larger bitmap, in either layout; edge words, K = 0)."""
    rng = np.random.default_rng(ncols + n_items + k)
    F = n_items + 17
    bits = rng.random((F, ncols)) < dens
    W = (ncols + 63) // 64
    Wp = -(-W // 64) * 64
    words = np.zeros((F, Wp * 64), dtype=np.uint8)
    words[:, :ncols] = bits
    wrd = np.packbits(words, axis=1, bitorder="little").view(np.uint64)          # [F, Wp]
    if blocked:
        bm = torch.from_numpy(np.ascontiguousarray(wrd.reshape(F, Wp // 8, 8).transpose(1, 0, 2)).view(np.int64)).to(DEV)
    else:
        bm = torch.from_numpy(wrd.view(np.int64)).to(DEV)
    rows = np.sort(rng.choice(F, n_items, replace=False)).astype(np.int32)
    got = ops.primitives.window_bitmap(bm, torch.from_numpy(rows).to(DEV), W, k, blocked=out_blocked)
    alive = bits[rows].sum(0) >= k
    K = int(alive.sum())
    assert got[0] == K
    if K == 0:
        assert got[1] is None
        return
    out = got[1].cpu().numpy().view(np.uint64)
    if out_blocked:                                                # [Wp / 8, n, 8] -> [n, Wp]
        out = np.ascontiguousarray(out.transpose(1, 0, 2)).reshape(n_items, -1)
    assert out.shape[0] == n_items and out.shape[1] * 64 >= K
    want = bits[rows][:, alive]
    assert np.array_equal(_unpack_rows(out, K), want)
    assert not _unpack_rows(out, out.shape[1] * 64)[:, K:].any()       # zero past the K rows
    assert ops.primitives.window_bitmap(bm, torch.from_numpy(rows).to(DEV), W, k, max_keep=K - 1) is None


def test_lane_deal_cross_row_sum():
    """levels.hip la_qsum (v_permlane16_swap / v_permlane32_swap): every lane of a wave gets
    the sum over lanes l, l ^ 16, l ^ 32, l ^ 48 -- the lane deal's four 16-lane rows must
    agree on every record's cost, or they would deal it to different groups."""
    out = torch.zeros(64, dtype=torch.int32, device=DEV)
    _native.check(_native.hip().fa_hip_debug_la_qsum(out.data_ptr(), torch.cuda.current_stream().cuda_stream),
                  "fa_hip_debug_la_qsum")
    lane = np.arange(64)
    assert np.array_equal(out.cpu().numpy(), 4 * (lane & 15) + 0 + 16 + 32 + 48)
