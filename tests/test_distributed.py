"""Count distribution across ranks (gloo, CPU): results must be bit-identical to world size 1.

Exercises everything that crosses ranks: the line total (X3),
the F1 histogram all-reduce (X4), the dictionary-mode hash exchange
(all_to_all + all_gather, X4 arbitrary vocab), pair and level all-reduces
(X12, X15), the identical-decision collectives (dedup / kernel choice), the U.dat
line offsets (X17) and the recommendation gather (X24).
"""
import os

import pytest

from fastapriori_amd.parallel.launch import spawn_local


def _mine_file(path_prefix: str, ms: float, dedup: str, strategy: str, par: str = "count"):
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.models.rules import AssociationRules
    from fastapriori_amd.parallel.comm import init_comm, shutdown_comm
    from fastapriori_amd.utils.io import read_shard
    from fastapriori_amd.utils.metrics import Logger

    comm = init_comm("cpu")
    try:
        from fastapriori_amd.parallel.comm import Comm
        shard = read_shard(path_prefix + "D.dat", comm if par == "count" else Comm())
        cfg = MinerConfig(trim_min_rows=0, min_support=ms, dedup=dedup, pair_strategy=strategy, parallelism=par)
        res = FastApriori(ms, comm, cfg, Logger(comm.rank, enabled=False)).run(shard)
        users = read_shard(path_prefix + "U.dat", comm)
        recs = AssociationRules(res, comm, Logger(comm.rank, enabled=False)).run(users)
        return {"items": res.items, "sets": res.as_dict(), "recs": recs, "rank": comm.rank,
                "lines": shard.n_lines, "base": shard.line_base}
    finally:
        shutdown_comm(comm)


def _mine_zipf(n: int, ms: float, f1: str):
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_zipf_shard
    from fastapriori_amd.utils.metrics import Logger

    comm = init_comm("cpu")
    try:
        shard = generate_zipf_shard(n, comm, "cpu", mean_len=40.0, n_items=1_500_000, n_topics=40, seed=3)
        res = FastApriori(ms, comm, MinerConfig(min_support=ms, f1=f1), Logger(comm.rank, enabled=False)).run(shard)
        return res.as_dict(), res.items
    finally:
        shutdown_comm(comm)


def _mine_candidate(n: int, ms: float, strategy: str, dedup: str):
    """Candidate distribution: every rank generates the WHOLE DB (local Comm)."""
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm, init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger

    comm = init_comm("cpu")
    try:
        shard = generate_shard(n, Comm(), "cpu", 12.0, 4.0, 100, 80, seed=7)
        cfg = MinerConfig(trim_min_rows=0, min_support=ms, parallelism="candidate", pair_strategy=strategy,
                          dedup=dedup)
        res = FastApriori(ms, comm, cfg, Logger(comm.rank, enabled=False)).run(shard)
        return res.as_dict(), res.items
    finally:
        shutdown_comm(comm)


def _mine_generated(n: int, ms: float):
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger

    comm = init_comm("cpu")
    try:
        shard = generate_shard(n, comm, "cpu", 8.0, 3.0, 100, 80, seed=5)
        res = FastApriori(ms, comm, MinerConfig(trim_min_rows=0, min_support=ms), Logger(comm.rank, enabled=False)).run(shard)
        return res.as_dict(), res.items
    finally:
        shutdown_comm(comm)


@pytest.fixture(scope="module")
def numeric_db(tmp_path_factory):
    from fastapriori_amd.utils.io import write_quest_file
    d = tmp_path_factory.mktemp("num")
    write_quest_file(str(d / "D.dat"), 4000, 8.0, 3.0, 60, 50, seed=2)
    write_quest_file(str(d / "U.dat"), 700, 8.0, 3.0, 60, 50, seed=2, users=True)
    return str(d) + "/"


@pytest.fixture(scope="module")
def dict_db(tmp_path_factory):
    import random
    rng = random.Random(4)
    words = [f"w{i}" for i in range(30)] + ["é", "ß", "x y"[0]]
    d = tmp_path_factory.mktemp("dict")
    with open(d / "D.dat", "w", encoding="utf-8") as f:
        for _ in range(1500):
            f.write(" ".join(rng.sample(words, rng.randint(0, 7))) + ("\r\n" if rng.random() < 0.2 else "\n"))
    with open(d / "U.dat", "w", encoding="utf-8") as f:
        for _ in range(300):
            f.write(" ".join(rng.sample(words, rng.randint(0, 3))) + "\n")
    return str(d) + "/"


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("dedup,strategy", [("off", "horizontal"), ("on", "gram")])
def test_numeric_file_matches_single_rank(numeric_db, world, dedup, strategy):
    ref = spawn_local(_mine_file, 1, numeric_db, 0.02, dedup, strategy)[0]
    outs = spawn_local(_mine_file, world, numeric_db, 0.02, dedup, strategy)
    for o in outs:
        assert o["items"] == ref["items"]
        assert o["sets"] == ref["sets"]
    assert outs[0]["recs"] == ref["recs"]
    assert all(o["recs"] is None for o in outs[1:])
    assert sum(o["lines"] for o in outs) == ref["lines"]
    assert [o["base"] for o in outs] == sorted(o["base"] for o in outs)


def test_dictionary_vocab_across_ranks(dict_db):
    ref = spawn_local(_mine_file, 1, dict_db, 0.008, "auto", "auto")[0]
    outs = spawn_local(_mine_file, 3, dict_db, 0.008, "auto", "auto")
    assert outs[0]["items"] == ref["items"] and outs[0]["sets"] == ref["sets"]
    assert outs[0]["recs"] == ref["recs"]
    assert len(ref["sets"]) > 40


def test_generated_shards_are_world_size_invariant():
    ref = spawn_local(_mine_generated, 1, 6000, 0.02)[0]
    for world in (2, 3):
        outs = spawn_local(_mine_generated, world, 6000, 0.02)
        assert all(o == ref for o in outs)


def test_heavy_hitter_f1_across_ranks():
    # sketch all-reduce -> identical candidates on every rank -> exact all-reduce
    ref = spawn_local(_mine_zipf, 1, 3000, 0.03, "histogram")[0]
    outs = spawn_local(_mine_zipf, 2, 3000, 0.03, "sketch")
    assert all(o == ref for o in outs) and len(ref[0]) > 20


@pytest.mark.parametrize("strategy,dedup", [("horizontal", "off"), ("gram", "on")])
def test_candidate_distribution_matches_single_rank(strategy, dedup):
    # replicated DB; pair counts split by rows / bitmap words, level candidates split by rank
    ref = spawn_local(_mine_candidate, 1, 5000, 0.01, strategy, dedup)[0]
    for world in (2, 3):
        outs = spawn_local(_mine_candidate, world, 5000, 0.01, strategy, dedup)
        assert all(o == ref for o in outs)
    assert len(ref[0]) > 200 and max(len(k) for k in ref[0]) >= 4


def test_candidate_distribution_file_and_rules(numeric_db):
    ref = spawn_local(_mine_file, 1, numeric_db, 0.02, "auto", "auto")[0]
    outs = spawn_local(_mine_file, 2, numeric_db, 0.02, "auto", "auto", "candidate")
    assert all(o["sets"] == ref["sets"] and o["items"] == ref["items"] for o in outs)
    assert outs[0]["recs"] == ref["recs"]


def test_forced_process_group_at_world_one(numeric_db):
    # FA_FORCE_PG=1: every collective runs at world size 1 (how a one-GPU box exercises
    # the RCCL paths); results must equal the collective-free run
    ref = spawn_local(_mine_file, 1, numeric_db, 0.02, "auto", "auto")[0]
    got = spawn_local(_mine_file, 1, numeric_db, 0.02, "auto", "auto", env={"FA_FORCE_PG": "1"})[0]
    assert got == ref


def _rs_select(n: int, thr: int):
    import torch
    from fastapriori_amd.parallel.comm import init_comm, shutdown_comm
    comm = init_comm("cpu")
    try:
        g = torch.Generator().manual_seed(11 + comm.rank)
        t = torch.randint(0, 3, (n,), generator=g, dtype=torch.int64)
        idx, val = comm.reduce_scatter_select(t.clone(), thr, bound=1 << 20)
        full = comm.all_reduce_(t.clone())
        return idx.tolist(), val.tolist(), full.tolist()
    finally:
        shutdown_comm(comm)


@pytest.mark.parametrize("thr", [0, 3])
def test_reduce_scatter_select_ignores_padding(thr):
    # 10 entries over 3 ranks: chunks of 4, two zero-padding slots that a threshold of 0
    # (min_support 0) must not select (parallel/comm.py reduce_scatter_select)
    for idx, val, full in spawn_local(_rs_select, 3, 10, thr):
        want = [i for i, v in enumerate(full) if v >= thr]
        assert idx == want and val == [full[i] for i in want]


@pytest.mark.parametrize("dedup,gathers", [("off", 2), ("on", 3)])
def test_layout_metrics_ride_on_the_decision_gather(dedup, gathers):
    # the run's T / distinct metrics come with the compression decisions' all-gather
    # unless a layout was deduplicated (then _finish gathers the distinct rows)
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger
    comm = Comm()
    calls = []
    orig = comm.all_gather_ints
    comm.all_gather_ints = lambda v: calls.append(len(v)) or orig(v)
    sh = generate_shard(3000, comm, "cpu", 10.0, 4.0, 200, 100, 2)
    m = FastApriori(0.02, comm, MinerConfig(min_support=0.02, dedup=dedup), Logger(0, enabled=False))
    m.run(sh)
    assert len(calls) == gathers, calls
    assert m.stats["T"] > 0 and 0 < m.stats["distinct"] <= m.stats["T"]


def _bucketed_sum(n: int):
    import torch
    from fastapriori_amd.parallel.comm import init_comm, shutdown_comm
    from fastapriori_amd.tuning import TUNING
    comm = init_comm("cpu")
    try:
        g = torch.Generator().manual_seed(5 + comm.rank)
        t = torch.randint(0, 1 << 20, (n,), generator=g, dtype=torch.int64)
        one = comm.all_reduce_(t.clone())
        calls0 = comm.comm_calls
        TUNING.bucket_mb = 1000 * 8 / (1 << 20)          # ~1000 int64 per bucket: forces bucketing
        b = comm.bucket_elems(8)
        buck = comm.all_reduce_(t.clone())
        return one.tolist(), buck.tolist(), b, comm.comm_calls - calls0, comm.world_size
    finally:
        shutdown_comm(comm)


def test_bucketed_all_reduce_is_bit_identical():
    # 3 ranks, a 10,007-entry vector in ~1000-element buckets (a multiple of world_size):
    # the same sums as one all-reduce of the whole vector
    for one, buck, b, calls, w in spawn_local(_bucketed_sum, 3, 10_007):
        assert b % w == 0 and b < 10_007
        assert buck == one and calls == 1
