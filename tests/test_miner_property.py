"""Property tests: the native/torch miner == the brute-force oracle on random DBs.

Every configuration knob that changes the computation but must not change the
result is swept: k=2 kernel (horizontal / Gram), dedup (on / off), trimming,
level kernel.  Random DBs include duplicate tokens, blank lines, count ties and
rows long enough to exercise the long-row paths.
"""
import itertools

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from fastapriori_amd.models.apriori import FastApriori, MinerConfig
from fastapriori_amd.models.oracle import mine as oracle_mine
from fastapriori_amd.ops.host import apriori_gen
from fastapriori_amd.utils.io import parse_bytes
from fastapriori_amd.utils.jvm import java_split_ws
from fastapriori_amd.utils.metrics import Logger


def _db_text(rows):
    return "\n".join(" ".join(r) for r in rows) + "\n"


def token_sets(res_items, itemsets):
    return {frozenset(res_items[r] for r in s): c for s, c in itemsets.items()}


row = st.lists(st.sampled_from([str(i) for i in range(1, 13)] + ["x", "y"]), min_size=0, max_size=9)


@settings(max_examples=60, deadline=None)
@given(st.lists(row, min_size=1, max_size=60), st.sampled_from([0.05, 0.1, 0.2, 0.34]),
       st.sampled_from(["horizontal", "gram"]), st.sampled_from(["on", "off"]), st.booleans())
def test_miner_matches_oracle(rows, ms, strategy, dedup, trim):
    text = _db_text(rows)
    lines = text.splitlines()
    exp = oracle_mine([java_split_ws(l) for l in lines], ms)
    res = FastApriori(ms, config=MinerConfig(min_support=ms, pair_strategy=strategy, dedup=dedup, trim=trim, trim_min_rows=0),
                      logger=Logger(enabled=False)).run(parse_bytes(text.encode()))
    assert res.min_count == exp.min_count
    assert res.items == exp.items                      # same rank order (count desc, Java string asc)
    assert token_sets(res.items, res.as_dict()) == token_sets(exp.items, exp.itemsets)


def test_deep_levels_long_rows():
    rng = np.random.default_rng(3)
    base = [str(i) for i in range(30)]
    rows = []
    for _ in range(300):
        k = rng.integers(5, 14)
        rows.append(list(rng.choice(base[:16], size=k, replace=False)))
    text = _db_text(rows)
    exp = oracle_mine([java_split_ws(l) for l in text.splitlines()], 0.05)
    for strat in ("horizontal", "gram"):
        res = FastApriori(0.05, config=MinerConfig(trim_min_rows=0, min_support=0.05, pair_strategy=strat),
                          logger=Logger(enabled=False)).run(parse_bytes(text.encode()))
        assert token_sets(res.items, res.as_dict()) == token_sets(exp.items, exp.itemsets)
        assert len(res.levels) >= 5


def brute_candidates(prev: np.ndarray):
    k = prev.shape[1] + 1
    fs = {tuple(r) for r in prev.tolist()}
    items = sorted({x for r in fs for x in r})
    out = set()
    for c in itertools.combinations(items, k):
        if all(tuple(c[:i] + c[i + 1:]) in fs for i in range(k)):
            out.add(c)
    return out


@settings(max_examples=80, deadline=None)
@given(st.integers(2, 4), st.lists(st.lists(st.integers(0, 9), min_size=4, max_size=4, unique=True),
                                  min_size=1, max_size=40))
def test_apriori_gen_matches_bruteforce(m, seeds):
    prev = sorted({tuple(sorted(s[:m])) for s in seeds})
    prev = np.array(prev, dtype=np.int32).reshape(-1, m)
    pidx, eoff, ext = apriori_gen(prev)
    got = set()
    for g in range(pidx.size):
        for e in ext[eoff[g]:eoff[g + 1]]:
            got.add(tuple(prev[pidx[g]].tolist()) + (int(e),))
    assert got == brute_candidates(prev)
    # candidates are produced in lexicographic order (F_k stays sorted after filtering)
    flat = [tuple(prev[pidx[g]].tolist()) + (int(e),) for g in range(pidx.size) for e in ext[eoff[g]:eoff[g + 1]]]
    assert flat == sorted(flat)


def test_no_frequent_items_and_single_txn():
    res = FastApriori(0.5).run(parse_bytes(b"1 2\n3 4\n5 6\n"))
    assert res.n_itemsets == 0
    res = FastApriori(1.0).run(parse_bytes(b"7 8 9\n"))
    assert res.n_itemsets == 7        # every subset of the single transaction


def test_occurrence_counts_for_f1():
    # duplicates inside a line count for F1 only (FastApriori.scala:55 vs :69)
    res = FastApriori(0.5, config=MinerConfig(min_support=0.5)).run(parse_bytes(b"1 1 1 2\n3\n3\n"))
    d = token_sets(res.items, res.as_dict())
    assert d[frozenset(["1"])] == 3 and d[frozenset(["3"])] == 2
    assert frozenset(["1", "2"]) not in d              # pair support is 1 < ceil(1.5)=2


def test_min_count_rounding():
    from fastapriori_amd.utils.jvm import min_count
    assert min_count(0.092, 100) == 10                 # ceil(9.2)
    assert min_count(0.07, 100) == 8                   # 0.07*100 = 7.000000000000001 in IEEE double
    assert min_count(0.25, 7) == 2
    assert min_count(0.0, 5) == 0


@pytest.mark.parametrize("data", [b"1 1 1 2\n3\n3\n", b"5 5 6\n5 6 7\n5 6\n\n6 6 6 6\n"])
def test_heavy_hitter_f1_matches_histogram(data):
    # sketch + exact pass (wide-vocabulary F1) must equal the plain histogram,
    # including duplicate-token "extras" and the empty-line token
    out = []
    for f1 in ("sketch", "histogram"):
        res = FastApriori(0.3, config=MinerConfig(min_support=0.3, f1=f1)).run(parse_bytes(data))
        out.append((res.items, res.as_dict()))
    assert out[0] == out[1]


def test_heavy_hitter_f1_wide_vocab():
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.utils.io import generate_zipf_shard
    sh = generate_zipf_shard(3000, Comm(), "cpu", mean_len=60.0, n_items=2_000_000, n_topics=50)
    a = FastApriori(0.03, config=MinerConfig(min_support=0.03, f1="sketch")).run(sh)
    b = FastApriori(0.03, config=MinerConfig(min_support=0.03, f1="histogram")).run(sh)
    assert a.items == b.items and a.as_dict() == b.as_dict() and a.n_itemsets > 50
