"""Rules, redundancy cut, ordering and recommendation vs the oracle (AssociationRules.scala)."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from fastapriori_amd.models.apriori import FastApriori, MinerConfig
from fastapriori_amd.models.oracle import OracleResult, gen_rules, recommend, sort_rules
from fastapriori_amd.models.oracle import mine as oracle_mine
from fastapriori_amd.models.rules import AssociationRules
from fastapriori_amd.utils.io import parse_bytes
from fastapriori_amd.utils.jvm import java_split_ws, rule_tiebreak_key
from fastapriori_amd.utils.metrics import Logger

row = st.lists(st.sampled_from([str(i) for i in range(1, 10)]), min_size=0, max_size=7)


def _text(rows):
    return "\n".join(" ".join(r) for r in rows) + "\n"


def _oracle_from(res) -> OracleResult:
    """Oracle object over the miner's own rank space (so rules compare rank-for-rank)."""
    return OracleResult(items=res.items, counts1=res.counts[0].tolist(), itemsets=res.as_dict(),
                        min_count=res.min_count, n_lines=res.n_lines)


@settings(max_examples=60, deadline=None)
@given(st.lists(row, min_size=1, max_size=50), st.lists(row, min_size=0, max_size=20),
       st.sampled_from([0.05, 0.1, 0.2]))
def test_rules_and_recommendations_match_oracle(drows, urows, ms):
    res = FastApriori(ms, config=MinerConfig(min_support=ms), logger=Logger(enabled=False)).run(
        parse_bytes(_text(drows).encode()))
    ar = AssociationRules(res, logger=Logger(enabled=False))
    orc = _oracle_from(res)
    exp = sort_rules(gen_rules(orc), res.items)
    got = ar.rule_list()
    assert [(frozenset(a), c) for a, c, _ in got] == [(a, c) for a, c, _ in exp]
    assert [conf for _, _, conf in got] == [conf for _, _, conf in exp]     # bit-identical doubles
    utext = _text(urows) if urows else ""
    users = parse_bytes(utext.encode())
    assert ar.run(users) == recommend(orc, [java_split_ws(l) for l in utext.splitlines()])


def test_no_rules_gives_all_zero():
    # the reference throws on rules.keys.min here (AssociationRules.scala:147); we answer "0"
    res = FastApriori(0.5).run(parse_bytes(b"1\n1\n2\n"))
    ar = AssociationRules(res)
    assert ar.rules().n_rules == 0
    assert ar.run(parse_bytes(b"1\n2\n\n3 4\n")) == ["0", "0", "0", "0"]


def test_cut_semantics_strict_less():
    # {2}->1 and {4}->1 have conf 4/6 and 4/5; {2,4}->1 has conf 2/4=0.5: cut (not strictly larger)
    d = b"1 2 3\n1 2 4\n2 3 4\n1 2 4\n2 4\n4 5\n1 2\n"
    res = FastApriori(0.25, config=MinerConfig(min_support=0.25)).run(parse_bytes(d))
    rt = AssociationRules(res).rules()
    assert rt.level_stats[1] == (2, 3, 0)
    sizes = np.diff(rt.ante_off)
    assert (sizes == 1).all()


def test_tiebreak_order():
    toks = ["10", "9", "a", "-3", "09", "b", "+7"]
    got = sorted(toks, key=rule_tiebreak_key)
    assert got == ["-3", "+7", "09", "9", "10", "a", "b"]


def test_rule_confidence_is_ieee_double():
    res = FastApriori(0.01).run(parse_bytes(("\n".join(["1 2 3"] * 3 + ["1 2"] * 4 + ["1"] * 2) + "\n").encode()))
    ar = AssociationRules(res)
    for ante, cons, conf in ar.rule_list():
        s = frozenset(ante) | {cons}
        d = res.as_dict()
        assert conf == d[s] / d[frozenset(ante)]


def test_duplicate_baskets_recommended_once():
    # removeRedundancy (AssociationRules.scala:51-58): identical baskets, in any token
    # order and with repeats, are one distinct basket; results fan out to every line
    rng = np.random.default_rng(5)
    drows = [" ".join(map(str, rng.choice(12, size=rng.integers(1, 6), replace=False))) for _ in range(400)]
    res = FastApriori(0.05, config=MinerConfig(min_support=0.05),
                      logger=Logger(enabled=False)).run(parse_bytes(("\n".join(drows) + "\n").encode()))
    pool = [[1, 2], [3], [2, 4, 5], [], [7, 1], [11, 10, 3]]
    urows = []
    for _ in range(300):
        b = list(pool[rng.integers(len(pool))])
        rng.shuffle(b)
        urows.append(" ".join(map(str, b + b[:1])))      # shuffled, with a repeated token
    users = parse_bytes(("\n".join(urows) + "\n").encode())
    on = AssociationRules(res, logger=Logger(enabled=False))
    got = on.run(users)
    off = AssociationRules(res, logger=Logger(enabled=False))
    off.dedup_baskets = False
    assert got == off.run(users)
    assert on.stats["distinct_baskets"] <= len(pool) < off.stats["distinct_baskets"] == 300
    assert got == recommend(_oracle_from(res), [java_split_ws(r) for r in urows])
