"""Golden tests: the SURVEY §2.7 worked example, end to end, byte for byte.

Expected outputs are hand-traced through the reference semantics
(Main.scala, Utils.scala, FastApriori.scala, AssociationRules.scala) in
SURVEY.md §2.7; the reference itself cannot run here (no JVM/Spark).
"""
import os
import subprocess
import sys

import pytest

from fastapriori_amd.config import JobConfig
from fastapriori_amd.models.apriori import FastApriori, MinerConfig
from fastapriori_amd.models.oracle import run_oracle
from fastapriori_amd.models.rules import AssociationRules
from fastapriori_amd.parallel.comm import Comm
from fastapriori_amd.pipeline import run_job
from fastapriori_amd.utils.io import OutputExistsError, parse_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = "1 2 3\n1 2 4\n2 3 4\n1 2 4\n2 4\n4 5\n1 2\n"
U = "1\n2\n7 8\n2 4\n4 1 2\n3\n1\n"
FREQ = "1\n1 2\n1 4\n1 4 2\n2\n3\n3 2\n4\n4 2\n"
RECS = "2\n1\n0\n1\n3\n2\n2\n"
FREQ_COUNTS = "1 2[4]\n1 4 2[2]\n1 4[2]\n1[4]\n2[6]\n3 2[2]\n3[2]\n4 2[4]\n4[5]\n"


def test_oracle_golden():
    lines, recs, res = run_oracle(D.splitlines(), U.splitlines(), 0.25)
    assert "\n".join(lines) + "\n" == FREQ
    assert "\n".join(recs) + "\n" == RECS
    assert res.min_count == 2 and res.items == ["2", "4", "1", "3"]


@pytest.mark.parametrize("strategy", ["horizontal", "gram"])
@pytest.mark.parametrize("dedup", ["on", "off"])
def test_miner_golden(strategy, dedup):
    sh = parse_bytes(D.encode())
    cfg = MinerConfig(min_support=0.25, pair_strategy=strategy, dedup=dedup)
    res = FastApriori(0.25, config=cfg).run(sh)
    assert res.items == ["2", "4", "1", "3"]
    assert [c.tolist() for c in res.counts] == [[6, 5, 4, 2], [4, 4, 2, 2], [2]]
    ar = AssociationRules(res)
    rules = ar.rule_list()
    assert len(rules) == 8                       # the 3 level-2 rules are cut
    tok = res.items
    assert [(tuple(tok[a] for a in ante), tok[c]) for ante, c, _ in rules[:4]] == \
        [(("1",), "2"), (("3",), "2"), (("4",), "2"), (("2",), "1")]
    assert ar.run(parse_bytes(U.encode())) == RECS.split()


def _write_inputs(d):
    with open(os.path.join(d, "D.dat"), "w") as f:
        f.write(D)
    with open(os.path.join(d, "U.dat"), "w") as f:
        f.write(U)


def test_cli_end_to_end_bytes(tmp_path):
    _write_inputs(tmp_path)
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "fastapriori_amd", f"{tmp_path}/", f"{tmp_path}/out_",
                        f"{tmp_path}/tmp", "--min-support", "0.25", "--device", "cpu", "--with-counts"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    assert open(tmp_path / "out_freqItemset" / "part-00000").read() == FREQ
    assert open(tmp_path / "out_recommends" / "part-00000").read() == RECS
    assert open(tmp_path / "out_freqItems" / "part-00000").read() == FREQ_COUNTS
    assert (tmp_path / "out_freqItemset" / "_SUCCESS").exists()
    assert "==== Total time for get freqItemsets" in r.stdout
    assert "==== Size association rules 8" in r.stdout


def test_refuses_existing_output(tmp_path):
    _write_inputs(tmp_path)
    cfg = JobConfig(input=f"{tmp_path}/", output=f"{tmp_path}/o_", min_support=0.25, device="cpu")
    run_job(cfg, Comm())
    with pytest.raises(OutputExistsError):
        run_job(cfg, Comm())
    cfg.overwrite = True
    run_job(cfg, Comm())
    assert open(tmp_path / "o_recommends" / "part-00000").read() == RECS


# equal counts of "9" and "10": String order puts "10" first, the numeric tiebreak "9"
TIE_D = "9 10\n9 10\n9 10 3\n3\n"


@pytest.mark.parametrize("tb,want", [("string", ["10", "9", "3"]), ("numeric", ["9", "10", "3"])])
def test_tiebreak_orders_equal_counts(tmp_path, tb, want):
    # --tiebreak: the rank order of equal-count items; the itemsets as token
    # sets and their counts do not depend on it, only the token order inside a line
    res = FastApriori(0.5, config=MinerConfig(min_support=0.5, tiebreak=tb)).run(parse_bytes(TIE_D.encode()))
    assert res.items == want
    lines, _, ores = run_oracle(TIE_D.splitlines(), [], 0.5, tiebreak=tb)
    assert ores.items == want
    sets = {frozenset(l.split()) for l in lines}
    assert sets == {frozenset(l.split()) for l in run_oracle(TIE_D.splitlines(), [], 0.5)[0]}
    with open(tmp_path / "D.dat", "w") as f:
        f.write(TIE_D)
    with open(tmp_path / "U.dat", "w") as f:
        f.write("9\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "fastapriori_amd", f"{tmp_path}/", f"{tmp_path}/o_", "--min-support",
                        "0.5", "--device", "cpu", "--tiebreak", tb], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert open(tmp_path / "o_freqItemset" / "part-00000").read() == "\n".join(lines) + "\n"
