"""Expected outputs of a mid-size, deep database from the independent brute-force
oracle (fastapriori_amd/models/oracle.py: plain Python sets, the reference's
semantics restated), for tests/test_gpu_oracle_deep.py.  The database is the seeded
Quest generator's (csrc/host/quest.cpp), so only the oracle's answer is stored:
sha256 of the exact freqItemset and recommends file bytes plus per-level counts.

    python tests/fixtures/make_oracle_fixture.py      (about 2 minutes on one core)
"""
import hashlib
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

GEN = dict(n_txn=20000, avg_len=12.0, avg_pat=6.0, n_patterns=100, n_items=200, seed=5)
GEN_U = dict(n_txn=2000, avg_len=12.0, avg_pat=6.0, n_patterns=100, n_items=200, seed=5, users=True)
MIN_SUPPORT = 0.02


def write_inputs(d: str) -> None:
    from fastapriori_amd.utils.io import write_quest_file
    g = dict(GEN)
    write_quest_file(os.path.join(d, "D.dat"), g.pop("n_txn"), **g)
    u = dict(GEN_U)
    write_quest_file(os.path.join(d, "U.dat"), u.pop("n_txn"), **u)


def main() -> None:
    from fastapriori_amd.models.oracle import run_oracle
    with tempfile.TemporaryDirectory() as d:
        write_inputs(d)
        D = open(os.path.join(d, "D.dat")).read().splitlines()
        U = open(os.path.join(d, "U.dat")).read().splitlines()
    lines, recs, res = run_oracle(D, U, MIN_SUPPORT)
    levels = {}
    for s in res.itemsets:
        levels[len(s)] = levels.get(len(s), 0) + 1
    freq = ("\n".join(lines) + "\n").encode() if lines else b""
    rec = ("\n".join(recs) + "\n").encode() if recs else b""
    out = dict(gen=GEN, gen_users=GEN_U, min_support=MIN_SUPPORT, oracle="fastapriori_amd/models/oracle.py",
               freqItemset_sha256=hashlib.sha256(freq).hexdigest(), recommends_sha256=hashlib.sha256(rec).hexdigest(),
               n_itemsets=len(res.itemsets), levels={str(k): v for k, v in sorted(levels.items())})
    with open(os.path.join(HERE, "oracle_q20k.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
