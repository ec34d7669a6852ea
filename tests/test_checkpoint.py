"""Checkpoint / resume / rules-only / getAll-format reload and fault injection."""
import os
import subprocess
import sys

import numpy as np

from fastapriori_amd.config import JobConfig
from fastapriori_amd.models.apriori import FastApriori, MinerConfig
from fastapriori_amd.parallel.comm import Comm
from fastapriori_amd.pipeline import run_job
from fastapriori_amd.utils.checkpoint import Checkpointer
from fastapriori_amd.utils.io import load_saved_results, write_freq_itemsets, write_items_to_rank, \
    write_quest_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _inputs(d):
    write_quest_file(str(d / "D.dat"), 3000, 9.0, 4.0, 40, 40, seed=3)
    write_quest_file(str(d / "U.dat"), 400, 9.0, 4.0, 40, 40, seed=3, users=True)


def _read(p):
    return open(p).read()


def test_fault_then_resume_gives_identical_outputs(tmp_path):
    _inputs(tmp_path)
    env = dict(os.environ, PYTHONPATH=ROOT, FA_FAULT_AT_LEVEL="3")
    args = [sys.executable, "-m", "fastapriori_amd", f"{tmp_path}/", f"{tmp_path}/a_", f"{tmp_path}/tmp",
            "--min-support", "0.02", "--device", "cpu"]
    r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 17, r.stderr                      # injected crash after level 3
    assert not os.path.exists(tmp_path / "a_freqItemset")
    ck = Checkpointer(str(tmp_path / "tmp")).load()
    assert ck is not None and len(ck.levels) == 3 and not ck.stats.get("complete")
    env.pop("FA_FAULT_AT_LEVEL")
    r = subprocess.run(args + ["--resume"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    # fresh run elsewhere for comparison
    run_job(JobConfig(input=f"{tmp_path}/", output=f"{tmp_path}/b_", min_support=0.02, device="cpu"), Comm())
    assert _read(tmp_path / "a_freqItemset/part-00000") == _read(tmp_path / "b_freqItemset/part-00000")
    assert _read(tmp_path / "a_recommends/part-00000") == _read(tmp_path / "b_recommends/part-00000")


def test_rules_only_from_checkpoint(tmp_path):
    _inputs(tmp_path)
    cfg = JobConfig(input=f"{tmp_path}/", output=f"{tmp_path}/a_", temp=str(tmp_path / "t"), min_support=0.02,
                    device="cpu")
    run_job(cfg, Comm())
    rec = _read(tmp_path / "a_recommends/part-00000")
    os.remove(tmp_path / "D.dat")                     # rules-only does not read the mining input
    cfg2 = JobConfig(input=f"{tmp_path}/", output=f"{tmp_path}/c_", temp=str(tmp_path / "t"), min_support=0.02,
                     device="cpu", rules_only=True)
    s = run_job(cfg2, Comm())
    assert "miner" not in s
    assert _read(tmp_path / "c_recommends/part-00000") == rec


def test_getall_format_roundtrip(tmp_path):
    from fastapriori_amd.utils.io import generate_shard
    sh = generate_shard(2000, Comm(), "cpu", 8.0, 3.0, 30, 30, seed=1)
    res = FastApriori(0.03, config=MinerConfig(min_support=0.03)).run(sh)
    write_freq_itemsets(res, str(tmp_path / "freqItems"), with_counts=True)
    write_items_to_rank(res, str(tmp_path / "ItemsToRank"))
    back = load_saved_results(str(tmp_path / "freqItems"), str(tmp_path / "ItemsToRank"))
    assert back.items == res.items
    assert back.as_dict() == res.as_dict()
    for a, b in zip(back.levels, res.levels):
        assert np.array_equal(a, b)


def test_rules_only_from_saved_results(tmp_path):
    # no checkpoint: --rules-only rebuilds the result from a --with-counts run's
    # freqItems + ItemsToRank (Utils.getAll, Utils.scala:65-81)
    _inputs(tmp_path)
    cfg = JobConfig(input=f"{tmp_path}/", output=f"{tmp_path}/a_", min_support=0.02, device="cpu", with_counts=True)
    run_job(cfg, Comm())
    rec = _read(tmp_path / "a_recommends/part-00000")
    os.remove(tmp_path / "D.dat")
    os.rename(tmp_path / "a_recommends", tmp_path / "a_recommends.first")
    cfg2 = JobConfig(input=f"{tmp_path}/", output=f"{tmp_path}/a_", min_support=0.02, device="cpu", rules_only=True)
    s = run_job(cfg2, Comm())
    assert "miner" not in s
    assert _read(tmp_path / "a_recommends/part-00000") == rec
