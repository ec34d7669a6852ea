"""Observability: ``--profile`` writes the JSON-lines metrics
stream (per-level candidates / frequent / ms / bytes reduced / HBM-bytes estimate)
and a Chrome trace of the mining phases; the "==== " lines of the reference
(FastApriori.scala:103-127) are unchanged."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_profile_writes_metrics_and_trace(tmp_path):
    from fastapriori_amd.utils.io import write_quest_file
    d = str(tmp_path) + "/"
    write_quest_file(d + "D.dat", 3000, 8.0, 3.0, 60, 50, seed=2)
    write_quest_file(d + "U.dat", 200, 8.0, 3.0, 60, 50, seed=2, users=True)
    tmp = tmp_path / "tmp"
    tmp.mkdir()
    env = {k: v for k, v in os.environ.items() if not k.startswith("FA_")}
    env["PYTHONPATH"] = ROOT
    r = subprocess.run([sys.executable, "-m", "fastapriori_amd", d, d + "out/", str(tmp), "--min-support", "0.02",
                        "--device", "cpu", "--profile"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "==== Total freq items sets" in r.stdout
    recs = [json.loads(l) for l in open(tmp / "fastapriori_metrics.jsonl")]
    levels = [x for x in recs if x.get("phase") == "level"]
    assert [x["k"] for x in levels][:2] == [2, 3]
    for x in levels:
        for key in ("candidates", "frequent", "ms", "bytes_reduced", "hbm_bytes_est"):
            assert key in x
    assert any(x.get("phase") == "job" for x in recs)
    trace = json.load(open(tmp / "fastapriori_trace.json"))
    names = {e["name"] for e in trace["traceEvents"]}
    assert {"f1", "compress", "pairs"} <= names


def test_world_size_guard_refuses_mismatch(tmp_path):
    from fastapriori_amd.utils.io import write_quest_file
    d = str(tmp_path) + "/"
    write_quest_file(d + "D.dat", 500, 8.0, 3.0, 60, 50, seed=2)
    write_quest_file(d + "U.dat", 50, 8.0, 3.0, 60, 50, seed=2, users=True)
    env = {k: v for k, v in os.environ.items() if not k.startswith("FA_")}
    env.update(PYTHONPATH=ROOT, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-m", "fastapriori_amd", d, d + "out/", "--device", "cpu",
                        "--world-size", "2"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "--world-size 2" in r.stderr


def test_world_size_launches_ranks(tmp_path):
    from fastapriori_amd.utils.io import write_quest_file
    d = str(tmp_path) + "/"
    write_quest_file(d + "D.dat", 2000, 8.0, 3.0, 60, 50, seed=2)
    write_quest_file(d + "U.dat", 100, 8.0, 3.0, 60, 50, seed=2, users=True)
    env = {k: v for k, v in os.environ.items() if not k.startswith("FA_") and k not in ("WORLD_SIZE", "RANK")}
    env["PYTHONPATH"] = ROOT
    r1 = subprocess.run([sys.executable, "-m", "fastapriori_amd", d, d + "o1/", "--device", "cpu",
                         "--min-support", "0.02"], capture_output=True, text=True, env=env, timeout=300)
    r2 = subprocess.run([sys.executable, "-m", "fastapriori_amd", d, d + "o2/", "--device", "cpu",
                         "--min-support", "0.02", "--world-size", "3"], capture_output=True, text=True, env=env,
                        timeout=300)
    assert r1.returncode == 0 and r2.returncode == 0, r2.stderr[-3000:]
    for part in ("freqItemset/part-00000", "recommends/part-00000"):
        assert open(d + "o1/" + part).read() == open(d + "o2/" + part).read()


def test_fallbacks_are_reported_by_the_run_that_took_them(tmp_path):
    # a fallback noted by an earlier phase is not re-reported by a later mining run,
    # and the rules phase reports its own (ops.primitives.reset_fallbacks)
    from fastapriori_amd import ops
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.models.rules import AssociationRules
    from fastapriori_amd.utils.io import parse_bytes
    from fastapriori_amd.utils.metrics import Logger
    ops.primitives.note_fallback("test: an earlier phase took a host fallback")
    shard = parse_bytes(b"1 2 3\n1 2 4\n2 3 4\n1 2 4\n2 4\n4 5\n1 2\n")
    m = FastApriori(0.25, config=MinerConfig(min_support=0.25), logger=Logger(0, enabled=False))
    res = m.run(shard)
    assert "fallbacks" not in m.stats and ops.primitives.FALLBACKS == []
    ar = AssociationRules(res, logger=Logger(0, enabled=False))
    ar.run(parse_bytes(b"1\n2\n"))
    assert "fallbacks" not in ar.stats


def test_retired_env_variables_are_reported():
    # a job script still setting a variable of an earlier version is told
    # what replaced it, instead of running with the default silently
    from fastapriori_amd.config import unread_env
    w = unread_env({"FA_DEDUP": "on", "FA_DL_MULTI": "0", "FA_TUNE": "x=1", "FA_MIN_SUPPORT": "0.1",
                    "FA_TYPO": "1", "HOME": "/"})
    assert any(x.startswith("FA_DEDUP is no longer read: use --dedup") for x in w)
    assert any("FA_DL_MULTI" in x and "dl_multi" in x for x in w)
    assert any("FA_TYPO" in x and "unknown" in x for x in w)
    assert not any(x.startswith(("FA_TUNE", "FA_MIN_SUPPORT")) for x in w)
