"""World-size 8 (the MI355X node) on gloo: skewed shards must not crash, hang or diverge.

Every collective call site is reached by every rank regardless of its local data
(a rank with no lines, a rank whose lines keep no row with two frequent items, a
rank that votes against a layout its peers chose).  Results must be bit-identical
to world size 1.  Reference: Main.scala:18 (parallelism is configuration),
FastApriori.scala:66-79 (compression + dedup), :98-100,140 (candidate mode).
"""
import os

import pytest

from fastapriori_amd.parallel.launch import spawn_local

from test_distributed import _mine_file

TIMEOUT = 240


def _write(path, lines):
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


@pytest.fixture(scope="module")
def skew_db(tmp_path_factory):
    # 300 lines "1 2" then 900 single-item lines: the byte-range shards of the
    # later ranks hold no row with two frequent items (T = 0 after compression)
    d = tmp_path_factory.mktemp("skew")
    lines = ["1 2"] * 300 + [str(3 + (i % 5)) for i in range(900)]
    _write(d / "D.dat", lines)
    _write(d / "U.dat", ["1", "2", "1 2", "3", "9", ""])
    return str(d) + "/"


@pytest.fixture(scope="module")
def tiny_db(tmp_path_factory):
    # fewer lines than ranks: some ranks' byte ranges start no line at all
    d = tmp_path_factory.mktemp("tiny")
    _write(d / "D.dat", ["1 2 3", "1 2", "2 3", "1 3 4", "1 2 3 4"])
    _write(d / "U.dat", ["1", "2 3", "4", "5", "1 2", "3", "2", "1 4", "3 4"])
    return str(d) + "/"


@pytest.fixture(scope="module")
def quest_db(tmp_path_factory):
    from fastapriori_amd.utils.io import write_quest_file
    d = tmp_path_factory.mktemp("q8")
    write_quest_file(str(d / "D.dat"), 6000, 8.0, 3.0, 60, 50, seed=11)
    write_quest_file(str(d / "U.dat"), 500, 8.0, 3.0, 60, 50, seed=11, users=True)
    return str(d) + "/"


def _check(outs, ref):
    for o in outs:
        assert o["items"] == ref["items"]
        assert o["sets"] == ref["sets"]
    assert outs[0]["recs"] == ref["recs"]
    assert sum(o["lines"] for o in outs) == ref["lines"]


@pytest.mark.parametrize("dedup", ["on", "auto", "off"])
def test_rank_with_no_compressed_rows(skew_db, dedup):
    ref = spawn_local(_mine_file, 1, skew_db, 0.1, dedup, "auto", timeout=TIMEOUT)[0]
    assert frozenset([0, 1]) in {frozenset(s) for s in ref["sets"]} or len(ref["sets"]) >= 3
    for world in (2, 8):
        outs = spawn_local(_mine_file, world, skew_db, 0.1, dedup, "auto", timeout=TIMEOUT)
        _check(outs, ref)


@pytest.mark.parametrize("strategy", ["horizontal", "gram"])
def test_ranks_without_lines(tiny_db, strategy):
    ref = spawn_local(_mine_file, 1, tiny_db, 0.3, "auto", strategy, timeout=TIMEOUT)[0]
    outs = spawn_local(_mine_file, 8, tiny_db, 0.3, "auto", strategy, timeout=TIMEOUT)
    _check(outs, ref)
    assert any(o["lines"] == 0 for o in outs)
    assert len(ref["recs"]) == 9


@pytest.mark.parametrize("dedup,strategy", [("on", "horizontal"), ("off", "gram"), ("auto", "auto")])
def test_world8_matches_single_rank(quest_db, dedup, strategy):
    ref = spawn_local(_mine_file, 1, quest_db, 0.02, dedup, strategy, timeout=TIMEOUT)[0]
    outs = spawn_local(_mine_file, 8, quest_db, 0.02, dedup, strategy, timeout=TIMEOUT)
    _check(outs, ref)
    assert max(len(s) for s in ref["sets"]) >= 3


@pytest.mark.parametrize("world", [2, 4, 8])
def test_pair_reduce_scatter_select(quest_db, world):
    # X12 as reduce-scatter + per-slice threshold + all-gather of the survivors
    # (forced for every triangle size): bit-identical to the all-reduce path
    ref = spawn_local(_mine_file, 1, quest_db, 0.02, "auto", "horizontal", timeout=TIMEOUT)[0]
    outs = spawn_local(_mine_file, world, quest_db, 0.02, "auto", "horizontal", timeout=TIMEOUT,
                       env={"FA_TUNE": "pair_rs_min=0"})
    _check(outs, ref)


def test_world8_candidate_mode(quest_db):
    ref = spawn_local(_mine_file, 1, quest_db, 0.02, "auto", "auto", timeout=TIMEOUT)[0]
    outs = spawn_local(_mine_file, 8, quest_db, 0.02, "auto", "auto", "candidate", timeout=TIMEOUT)
    _check([dict(o, lines=o["lines"] if i == 0 else 0) for i, o in enumerate(outs)], ref)


def _crash_rank1():
    from fastapriori_amd.parallel.comm import init_comm
    comm = init_comm("cpu")
    if comm.rank == 1:
        raise RuntimeError("injected")
    comm.allreduce_int(1)      # blocks: rank 1 never joins
    return comm.rank


def _hang_rank0():
    import time
    from fastapriori_amd.parallel.comm import init_comm
    comm = init_comm("cpu")
    if comm.rank == 0:
        time.sleep(3600)
    return comm.rank


def test_spawn_local_fails_fast_on_a_crashed_rank():
    import time
    t = time.monotonic()
    with pytest.raises(RuntimeError, match="injected"):
        spawn_local(_crash_rank1, 2, timeout=120)
    assert time.monotonic() - t < 100


def test_spawn_local_times_out_on_a_hang():
    with pytest.raises(TimeoutError):
        spawn_local(_hang_rank0, 2, timeout=20)


def test_bench_launches_and_checks_world_size():
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--device", "cpu",
                        "--config", "T10I4D1K", "--steps", "1", "--warmup", "0", "--e2e", "off"],
                       capture_output=True, text=True, timeout=TIMEOUT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["world_size"] == 4 and line["config"]["parallelism"] == "dp4"
    # under a launcher with a different world size the bench refuses to run
    env2 = dict(env, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r2 = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--device", "cpu",
                         "--config", "T10I4D1K", "--steps", "1", "--warmup", "0"],
                        capture_output=True, text=True, timeout=TIMEOUT, env=env2)
    assert r2.returncode == 2 and "WORLD_SIZE=2" in r2.stderr
