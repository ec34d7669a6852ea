"""Synthetic data generator properties and the bench.py output contract."""
import json
import os
import subprocess
import sys

import numpy as np

from fastapriori_amd.parallel.comm import Comm
from fastapriori_amd.utils.io import generate_shard, parse_file, write_quest_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _FakeComm(Comm):
    pass


def _rows(sh):
    off, it = sh.offsets.numpy(), sh.items.numpy()
    return [tuple(it[off[i]:off[i + 1]].tolist()) for i in range(sh.n_lines)]


def test_generation_is_shard_invariant():
    full = _rows(generate_shard(5000, Comm(), "cpu", 10.0, 4.0, 100, 200, seed=9))
    parts = []
    for r in range(3):
        parts += _rows(generate_shard(5000, Comm(rank=r, world_size=3), "cpu", 10.0, 4.0, 100, 200, seed=9))
    assert parts == full


def test_generation_statistics():
    sh = generate_shard(20000, Comm(), "cpu", 10.0, 4.0, 2000, 1000, seed=1)
    lens = np.diff(sh.offsets.numpy())
    assert 8.5 < lens.mean() < 12.5
    ids = sh.items.numpy()
    assert ids.min() >= 2 and ids.max() <= 1001          # items 1..N as numeric ids value+1


def test_file_writer_matches_in_memory(tmp_path):
    write_quest_file(str(tmp_path / "D.dat"), 3000, 10.0, 4.0, 100, 100, seed=4)
    a = _rows(parse_file(str(tmp_path / "D.dat")))
    b = _rows(generate_shard(3000, Comm(), "cpu", 10.0, 4.0, 100, 100, seed=4))
    assert a == b


def test_bench_json_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "T10I4D1K", "--device", "cpu",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["config"]["n_itemsets"] > 0
    assert abs(d["value"] - d["config"]["n_itemsets"] / (d["ms_per_step"] / 1e3)) / d["value"] < 0.01


def test_bench_per_rank_record_world8():
    # bench.py --gpus 8 relaunches itself under torch.distributed.run (gloo on the CPU here):
    # the JSON line carries one diagnostic record per rank plus the spread
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--device", "cpu",
                        "--config", "T10I4D1K", "--steps", "2", "--warmup", "1", "--e2e", "off"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["world_size"] == 8 and d["config"]["parallelism"] == "dp8"
    pr = d["per_rank"]
    assert [p["rank"] for p in pr] == list(range(8))
    for p in pr:
        assert p["ms_per_step"] > 0 and p["comm_ms_per_step"] >= 0 and p["collectives_per_step"] > 0
    assert d["ms_per_step"] == max(p["ms_per_step"] for p in pr)
    assert d["rank_spread_ms"] == round(max(p["ms_per_step"] for p in pr) - min(p["ms_per_step"] for p in pr), 3)


def test_bench_e2e_window_world2():
    # the e2e record through pipeline.mine_window (checkpointing on, its completion joined
    # after the window) with 2 ranks reading their byte ranges of one D.dat
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--config", "T10I4D1K", "--steps", "1", "--warmup", "1", "--e2e", "on"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    e = d["e2e"]
    assert e["n_itemsets"] == d["config"]["n_itemsets"] and e["warm_ms"] > 0 and e["cold_ms"] > 0
