"""End-to-end on the MI355X: CLI pipeline on cuda vs the oracle, and multi-rank runs
sharing the one GPU of the test box (gloo transport; the kernels are the HIP ones)."""
import os
import subprocess
import sys

import pytest
import torch

from fastapriori_amd.models.oracle import run_oracle
from fastapriori_amd.parallel.launch import spawn_local
from fastapriori_amd.utils.io import write_quest_file

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _job_record(path):
    import json
    recs = [json.loads(l) for l in open(path)]
    return [r for r in recs if r.get("phase") == "job"][-1]


def test_cli_on_gpu_matches_oracle(tmp_path):
    # the reference's three-argument form (input output temp: checkpointing on) mines
    # through the device level bundles, and its checkpoint is complete and resumable
    write_quest_file(str(tmp_path / "D.dat"), 2000, 8.0, 3.0, 40, 40, seed=6)
    write_quest_file(str(tmp_path / "U.dat"), 500, 8.0, 3.0, 40, 40, seed=6, users=True)
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "fastapriori_amd", f"{tmp_path}/", f"{tmp_path}/o_", f"{tmp_path}/t",
                        "--min-support", "0.03", "--device", "cuda", "--metrics", f"{tmp_path}/m.jsonl"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr
    d = open(tmp_path / "D.dat").read().splitlines()
    u = open(tmp_path / "U.dat").read().splitlines()
    lines, recs, res = run_oracle(d, u, 0.03)
    got = open(tmp_path / "o_freqItemset/part-00000").read().splitlines()
    # ties in F1 counts are ordered identically (count desc, Java string asc) -> exact lines
    assert got == lines
    assert open(tmp_path / "o_recommends/part-00000").read().splitlines() == recs
    assert _job_record(f"{tmp_path}/m.jsonl")["device_bundles"] > 0
    from fastapriori_amd.utils.checkpoint import Checkpointer
    ck = Checkpointer(str(tmp_path / "t")).load(require_complete=True)
    assert ck is not None
    got_ck = {frozenset(ck.items[r] for r in s): c for s, c in ck.as_dict().items()}
    want = {frozenset(res.items[r] for r in s): c for s, c in res.itemsets.items()}
    assert got_ck == want


def test_cli_fault_then_resume_on_gpu(tmp_path):
    # an injected crash after level 3 on the device path, then --resume: the device
    # loop restarts from the checkpoint's last level (uploaded as the first parents)
    write_quest_file(str(tmp_path / "D.dat"), 3000, 9.0, 4.0, 40, 40, seed=3)
    write_quest_file(str(tmp_path / "U.dat"), 400, 9.0, 4.0, 40, 40, seed=3, users=True)
    env = dict(os.environ, PYTHONPATH=ROOT, FA_FAULT_AT_LEVEL="3")
    args = [sys.executable, "-m", "fastapriori_amd", f"{tmp_path}/", f"{tmp_path}/a_", f"{tmp_path}/tmp",
            "--min-support", "0.02", "--device", "cuda", "--metrics", f"{tmp_path}/m.jsonl"]
    r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 17, r.stderr[-3000:]
    assert not os.path.exists(tmp_path / "a_freqItemset")
    from fastapriori_amd.utils.checkpoint import Checkpointer
    ck = Checkpointer(str(tmp_path / "tmp")).load()
    assert ck is not None and len(ck.levels) == 3 and not ck.stats.get("complete")
    env.pop("FA_FAULT_AT_LEVEL")
    r = subprocess.run(args + ["--resume"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _job_record(f"{tmp_path}/m.jsonl")["device_bundles"] > 0
    d = open(tmp_path / "D.dat").read().splitlines()
    u = open(tmp_path / "U.dat").read().splitlines()
    lines, recs, _ = run_oracle(d, u, 0.02)
    assert open(tmp_path / "a_freqItemset/part-00000").read().splitlines() == lines
    assert open(tmp_path / "a_recommends/part-00000").read().splitlines() == recs


def test_cli_under_torchrun_rccl_matches_oracle(tmp_path):
    # the CLI job through torchrun with an RCCL process group (world size 1, every
    # collective forced): shard reading, line offsets, gathers and rank-0 writes
    write_quest_file(str(tmp_path / "D.dat"), 3000, 8.0, 3.0, 40, 40, seed=8)
    write_quest_file(str(tmp_path / "U.dat"), 700, 8.0, 3.0, 40, 40, seed=8, users=True)
    env = dict(os.environ, PYTHONPATH=ROOT, FA_FORCE_PG="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", "-m", "fastapriori_amd",
                        f"{tmp_path}/", f"{tmp_path}/o_", f"{tmp_path}/t", "--min-support", "0.03",
                        "--device", "cuda"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = open(tmp_path / "D.dat").read().splitlines()
    u = open(tmp_path / "U.dat").read().splitlines()
    lines, recs, _ = run_oracle(d, u, 0.03)
    assert open(tmp_path / "o_freqItemset/part-00000").read().splitlines() == lines
    assert open(tmp_path / "o_recommends/part-00000").read().splitlines() == recs


def _gpu_rank(n, ms, par="count", dedup="auto"):
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm, init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger
    comm = init_comm("cuda")
    try:
        # candidate mode: every rank holds the whole DB
        sh = generate_shard(n, comm if par == "count" else Comm(device=comm.device), comm.device, 10.0, 4.0,
                            200, 200, seed=3)
        cfg = MinerConfig(trim_min_rows=0, min_support=ms, parallelism=par, dedup=dedup)
        res = FastApriori(ms, comm, cfg, Logger(comm.rank, enabled=False)).run(sh)
        return res.as_dict()
    finally:
        shutdown_comm(comm)


def test_two_ranks_share_gpu_match_one():
    ref = spawn_local(_gpu_rank, 1, 40000, 0.005, env={"FA_DIST_BACKEND": "gloo"})[0]
    outs = spawn_local(_gpu_rank, 2, 40000, 0.005, env={"FA_DIST_BACKEND": "gloo"})
    assert outs[0] == ref and outs[1] == ref
    outs = spawn_local(_gpu_rank, 2, 40000, 0.005, env={"FA_DIST_BACKEND": "gloo", "FA_TUNE": "pair_rs_min=0"})
    assert outs[0] == ref and outs[1] == ref
    assert len(ref) > 100


@pytest.mark.parametrize("dedup", ["off", "on"])
def test_two_ranks_share_gpu_candidate_mode(dedup):
    # candidate distribution: each rank counts its blocks of the device bundles' piece
    # records over the whole replicated DB (FastApriori._piece_part), unit and weighted
    # (dedup) layouts
    ref = spawn_local(_gpu_rank, 1, 40000, 0.005, "count", dedup, env={"FA_DIST_BACKEND": "gloo"})[0]
    outs = spawn_local(_gpu_rank, 2, 40000, 0.005, "candidate", dedup, env={"FA_DIST_BACKEND": "gloo"})
    assert outs[0] == ref and outs[1] == ref


def _rccl_rank(n, ms, strategy):
    """Mining, rules and recommendations through the RCCL code paths (world size 1,
    FA_FORCE_PG=1): every collective of the multi-GPU run executes on the device."""
    import numpy as np
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.models.rules import AssociationRules
    from fastapriori_amd.parallel.comm import init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_shard, parse_bytes
    from fastapriori_amd.utils.metrics import Logger
    comm = init_comm("cuda")
    try:
        if os.environ.get("FA_FORCE_PG") == "1":
            assert comm.backend == "nccl" and comm.distributed
        log = Logger(comm.rank, enabled=False)
        sh = generate_shard(n, comm, comm.device, 10.0, 4.0, 200, 200, seed=3)
        res = FastApriori(ms, comm, MinerConfig(min_support=ms, parallelism=strategy), log).run(sh)
        users = generate_shard(2000, comm, comm.device, 10.0, 4.0, 200, 200, seed=3, users=True)
        recs = AssociationRules(res, comm, log).run(users)
        # dictionary vocabulary: hash all-to-all + all_gather_object on RCCL
        words = parse_bytes(b"a b c\nb c d\na c\nc d e a\n" * 50, device=comm.device)
        dres = FastApriori(0.2, comm, MinerConfig(min_support=0.2), log).run(words)
        comm.barrier()
        t = comm.allreduce_float_max(1.5)
        return res.as_dict(), recs, dres.as_dict(), dres.items, t, comm.bytes_reduced
    finally:
        shutdown_comm(comm)


@pytest.mark.parametrize("strategy", ["count", "candidate"])
def test_rccl_code_paths_match_single_process(strategy):
    ref = spawn_local(_rccl_rank, 1, 60000, 0.004, strategy)[0]
    # FA_TUNE=pair_rs_min=0: the k = 2 triangle takes reduce-scatter + threshold + all-gather on RCCL
    got = spawn_local(_rccl_rank, 1, 60000, 0.004, strategy, env={"FA_FORCE_PG": "1", "FA_TUNE": "pair_rs_min=0"})[0]
    assert got[0] == ref[0] and got[1] == ref[1] and got[2] == ref[2] and got[3] == ref[3]
    assert got[4] == 1.5 and got[5] > 0 and ref[5] == 0
    if strategy == "count":
        # default threshold: the triangle is all-reduced on RCCL and F_2 compacted on the device
        # (no host round trip before the first device bundle)
        got = spawn_local(_rccl_rank, 1, 60000, 0.004, strategy, env={"FA_FORCE_PG": "1"})[0]
        assert got[0] == ref[0] and got[1] == ref[1] and got[2] == ref[2] and got[3] == ref[3]
