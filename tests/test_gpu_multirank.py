"""The 8-rank design on the one GPU of the test box: 8 gloo ranks share the card and
run the default device path -- device-compacted F_2, device level bundles with the
count all-reduce inside the bundle loop -- plus the k = 2 reduce-scatter path
(FA_TUNE=pair_rs_min=0) and candidate distribution.  Every rank's result must be
bit-identical to world size 1 (FastApriori.scala:98-100,140)."""
import pytest

from fastapriori_amd.parallel.launch import spawn_local

pytestmark = pytest.mark.gpu
N, MS = 80000, 0.005


def _rank(n, ms, par):
    from fastapriori_amd import ops
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import Comm, init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger
    comm = init_comm("cuda")
    try:
        sh = generate_shard(n, comm if par == "count" else Comm(device=comm.device), comm.device, 10.0, 4.0,
                            200, 200, seed=3)
        cfg = MinerConfig(trim_min_rows=0, min_support=ms, parallelism=par)
        m = FastApriori(ms, comm, cfg, Logger(comm.rank, enabled=False))
        c0, b0 = comm.comm_calls, comm.bytes_reduced
        res = m.run(sh)
        return dict(sets=res.as_dict(), bundles=int(m.stats.get("device_bundles", 0)),
                    cand_counted=m.stats.get("cand_counted"), cand_total=m.stats.get("cand_total"),
                    f2_dev=bool(m.stats.get("f2_on_device", False)), calls=comm.comm_calls - c0,
                    bytes=comm.bytes_reduced - b0, fallbacks=list(ops.primitives.FALLBACKS),
                    world=comm.world_size)
    finally:
        shutdown_comm(comm)


@pytest.fixture(scope="module")
def ref():
    r = spawn_local(_rank, 1, N, MS, "count", env={"FA_DIST_BACKEND": "gloo"})[0]
    assert len(r["sets"]) > 500 and r["bundles"] > 0 and r["f2_dev"]
    return r


def test_eight_ranks_default_path_match_one(ref):
    outs = spawn_local(_rank, 8, N, MS, "count", env={"FA_DIST_BACKEND": "gloo"})
    for o in outs:
        assert o["world"] == 8 and o["sets"] == ref["sets"]
        assert o["bundles"] > 0 and o["f2_dev"] and o["calls"] > 0 and o["bytes"] > 0
        assert not o["fallbacks"]
        # line total, F1, layout decisions, F_2, one per device bundle (no metrics-only gather)
        assert o["calls"] <= 4 + o["bundles"], o


def test_eight_ranks_pair_reduce_scatter_match_one(ref):
    outs = spawn_local(_rank, 8, N, MS, "count", env={"FA_DIST_BACKEND": "gloo", "FA_TUNE": "pair_rs_min=0"})
    for o in outs:
        assert o["sets"] == ref["sets"] and o["bundles"] > 0 and not o["f2_dev"]


def test_eight_ranks_candidate_mode_match_one(ref):
    # candidate distribution on the device level loop: every rank holds the whole DB and
    # counts its row slice of it in the bundles (FastApriori._count_view)
    outs = spawn_local(_rank, 8, N, MS, "candidate", env={"FA_DIST_BACKEND": "gloo"})
    for o in outs:
        assert o["sets"] == ref["sets"]
        assert o["bundles"] > 0 and o["f2_dev"] and not o["fallbacks"]
    # each rank counted its own ~1/8 of the bundles' candidates (over all rows), not all
    # of them over 1/8 of the rows: the ranks' non-zero local counts add up to at most
    # the candidates, and no rank holds much more than its share
    tot = outs[0]["cand_total"]
    counted = [o["cand_counted"] for o in outs]
    assert tot > 8 * 512 and sum(counted) <= tot, (tot, counted)
    assert max(counted) <= tot / 8 * 1.5 + 512 and min(counted) > 0, (tot, counted)


def _job_rank(d, resume):
    from fastapriori_amd.config import JobConfig
    from fastapriori_amd.parallel.comm import init_comm, shutdown_comm
    from fastapriori_amd.pipeline import run_job
    comm = init_comm("cuda")
    try:
        cfg = JobConfig(input=f"{d}/", output=f"{d}/{'b' if resume else 'a'}_", temp=f"{d}/tmp", min_support=0.02,
                        device="cuda", resume=resume)
        s = run_job(cfg, comm)
        return dict(bundles=s.get("device_bundles", 0), n=s["n_itemsets"])
    finally:
        shutdown_comm(comm)


def test_two_ranks_device_loop_checkpoint_fault_resume(tmp_path):
    # only rank 0 writes the device loop's staged checkpoint (level files and
    # meta.json).  2 gloo ranks on the GPU, an injected crash of rank 0 at the level-3
    # bundle boundary, then --resume: meta.json counts exactly the level files present,
    # and the resumed job writes what a fresh world-1 job writes.
    import json
    import os

    from fastapriori_amd.config import JobConfig
    from fastapriori_amd.parallel.comm import Comm
    from fastapriori_amd.pipeline import run_job
    from fastapriori_amd.utils.io import write_quest_file
    write_quest_file(str(tmp_path / "D.dat"), 3000, 9.0, 4.0, 40, 40, seed=3)
    write_quest_file(str(tmp_path / "U.dat"), 400, 9.0, 4.0, 40, 40, seed=3, users=True)
    env = {"FA_DIST_BACKEND": "gloo", "FA_FAULT_AT_LEVEL": "3", "FA_FAULT_RANK": "0"}
    with pytest.raises(RuntimeError, match="InjectedFault"):
        spawn_local(_job_rank, 2, str(tmp_path), False, env=env, timeout=300)
    ck = tmp_path / "tmp" / "fastapriori_ckpt"
    meta = json.load(open(ck / "meta.json"))
    done = int(meta["levels_done"])
    assert done == 3 and not meta.get("complete")
    present = sorted(int(f[6:-4]) for f in os.listdir(ck) if f.startswith("level_") and f.endswith(".npz"))
    assert present == list(range(1, done + 1)), present
    outs = spawn_local(_job_rank, 2, str(tmp_path), True, env={"FA_DIST_BACKEND": "gloo"}, timeout=300)
    assert all(o["bundles"] > 0 for o in outs)
    import torch
    run_job(JobConfig(input=f"{tmp_path}/", output=f"{tmp_path}/c_", min_support=0.02, device="cuda"),
            Comm(device=torch.device("cuda", 0)))
    for name in ("freqItemset", "recommends"):
        assert (open(tmp_path / f"b_{name}/part-00000").read()
                == open(tmp_path / f"c_{name}/part-00000").read())
