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
