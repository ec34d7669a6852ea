"""World-size-W rehearsal of the count-distributed miner on ONE GPU: W gloo ranks
share the card (FA_DIST_BACKEND=gloo), each mining its 1/W row shard of the config
through the default device path.  Timings of ranks sharing one GPU say nothing
about scaling; what this measures exactly is the communication each rank issues
per mining run: every top-level collective (Comm.trace) with the bytes it moves,
and the result's identity with world size 1.

    python benchmarks/multirank_probe.py [--world 8] [--n-txn 10000000] [--config T10I4D100M]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _ranges(cpus: list) -> str:
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def _rank(n, cfgv, ms):
    import torch
    from fastapriori_amd.models.apriori import FastApriori, MinerConfig
    from fastapriori_amd.parallel.comm import init_comm, shutdown_comm
    from fastapriori_amd.utils.io import generate_shard
    from fastapriori_amd.utils.metrics import Logger
    _, avg_len, avg_pat, n_pat, n_items, _ = cfgv
    comm = init_comm("cuda")
    try:
        sh = generate_shard(n, comm, comm.device, avg_len, avg_pat, n_pat, n_items, 1)
        m = FastApriori(ms, comm, MinerConfig(min_support=ms), Logger(comm.rank, enabled=False))
        m.run(sh)                       # warm-up
        comm.trace = []
        res = m.run(sh)
        torch.cuda.synchronize()
        tr = comm.trace
        comm.trace = None
        from fastapriori_amd.parallel.affinity import PLACEMENT
        from fastapriori_amd.utils.env import num_threads
        cpus = sorted(os.sched_getaffinity(0))
        place = dict(numa_node=PLACEMENT.get("node"), peers=PLACEMENT.get("peers"), cpus=_ranges(cpus),
                     n_cpus=len(cpus), host_threads=num_threads())
        return dict(rank=comm.rank, n_itemsets=res.n_itemsets, levels=[len(c) for c in res.counts], place=place,
                    cpu_list=cpus,
                    bundles=int(m.stats.get("device_bundles", 0)), f2_on_device=bool(m.stats.get("f2_on_device")),
                    collectives=tr, calls=len(tr), bytes=int(sum(b for _, b, _ in tr)),
                    digest=hash(tuple(sorted((tuple(sorted(k)), v) for k, v in res.as_dict().items()))))
    finally:
        shutdown_comm(comm)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--n-txn", type=int, default=10_000_000)
    ap.add_argument("--config", default="T10I4D100M")
    args = ap.parse_args()
    from bench import CONFIGS
    from fastapriori_amd.parallel.launch import spawn_local
    cfgv = CONFIGS[args.config]
    ms = cfgv[5]
    env = {"FA_DIST_BACKEND": "gloo", "FA_NUM_THREADS": "2"}
    one = spawn_local(_rank, 1, args.n_txn, cfgv, ms, env=env, timeout=900)[0]
    outs = spawn_local(_rank, args.world, args.n_txn, cfgv, ms, env=env, timeout=900)
    same = all(o["digest"] == one["digest"] for o in outs)
    r0 = outs[0]
    print(json.dumps(dict(config=args.config, n_txn=args.n_txn, world=args.world, identical_to_world1=same,
                          n_itemsets=r0["n_itemsets"], bundles=r0["bundles"], f2_on_device=r0["f2_on_device"],
                          calls_per_run=r0["calls"], bytes_per_rank=r0["bytes"],
                          calls_world1=one["calls"], collectives_rank0=r0["collectives"],
                          all_ranks_same_calls=len({o["calls"] for o in outs}) == 1,
                          # every rank's host placement on this box's real /sys (parallel.affinity:
                          # the GPU's NUMA node, its CPUs split among the local ranks)
                          placement=[dict(rank=o["rank"], **o["place"]) for o in outs],
                          cpu_slices_disjoint=sum(len(o["cpu_list"]) for o in outs)
                          == len({c for o in outs for c in o["cpu_list"]}))), flush=True)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
