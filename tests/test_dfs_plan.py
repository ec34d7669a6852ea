"""Level-bundle work plan for the depth-2 prefix-reuse kernel (ops.plan_bundle_dfs):
emulating the kernel's walk on random item columns must give every bundled
candidate's exact support (CPU; the kernel itself is covered by the GPU tests)."""
import numpy as np

from fastapriori_amd.ops import primitives as prim
from fastapriori_amd.ops.host import apriori_gen


def _chain(prev, depth):
    """Bundle levels as FastApriori._plan_bundle builds them: level j+1 from level j's candidates."""
    levels, cur = [], prev
    for _ in range(depth):
        pi, eo, ex = apriori_gen(cur)
        if ex.size == 0:
            break
        levels.append((cur, pi, eo, ex))
        g = np.repeat(np.arange(pi.size), np.diff(eo))
        cur = np.ascontiguousarray(np.concatenate([cur[pi[g]], ex[:, None]], axis=1), dtype=np.int32)
    return levels


def _emulate(plan, cols):
    """The kernel's walk: prefix AND, depth-1 AND kept for the depth-2 children."""
    used_cols = cols[plan["used"]]                     # slab row -> column bits (bool [n_used, T])
    out = np.zeros(plan["C"], dtype=np.int64)
    for (po, pl), (b, e) in zip(plan["gpm"], plan["prng"]):
        p = np.logical_and.reduce(used_cols[plan["gpre"][po:po + pl]], axis=0)
        for u, o, c0, c1 in plan["node1"][b:e]:
            v1 = p & used_cols[u]
            out[o] += v1.sum()
            for u2, o2 in plan["node2"][c0:c1]:
                out[o2] += (v1 & used_cols[u2]).sum()
    return out


def test_dfs_plan_counts_every_candidate_once():
    rng = np.random.default_rng(4)
    F1, T = 40, 3000
    cols = rng.random((F1, T)) < 0.35
    # a dense frequent level of 3-itemsets over 14 items -> several bundled levels
    items = np.arange(14)
    rows = np.array([(a, b, c) for a in items for b in items if b > a for c in items if c > b], dtype=np.int32)
    levels = _chain(rows, 4)
    assert len(levels) >= 3
    plan = prim.plan_bundle_dfs(levels, F1)
    got = _emulate(plan, cols)
    want = []
    for pv, pi, eo, ex in levels:
        g = np.repeat(np.arange(pi.size), np.diff(eo))
        cand = np.concatenate([pv[pi[g]], ex[:, None]], axis=1)
        want.append(np.logical_and.reduce(cols[cand], axis=1).sum(axis=1))
    assert np.array_equal(got, np.concatenate(want))
    # every candidate is exactly one node: depth-1 nodes for even levels, depth-2 for odd ones
    assert plan["node1"].shape[0] + (plan["node2"].shape[0] if len(levels) > 1 else 0) == plan["C"]
    assert set(plan["node1"][:, 1]) | set(plan["node2"][:, 1]) == set(range(plan["C"]))


def test_native_plan_matches_numpy_plan():
    items = np.arange(3, 15)
    rows = np.array([(a, b, c) for a in items for b in items if b > a for c in items if c > b], dtype=np.int32)
    levels = _chain(rows, 5)
    assert len(levels) >= 3
    ref = prim.plan_bundle_dfs(levels, 30)
    buf, info = prim.plan_bundle_dfs_native(levels, 30)
    b = buf.numpy()
    n_used, NP, N1, N2 = (int(x) for x in info[:4])
    o = [int(x) for x in info[5:12]]
    assert int(info[4]) == ref["C"]
    assert np.array_equal(b[o[0]:o[0] + 30], ref["item_map"][:30])
    assert np.array_equal(b[o[1]:o[1] + n_used], ref["used"])
    assert np.array_equal(b[o[2]:o[2] + ref["gpre"].size], ref["gpre"])
    assert np.array_equal(b[o[3]:o[3] + 2 * NP].reshape(-1, 2), ref["gpm"])
    assert np.array_equal(b[o[4]:o[4] + 2 * NP].reshape(-1, 2), ref["prng"])
    assert np.array_equal(b[o[5]:o[5] + 4 * N1].reshape(-1, 4), ref["node1"])
    assert np.array_equal(b[o[6]:o[6] + 2 * N2].reshape(-1, 2), ref["node2"])
