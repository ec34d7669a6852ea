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
    buf, info, passes = prim.plan_bundle_dfs_native(levels, 30)
    assert passes.tolist() == [[0, int(info[1]), 0, int(info[4]), int(info[4])]]
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


def _emulate_dfs(bits_by_rank, buf, info, passes):
    """CPU model of k_count_slab<kDfs> over a plan of fa_plan_dfs, pass by pass:
    counters [0, nA) of a pass go to out[A0 ..], [nA, ..) to out[B0 ..]."""
    n_used, NP, N1, N2, C = (int(x) for x in info[:5])
    o = [int(x) for x in info[5:12]]
    used = buf[o[1]:o[1] + n_used]
    bits = bits_by_rank[used]
    gpre = buf[o[2]:o[3]]
    gpm = buf[o[3]:o[3] + 2 * NP].reshape(-1, 2)
    prng = buf[o[4]:o[4] + 2 * NP].reshape(-1, 2)
    node1 = buf[o[5]:o[5] + 4 * N1].reshape(-1, 4)
    node2 = buf[o[6]:o[6] + 2 * max(N2, 1)].reshape(-1, 2)
    out = np.zeros(C, np.int64)
    for p0, p1, a0, na, b0 in passes.tolist():
        acc = {}
        for g in range(p0, p1):
            p = np.logical_and.reduce(bits[gpre[gpm[g, 0]:gpm[g, 0] + gpm[g, 1]]])
            for i in range(prng[g, 0], prng[g, 1]):
                v1 = p & bits[node1[i, 0]]
                acc[node1[i, 1]] = acc.get(node1[i, 1], 0) + int(v1.sum())
                for j in range(node1[i, 2], node1[i, 3]):
                    acc[node2[j, 1]] = acc.get(node2[j, 1], 0) + int((v1 & bits[node2[j, 0]]).sum())
        for key, v in acc.items():
            out[a0 + key if key < na else b0 + key - na] += v
    return out


def test_multipass_dfs_plan_counts_exactly():
    # two bundled levels split into accumulator passes of <= cap counters: every pass
    # holds whole pieces, their nodes and those nodes' children; counts must be exact
    rng = np.random.default_rng(5)
    F1, T = 14, 700
    bits = rng.random((F1, T)) < 0.55
    items = np.arange(F1)
    rows = np.array([(a, b, c) for a in items for b in items if b > a for c in items if c > b], dtype=np.int32)
    levels = _chain(rows, 2)
    assert len(levels) == 2
    C0, C1 = levels[0][3].size, levels[1][3].size
    for cap in (40, 97, 10 ** 6):
        buf, info, passes = prim.plan_bundle_dfs_native(levels, F1, cap=cap)
        assert int(info[4]) == C0 + C1
        if cap < C0 + C1:
            assert len(passes) > 1
        got = _emulate_dfs(bits, buf.numpy(), info, passes)
        # exact supports of the candidate rows of both levels
        want = []
        for pv, pi, eo, ex in levels:
            for g in range(pi.size):
                pre = pv[pi[g]]
                for e in range(eo[g], eo[g + 1]):
                    want.append(int(np.logical_and.reduce(bits[list(pre) + [ex[e]]]).sum()))
        assert np.array_equal(got, np.array(want))
