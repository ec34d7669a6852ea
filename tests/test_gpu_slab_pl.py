"""Lane-pair slab kernel (csrc/hip/count.hip k_count_slab_pl: unpadded 256-B rows,
two lanes per piece, conflict-free LDS reads) against the padded record kernel
(k_count_slab_rec) and the C++ CPU miner: identical itemsets and counts.

Covers the three slab builds (rows -> LDS, dedup columns, copies from the used-item
bitmap on multi-pass levels), unit and weighted layouts (weight-uniform and mixed
slabs), the device-resident bundles and the host level loop.
Reference semantics: FastApriori.scala:143-154.
"""
import numpy as np
import pytest
import torch

import fastapriori_amd.models.apriori as ap
import fastapriori_amd.ops.primitives as prim
from fastapriori_amd import ops
from fastapriori_amd.models.apriori import FastApriori, MinerConfig
from fastapriori_amd.ops.host import apriori_gen
from fastapriori_amd.parallel.comm import Comm
from fastapriori_amd.utils.io import generate_shard
from fastapriori_amd.utils.metrics import Logger

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _spy(monkeypatch):
    calls = []
    real = prim._hip_call

    def rec(name, *a):
        calls.append(name)
        return real(name, *a)
    monkeypatch.setattr(prim, "_hip_call", rec)
    return calls


def _mine(shard, ms, **kw):
    return FastApriori(ms, config=MinerConfig(min_support=ms, **kw), logger=Logger(0, enabled=False)).run(shard)


@pytest.mark.parametrize("device_levels", [True, False])
@pytest.mark.parametrize("dedup", ["off", "on"])
def test_pl_mining_matches_padded_and_cpu(monkeypatch, device_levels, dedup):
    cpu = generate_shard(200_000, Comm(), "cpu", 10.0, 4.0, 2000, 1000, 5)
    ref = _mine(cpu, 0.002, dedup="off")
    g = cpu.to(DEV)
    monkeypatch.setattr(ap, "DEVICE_LEVELS", device_levels)
    monkeypatch.setattr(prim, "SLAB_PL_MIN_CAP", 0)
    pad = _mine(g, 0.002, dedup=dedup)
    monkeypatch.setattr(prim, "SLAB_PL_MIN_CAP", 1024)
    calls = _spy(monkeypatch)
    got = _mine(g, 0.002, dedup=dedup)
    assert "fa_hip_count_slab_pl" in calls
    assert got.as_dict() == pad.as_dict() == ref.as_dict()
    for x, y in zip(got.levels, pad.levels):
        assert np.array_equal(x, y)


def test_pl_multipass_from_bitmap(monkeypatch):
    # small LDS budget: several accumulator passes, slabs copied from the used items' bitmap
    cpu = generate_shard(60_000, Comm(), "cpu", 14.0, 6.0, 300, 120, 11)
    ref = _mine(cpu, 0.004, trim_min_rows=0, dedup="off")
    monkeypatch.setattr(prim, "_LDS_BYTES", 64 * 1024)
    monkeypatch.setattr(prim, "SLAB_PL_MIN_CAP", 1024)
    monkeypatch.setattr(ap, "DEVICE_LEVELS", False)
    calls = _spy(monkeypatch)
    got = _mine(cpu.to(DEV), 0.004, trim_min_rows=0, dedup="off")
    assert "fa_hip_count_slab_pl" in calls
    assert got.as_dict() == ref.as_dict()
    got_w = _mine(cpu.to(DEV), 0.004, trim_min_rows=0, dedup="on")
    assert got_w.as_dict() == ref.as_dict()


@pytest.mark.parametrize("n,V,frac", [(70_001, 300, 0.8), (4097, 120, 1.0), (9000, 900, 0.5)])
def test_pl_count_level_edges(monkeypatch, n, V, frac):
    # column counts ending inside a slab word and inside a 2048-column slab; the padded
    # record kernel, the lane-pair kernel and the CPU bitmap counts must agree
    from test_gpu_kernels import _compress_inputs, _prep
    off, items, lut, F1 = _prep(n=n, V=V, max_len=14, seed=n % 97, long_rows=3, F1_frac=frac)
    _, kept, roff = _compress_inputs(off, items, lut)
    ranks = ops.compress(off, items, lut, kept, roff)
    T = kept.numel()
    bm, W = ops.build_bitmaps(roff, ranks, None, T, F1)
    ph = ops.pair_counts_horizontal(roff, ranks, None, F1)
    iu = torch.triu_indices(F1, F1, 1)
    pc = ph[iu[0], iu[1]]
    sel = torch.nonzero(pc >= max(1, int(pc.float().quantile(0.8).item()))).flatten()
    prev = torch.stack([iu[0][sel], iu[1][sel]], 1).numpy().astype(np.int32)
    pidx, eoff, ext = apriori_gen(prev)
    assert ext.size > 0
    ref = ops.count_candidates(bm, W, torch.from_numpy(prev[pidx].copy()), eoff, torch.from_numpy(ext.copy()), None)
    g = dict(roff=roff.to(DEV), ranks=ranks.to(DEV))
    monkeypatch.setattr(prim, "SLAB_PL_MIN_CAP", 0)
    a = ops.count_level(g["roff"], g["ranks"], None, T, F1, prev[pidx], eoff, ext, None, kernel="slab")
    assert prim.LAST_LEVEL_PLAN["kernel"] == "slab"
    monkeypatch.setattr(prim, "SLAB_PL_MIN_CAP", 1024)
    b = ops.count_level(g["roff"], g["ranks"], None, T, F1, prev[pidx], eoff, ext, None, kernel="slab")
    assert prim.LAST_LEVEL_PLAN["kernel"] == "slab_pl"
    assert torch.equal(ref, a.cpu()) and torch.equal(ref, b.cpu())
