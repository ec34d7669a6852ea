"""Device parser (csrc/hip/parse.hip) against the host parser (csrc/host/parse.cpp)
on the same bytes and byte ranges: line splitting (\\n, \\r\\n, lone \\r, no final
terminator), trim + split, blank lines, duplicate tokens (short lines and lines
with more distinct tokens than the per-thread LDS column), and the fallback to
the host parser for non-canonical or non-numeric tokens."""
import os

import numpy as np
import pytest
import torch

from fastapriori_amd.utils import io

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _same(path, b=0, e=-1):
    got = io.parse_file_device(path, b, e, DEV)
    ref = io.parse_file(path, b, e, 0, "cpu")
    assert got is not None and ref.vocab.numeric
    assert torch.equal(got.offsets.cpu(), ref.offsets)
    assert torch.equal(got.items.cpu(), ref.items)
    assert np.array_equal(got.extras, ref.extras)
    assert got.vocab.size == ref.vocab.size
    return got


def _write(tmp_path, data: bytes, name="D.dat"):
    p = os.path.join(tmp_path, name)
    with open(p, "wb") as f:
        f.write(data)
    return p


@pytest.mark.parametrize("data", [
    b"1 2 3\n4 5\n",
    b"1 2 3\n4 5",                       # no final terminator
    b"1 2\r\n3 4\r\n\r\n5\r",              # CRLF, blank CRLF line, lone CR at EOF
    b"1\r2\r\r3 3 3\n",                  # lone CRs, duplicates
    b"\n\n  \t \n7\n",                   # blank and whitespace-only lines -> token ""
    b"  9\t\t8 \x0b 7\x0c6  \n0 0 2147483646\n",
    b"\x01 5 \x02\n",                    # control bytes trimmed at both ends
    b"",
    b"\n",
])
def test_device_parser_edge_cases(tmp_path, data):
    p = _write(tmp_path, data)
    if data:
        _same(p)


def test_long_lines_with_duplicates(tmp_path):
    rng = np.random.default_rng(3)
    lines = []
    for L in (10, 63, 64, 65, 130, 400):
        toks = rng.integers(0, 300, L)          # many repeats, > 64 distinct in the long ones
        lines.append(" ".join(map(str, toks)))
    p = _write(tmp_path, ("\n".join(lines) + "\n").encode())
    g = _same(p)
    assert g.extras.size > 0


def _same_dict(path, b=0, e=-1):
    """Device dictionary parse vs host dictionary parse: ids differ (slot order vs hash
    order), so compare through the 64-bit token hashes and the decoded strings."""
    got = io.parse_file_device(path, b, e, DEV, force_dict=True)
    ref = io.parse_file(path, b, e, 1, "cpu")
    assert got is not None and not got.vocab.numeric and not ref.vocab.numeric
    assert torch.equal(got.offsets.cpu(), ref.offsets)
    gh, rh = got.vocab.hashes, ref.vocab.hashes
    assert np.array_equal(gh[got.items.cpu().numpy()], rh[ref.items.numpy()])
    assert np.array_equal(gh[got.extras], rh[ref.extras])
    assert got.vocab.size == ref.vocab.size
    gs = dict(zip(gh.tolist(), got.vocab.decode(np.arange(got.vocab.size))))
    rs = dict(zip(rh.tolist(), ref.vocab.decode(np.arange(ref.vocab.size))))
    assert gs == rs
    return got


@pytest.mark.parametrize("data", [b"1 2\n007 3\n", b"1 2\nx y\n", b"1 2147483647\n", b"1 2\x013\n",
                                  b"12345678901\n"])
def test_non_numeric_takes_device_dictionary(tmp_path, data):
    p = _write(tmp_path, data)
    assert not io.parse_file(p, 0, -1, 0, "cpu").vocab.numeric
    got = io.parse_file_device(p, 0, -1, DEV)
    assert got is not None and not got.vocab.numeric
    _same_dict(p)


def test_device_dictionary_random_words(tmp_path):
    rng = np.random.default_rng(7)
    words = [("w%x" % i).encode() for i in range(5000)] + ["é".encode(), "ß".encode(), b"a\x01b", b"0", b""]
    parts = []
    for _ in range(4000):
        L = int(rng.integers(0, 90))
        toks = [words[int(rng.integers(0, len(words) - 1))] for _ in range(L)]   # repeats included
        parts.append(b" ".join(toks) + [b"\n", b"\r\n", b"\r"][int(rng.integers(0, 3))])
    p = _write(tmp_path, b"".join(parts))
    g = _same_dict(p)
    assert g.extras.size > 0 and g.vocab.size > 4000
    size = os.path.getsize(p)
    for b, e in ((0, size // 3), (size // 3, size)):
        _same_dict(p, b, e)


def test_random_files_and_byte_ranges(tmp_path):
    rng = np.random.default_rng(11)
    terms = [b"\n", b"\r\n", b"\r"]
    seps = [b" ", b"\t", b"  ", b" \t "]
    parts = []
    for _ in range(3000):
        L = int(rng.integers(0, 25))
        toks = [str(int(v)).encode() for v in rng.integers(0, 50 if rng.random() < 0.5 else 5000, L)]
        line = b""
        for t in toks:
            line += t + seps[int(rng.integers(0, len(seps)))]
        if rng.random() < 0.2:
            line = b" " + line
        parts.append(line + terms[int(rng.integers(0, len(terms)))])
    data = b"".join(parts)
    p = _write(tmp_path, data)
    _same(p)
    size = len(data)
    cuts = sorted(set([0, size] + [int(x) for x in rng.integers(0, size, 9)]))
    total = 0
    for b, e in zip(cuts[:-1], cuts[1:]):
        total += _same(p, b, e).n_lines
    assert total == io.parse_file(p, 0, -1, 0, "cpu").n_lines


def test_read_shard_uses_device_parser(tmp_path, monkeypatch):
    from fastapriori_amd.parallel.comm import Comm
    p = _write(tmp_path, b"1 2 3\n2 3\n3 4 4\n" * 1000)
    calls = []
    orig = io.parse_file_device
    monkeypatch.setattr(io, "parse_file_device", lambda *a, **k: calls.append(1) or orig(*a, **k))
    sh = io.read_shard(p, Comm(device=DEV), DEV)
    assert calls and sh.items.is_cuda and sh.n_lines == 3000 and sh.extras.size == 1000


def test_lines_longer_than_the_halo_and_tiles(tmp_path):
    # the tile parser stages 2 KB before each 16 KB tile: longer lines read their head
    # from HBM, and a 40 KB line spans whole tiles without a line end
    rng = np.random.default_rng(5)
    lines = [" ".join(map(str, rng.integers(0, 1000, L))) for L in (3, 700, 5, 9000, 2, 1, 1200)]
    p = _write(tmp_path, ("\n".join(lines) + "\n" + "\n".join(lines)).encode())
    g = _same(p)
    assert g.extras.size > 0


def test_parser_histogram_counts_occurrences(tmp_path):
    rng = np.random.default_rng(9)
    lines = [" ".join(map(str, rng.integers(0, 3000, int(rng.integers(0, 40))))) for _ in range(5000)]
    p = _write(tmp_path, ("\n".join(lines) + "\n").encode())
    g = _same(p)
    assert g.hist is not None and g.hist.numel() == g.vocab.size
    want = torch.bincount(g.items.cpu().long(), minlength=g.vocab.size)
    want += torch.bincount(torch.from_numpy(g.extras.astype(np.int64)), minlength=g.vocab.size)
    assert torch.equal(g.hist.cpu(), want)


def test_wide_ids_skip_the_parser_histogram(tmp_path):
    p = _write(tmp_path, b"1 2 3\n9000 2\n")      # id 9001 >= the LDS histogram's 8192 bins
    g = _same(p)
    assert g.hist is None


def test_repeat_buffer_overflow_parses_again(tmp_path):
    p = _write(tmp_path, b"1 1 1 2 2\n" * 40000)   # 120K repeats > the first pass's repeat buffer
    g = _same(p)
    assert g.extras.size == 120000


@pytest.mark.parametrize("slot", [4096, 6000])
def test_streamed_regions_match_host_parser(tmp_path, monkeypatch, slot):
    # small ring slots: the bytes arrive in many chunks, each parsed as its copy lands
    # (lines carried across chunks, a line longer than a chunk, a '\r' in a late chunk
    # that turns the rest into the final region)
    rng = np.random.default_rng(13)
    parts = []
    for i in range(4000):
        L = int(rng.integers(0, 30)) if i != 1500 else 3000
        toks = rng.integers(0, 400, L)
        parts.append(" ".join(map(str, toks)).encode() + (b"\r\n" if i == 3500 else b"\n"))
    data = b"".join(parts)
    monkeypatch.setattr(io, "_RING_SLOT", slot)
    p = _write(tmp_path, data)
    _same(p)
    p2 = _write(tmp_path, data.replace(b"\r\n", b"\n") + b"5 6", name="D2.dat")
    g = _same(p2)
    assert g.hist is not None
    size = len(data)
    total = 0
    for b, e in ((0, size // 3), (size // 3, size)):
        total += _same(p, b, e).n_lines
    assert total == io.parse_file(p, 0, -1, 0, "cpu").n_lines
