"""Native parser vs a pure-Python statement of the reference's input semantics.

Utils.scala:21-23: textFile (Hadoop LineRecordReader: \\n, \\r\\n, \\r) then
``trim().split("\\\\s+")``; an empty line is the single token "".
"""
import random

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from fastapriori_amd.models.data import Vocabulary
from fastapriori_amd.ops import _native
from fastapriori_amd.utils.io import parse_bytes
from fastapriori_amd.utils.jvm import java_split_ws, split_lines


def decode(shard):
    off = shard.offsets.numpy()
    items = shard.items.numpy()
    rows = []
    for i in range(shard.n_lines):
        rows.append([shard.vocab.token(int(t)) for t in items[off[i]:off[i + 1]]])
    extras = [shard.vocab.token(int(t)) for t in shard.extras]
    return rows, extras


def expected(text: str):
    rows, extras = [], []
    for line in split_lines(text):
        toks = java_split_ws(line)
        seen, row = set(), []
        for t in toks:
            if t in seen:
                extras.append(t)
            else:
                seen.add(t)
                row.append(t)
        rows.append(row)
    return rows, extras


CASES = [
    "1 2 3\n4 5\n",
    "1 2 3\n4 5",                      # no trailing newline
    "",                                 # empty file
    "\n\n",                             # blank lines -> token ""
    "  7\t 8 \r\n9\r10\n",              # CRLF, lone CR, tabs, padding
    "1 1 2 1\n2 2\n",                   # duplicate tokens -> extras
    "a b\nc  a\n\nb\x0bc\x0cd\n",       # dictionary mode, \x0b \x0c separators
    "01 1 +1 -1\n",                     # non-canonical numerics are distinct tokens
    "x\x01y z\n",                       # \x01 is not a separator (but is trimmed at ends)
    "héllo wörld héllo\n",              # utf-8
]


@pytest.mark.parametrize("text", CASES)
def test_parse_cases(text):
    sh = parse_bytes(text.encode("utf-8"))
    got_rows, got_extras = decode(sh)
    exp_rows, exp_extras = expected(text)
    assert got_rows == exp_rows
    assert sorted(got_extras) == sorted(exp_extras)


def test_numeric_mode_ids():
    sh = parse_bytes(b"0 5\n\n2147483646\n")
    assert sh.vocab.numeric
    assert Vocabulary.numeric_id("5") == 6 and Vocabulary.numeric_id("") == 0
    assert Vocabulary.numeric_id("05") == -1
    sh2 = parse_bytes(b"2147483647\n")          # beyond the numeric id range -> dict mode
    assert not sh2.vocab.numeric


alphabet = st.sampled_from(list("0123456789ab \t\n\r\x0b"))


@settings(max_examples=150, deadline=None)
@given(st.text(alphabet=alphabet, max_size=200))
def test_parse_random(text):
    sh = parse_bytes(text.encode())
    got_rows, got_extras = decode(sh)
    exp_rows, exp_extras = expected(text)
    assert got_rows == exp_rows
    assert sorted(got_extras) == sorted(exp_extras)


def test_byte_range_shards_partition_lines(tmp_path):
    rng = random.Random(0)
    lines = [" ".join(str(rng.randint(0, 50)) for _ in range(rng.randint(0, 8))) for _ in range(500)]
    seps = ["\n", "\r\n", "\r"]
    text = "".join(l + rng.choice(seps) for l in lines)
    p = tmp_path / "D.dat"
    p.write_bytes(text.encode())
    from fastapriori_amd.utils.io import parse_file
    size = len(text.encode())
    full = decode(parse_file(str(p)))[0]
    for W in (2, 3, 7, 16):
        rows = []
        for r in range(W):
            rows += decode(parse_file(str(p), size * r // W, size * (r + 1) // W))[0]
        assert rows == full


def test_next_line_start():
    lib = _native.host()
    d = b"ab\r\ncd\ref\n"
    assert lib.fa_next_line_start(d, len(d), 0) == 0
    assert lib.fa_next_line_start(d, len(d), 3) == 4     # inside CRLF
    assert lib.fa_next_line_start(d, len(d), 4) == 4
    assert lib.fa_next_line_start(d, len(d), 6) == 7     # after lone CR
    assert lib.fa_next_line_start(d, len(d), 10) == 10


def test_many_threads_consistent(monkeypatch):
    rng = np.random.default_rng(1)
    text = "\n".join(" ".join(map(str, rng.integers(0, 100, rng.integers(1, 12)))) for _ in range(20000))
    monkeypatch.setenv("FA_NUM_THREADS", "1")
    a = parse_bytes(text.encode())
    monkeypatch.setenv("FA_NUM_THREADS", "8")
    b = parse_bytes(text.encode())
    assert a.offsets.equal(b.offsets) and a.items.equal(b.items)
