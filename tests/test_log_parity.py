"""The reference's stdout: the exact set and order of its "==== " lines.

Reference format strings: FastApriori.scala:107-108 (level 2), :114 (k candidate
items = candidates.length, i.e. the number of non-empty (prefix, extensions)
groups genCandidates returns, :189-190), :118-119, :127 (total, without the
1-itemsets), :226 (2 candidates items, printed inside genTwoFreqItems);
AssociationRules.scala:155, :177, :181 (per cut level), :75 (rule total);
Main.scala:32, :37 (phase totals).  Millisecond values are masked.
"""
import os
import re
import subprocess
import sys

import pytest

from fastapriori_amd.models import oracle
from fastapriori_amd.utils.jvm import java_split_ws

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GOLDEN_D = "1 2 3\n1 2 4\n2 3 4\n1 2 4\n2 4\n4 5\n1 2\n"
GOLDEN_U = "1\n2\n7 8\n2 4\n4 1 2\n3\n1\n"

# SURVEY §2.7 hand trace at min_support 0.25 (minCount 2): F1 = 4 items, 6 pairs,
# F2 = 4, one level-3 group {0,1} -> [2], F3 = 1 (< 4: the loop stops); 8 level-1
# rules kept, 3 level-2 rules all cut
GOLDEN_LINES = [
    "2 candidates items 6",
    "2 freq items 4",
    "Use Time 2 items #",
    "3 candidate items 1",
    "3 freq items 1",
    "Use Time 3 items #",
    "Total freq items sets 5",
    "Total time for get freqItemsets #",
    "Before cut level 2 Nums: 3",
    "After cut level 2 Nums: 0",
    "Use Time cut leaves 2 Time: #",
    "Size association rules 8",
    "Total time for get recommends #",
]

# items 1..4 always together, 5 and 6 each with 1: level 3 has 3 prefix groups
# ({1,2} -> [3,4], {1,3} -> [4], {2,3} -> [4]) holding 4 candidates, level 4 one group
MULTI_D = "1 2 3 4\n1 2 3 4\n1 2 3 4\n1 5\n1 6\n2 7\n"
MULTI_U = "1\n1 2\n"


def _masked(stdout: str) -> list[str]:
    out = []
    for line in stdout.splitlines():
        if line.startswith("==== "):
            body = line[5:]
            body = re.sub(r"(Use Time \d+ items |Time: |freqItemsets |recommends )\d+$", r"\g<1>#", body)
            out.append(body)
    return out


def _run_cli(tmp_path, d_text, u_text, min_sup, device="cpu", temp=False):
    d = str(tmp_path) + "/"
    with open(d + "D.dat", "w") as f:
        f.write(d_text)
    with open(d + "U.dat", "w") as f:
        f.write(u_text)
    env = {k: v for k, v in os.environ.items() if not k.startswith("FA_")}
    env["PYTHONPATH"] = ROOT
    args = [sys.executable, "-m", "fastapriori_amd", d, d + "out/"]
    if temp:
        os.makedirs(d + "tmp", exist_ok=True)
        args.append(d + "tmp")
    r = subprocess.run(args + ["--min-support", str(min_sup), "--device", device], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return _masked(r.stdout)


def test_golden_log_lines_match_the_reference(tmp_path):
    assert _run_cli(tmp_path, GOLDEN_D, GOLDEN_U, 0.25) == GOLDEN_LINES


def _mining_part(lines: list[str]) -> list[str]:
    return lines[:lines.index(next(l for l in lines if l.startswith("Total freq items sets"))) + 1]


def _expected(d_text: str, min_sup: float) -> list[str]:
    # the reference loop replayed from the oracle's itemsets (models/oracle.mining_log_lines)
    res = oracle.mine([java_split_ws(l) for l in d_text.splitlines()], min_sup)
    return oracle.mining_log_lines(len(res.items), res.itemsets)


# the loop's edges (FastApriori.scala:111-119):
# STOP_D: F_4 = 4 rows < 5, so the reference never enters level 5 (no level-5 lines,
# even though a bundle may count level 5 speculatively)
STOP_D = "1 2 3 4\n1 2 3 5\n1 2 4 5\n1 3 4 5\n" * 2
# NOCAND_D: F_2 = 3 disjoint pairs (3 >= 3), so level 3 is entered with no candidates
# and prints all three lines
NOCAND_D = "1 2\n1 2\n3 4\n3 4\n5 6\n5 6\n"
EDGE_CASES = [(STOP_D, 0.25, ["3 candidate items 6", "3 freq items 10", "Use Time 3 items #",
                               "4 candidate items 4", "4 freq items 4", "Use Time 4 items #"]),
              (NOCAND_D, 0.3, ["3 candidate items 0", "3 freq items 0", "Use Time 3 items #"])]


def test_candidate_line_counts_prefix_groups(tmp_path):
    lines = _mining_part(_run_cli(tmp_path, MULTI_D, MULTI_U, 0.5))
    assert "3 candidate items 3" in lines          # 3 groups (4 candidates)
    assert lines == _expected(MULTI_D, 0.5)


@pytest.mark.parametrize("case", range(len(EDGE_CASES)))
def test_loop_edges_match_the_reference(tmp_path, case):
    d, sup, levels = EDGE_CASES[case]
    lines = _mining_part(_run_cli(tmp_path, d, "1\n", sup))
    assert lines == _expected(d, sup)
    assert [l for l in lines if not l.startswith(("2 ", "Use Time 2", "Total"))] == levels


@pytest.mark.gpu
def test_golden_log_lines_on_gpu_with_temp(tmp_path):
    # the CLI's three-argument form (checkpointing on) through the device path
    assert _run_cli(tmp_path, GOLDEN_D, GOLDEN_U, 0.25, device="cuda", temp=True) == GOLDEN_LINES


@pytest.mark.gpu
def test_candidate_line_counts_prefix_groups_on_gpu(tmp_path):
    lines = _run_cli(tmp_path, MULTI_D, MULTI_U, 0.5, device="cuda", temp=True)
    assert _mining_part(lines) == _expected(MULTI_D, 0.5)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(EDGE_CASES)))
def test_loop_edges_match_the_reference_on_gpu(tmp_path, case):
    # the device level loop (bundles with speculative levels, device stop test)
    d, sup, levels = EDGE_CASES[case]
    for temp in (False, True):
        sub = tmp_path / f"t{int(temp)}"
        sub.mkdir()
        lines = _mining_part(_run_cli(sub, d, "1\n", sup, device="cuda", temp=temp))
        assert lines == _expected(d, sup), (temp, lines)
