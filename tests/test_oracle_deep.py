"""Parity at depth against the independent oracle: a 20K-row Quest database with 14
levels at min_support 2 %, mined by the CLI (the three-argument form, checkpointing
on; on the GPU through the device level bundles), must reproduce byte for byte the
freqItemset and recommends files of the brute-force Python oracle
(fastapriori_amd/models/oracle.py), whose answer tests/fixtures/oracle_q20k.json
holds (tests/fixtures/make_oracle_fixture.py regenerates it)."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "fixtures", "oracle_q20k.json")


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_deep_database_matches_the_oracle_byte_for_byte(tmp_path, device):
    sys.path.insert(0, os.path.join(ROOT, "tests", "fixtures"))
    from make_oracle_fixture import write_inputs
    want = json.load(open(FIX))
    d = str(tmp_path) + "/"
    write_inputs(d)
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "fastapriori_amd", d, d + "o_", d + "tmp", "--min-support",
                        str(want["min_support"]), "--device", device, "--metrics", d + "m.jsonl"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    freq = open(d + "o_freqItemset/part-00000", "rb").read()
    rec = open(d + "o_recommends/part-00000", "rb").read()
    assert hashlib.sha256(freq).hexdigest() == want["freqItemset_sha256"]
    assert hashlib.sha256(rec).hexdigest() == want["recommends_sha256"]
    assert len(freq.splitlines()) == want["n_itemsets"] and max(int(k) for k in want["levels"]) >= 14
    job = [json.loads(l) for l in open(d + "m.jsonl") if '"phase": "job"' in l][-1]
    assert job["device_bundles"] > 0 or device == "cpu"
