"""The installable artifact (L4; the reference's Maven jar, pom.xml:53-108): a wheel that
carries both native libraries, installed outside the source tree, runs the CLI (console
entry point module) on the SURVEY §2.7 golden example with byte-identical outputs."""
import glob
import os
import subprocess
import sys
import zipfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

D = "1 2 3\n1 2 4\n2 3 4\n1 2 4\n2 4\n4 5\n1 2\n"
U = "1\n2\n7 8\n2 4\n4 1 2\n3\n1\n"


def test_wheel_installs_and_runs_outside_the_tree(tmp_path):
    # build from a copy of the project files, so the in-tree build's build/ and egg-info
    # land there and not in the checkout
    import shutil
    src = tmp_path / "src"
    src.mkdir()
    for f in ("setup.py", "pyproject.toml", "README.md"):
        shutil.copy(os.path.join(ROOT, f), src / f)
    for d in ("fastapriori_amd", "csrc"):
        shutil.copytree(os.path.join(ROOT, d), src / d, ignore=shutil.ignore_patterns("__pycache__"))
    wh = tmp_path / "wh"
    r = subprocess.run([sys.executable, "-m", "pip", "wheel", str(src), "--no-build-isolation", "--no-deps", "-w",
                        str(wh), "-q"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    whl = glob.glob(str(wh / "fastapriori_amd-*.whl"))
    assert len(whl) == 1 and "none-any" not in whl[0]           # a platform wheel
    names = zipfile.ZipFile(whl[0]).namelist()
    for lib in ("libfa_host.so", "libfa_hip.so"):
        assert any(n.endswith("fastapriori_amd/ops/" + lib) for n in names), lib
    assert any(n.endswith("entry_points.txt") for n in names)
    site = tmp_path / "site"
    r = subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--no-index", "-q", "--target",
                        str(site), whl[0]], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    data = tmp_path / "data"
    data.mkdir()
    (data / "D.dat").write_text(D)
    (data / "U.dat").write_text(U)
    env = dict(os.environ, PYTHONPATH=str(site))
    r = subprocess.run([sys.executable, "-m", "fastapriori_amd", f"{data}/", f"{data}/o_", "--device", "cpu",
                        "--min-support", "0.25"], capture_output=True, text=True, timeout=600, env=env,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    got = (data / "o_freqItemset" / "part-00000").read_text().splitlines()
    assert got == ["1", "1 2", "1 4", "1 4 2", "2", "3", "3 2", "4", "4 2"]
    assert (data / "o_recommends" / "part-00000").read_text().splitlines() == ["2", "1", "0", "1", "3", "2", "2"]
    # the installed copy, not the checkout, was imported
    r = subprocess.run([sys.executable, "-c", "import fastapriori_amd, os; print(os.path.dirname(fastapriori_amd.__file__))"],
                       capture_output=True, text=True, env=env, cwd=str(tmp_path))
    assert r.stdout.strip().startswith(str(site))
