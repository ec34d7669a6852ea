"""ctypes bindings (fastapriori_amd/ops/_native.py) against the C signatures in csrc/.

ctypes passes arguments beyond a binding's argtypes as C varargs, so a binding that
lags its C function silently truncates pointers (a device fault, not an error).
Every FA_API function's parameter count must equal its binding's."""
import glob
import os
import re

import fastapriori_amd.ops._native as native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c_signatures() -> dict:
    src = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "csrc", "hip", "*.hip")) +
                  glob.glob(os.path.join(ROOT, "csrc", "host", "*.cpp")))
    sigs = {}
    for m in re.finditer(r"FA_API\s+\w+\s+(\w+)\s*\(([^)]*)\)", src, re.S):
        params = [p for p in m.group(2).split(",") if p.strip() and p.strip() != "void"]
        sigs[m.group(1)] = len(params)
    return sigs


def test_binding_arity_matches_c():
    sigs = _c_signatures()
    tables = [v for v in vars(native).values()
              if isinstance(v, dict) and v and all(str(k).startswith("fa_") for k in v)]
    checked = 0
    for t in tables:
        for name, (_, args) in t.items():
            if name in sigs:
                assert sigs[name] == len(args), f"{name}: C has {sigs[name]} parameters, binding {len(args)}"
                checked += 1
    assert checked >= 60
