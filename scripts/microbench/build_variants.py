"""Build kernel-variant copies of libfa_hip.so for A/B timing runs (FA_HIP_LIB=...).
    python scripts/microbench/build_variants.py NAME=-DMACRO[,-DMACRO2] ...
Each variant is the tree's HIP sources with extra -D flags, written to
scripts/microbench/var/libfa_hip_NAME.so (git-ignored; travels with gpurun)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fastapriori_amd.ops import build as b  # noqa: E402

out_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "var")
os.makedirs(out_dir, exist_ok=True)
for spec in sys.argv[1:]:
    name, _, defs = spec.partition("=")
    out = os.path.join(out_dir, f"libfa_hip_{name}.so")
    b._build(out, [b._hipcc()], b.hip_sources(), b.HIP_FLAGS + [d for d in defs.split(",") if d],
             b.source_id("hip"))
    print("built", out)
