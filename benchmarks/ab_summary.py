"""Summarise scripts/gpu_cycle.sh A/B runs: ms per step of each variant and config.

    python benchmarks/ab_summary.py gpurun_out/cy
"""
import glob
import json
import sys
from collections import defaultdict


def main():
    pre = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/cy"
    res = defaultdict(list)
    for f in sorted(glob.glob(pre + "_*.json")):
        parts = f[len(pre) + 1:-5].split("_")
        if len(parts) < 3:
            continue
        cfg, val = parts[0], "_".join(parts[1:-1])
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
            res[(cfg, val)].append(d["ms_per_step"])
        except Exception as e:        # a failed run: show why
            res[(cfg, val)].append(f"err:{type(e).__name__}")
    for (cfg, val), xs in sorted(res.items()):
        print(f"{cfg:5s} {val:>6s}  {xs}")


if __name__ == "__main__":
    main()
