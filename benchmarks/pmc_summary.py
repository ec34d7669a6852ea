"""Summarise rocprofv3 --pmc counter CSVs into a per-kernel markdown table.

    python benchmarks/pmc_summary.py gpurun_out/pmc/r3_a [gpurun_out/pmc/r3_b ...]

Counters are summed over every dispatch of a kernel (all runs in the trace) and divided
by the number of mining runs given with --runs.  "conflict share" =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (the LDS cycles spent on bank conflicts).
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    acc = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        name = r.get("Kernel_Name", "")
        ctr = r.get("Counter_Name", "")
        try:
            acc[name][ctr] += float(r.get("Counter_Value", 0))
        except ValueError:
            pass
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--runs", type=float, default=1.0)
    a = ap.parse_args()
    tot = defaultdict(dict)
    for d in a.dirs:
        for k, v in load(d).items():
            tot[k].update(v)
    cols = sorted({c for v in tot.values() for c in v})
    short = lambda n: n.split("(")[0].replace("void ", "")[:48]   # noqa: E731
    print("| kernel | " + " | ".join(cols) + " | conflict share |")
    print("|---|" + "---:|" * (len(cols) + 1))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_LDS_IDX_ACTIVE", 0)):
        share = ""
        if v.get("SQ_LDS_IDX_ACTIVE"):
            share = f"{100 * v.get('SQ_LDS_BANK_CONFLICT', 0) / v['SQ_LDS_IDX_ACTIVE']:.0f} %"
        print(f"| `{short(k)}` | " + " | ".join(f"{v.get(c, 0) / a.runs:.3g}" for c in cols) + f" | {share} |")


if __name__ == "__main__":
    main()
