"""Per-dispatch PMC table of one workload from several rocprofv3 --pmc passes.

    python benchmarks/pmc_table.py gpurun_out/pmc_T40/{a,b,c,d} [--regex k_count_slab] [--first N]

The passes ran the same workload (scripts/gpu_pass.sh pmc), so the matching dispatches
are aligned by their order.  Per dispatch: kernel, LDS busy cycles and their bank-conflict
share, VALU and LDS wave-instructions, LDS-wait share of wave cycles, HBM bytes
(FETCH_SIZE + WRITE_SIZE, KB counters).  --first: only the first N matching dispatches
(one mining run of a multi-run pass).
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def load(d, rx):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return []
    disp = defaultdict(lambda: {"ctr": defaultdict(float)})
    for r in csv.DictReader(open(f[0])):
        name = r.get("Kernel_Name", "")
        if not re.search(rx, name):
            continue
        x = disp[int(r["Dispatch_Id"])]
        x["name"] = name
        x["ctr"][r["Counter_Name"]] += float(r["Counter_Value"])
    return [disp[i] for i in sorted(disp)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--regex", default="k_count_slab")
    ap.add_argument("--first", type=int, default=0)
    a = ap.parse_args()
    runs = [load(d, a.regex) for d in a.dirs]
    n = min(len(r) for r in runs if r) if any(runs) else 0
    if a.first:
        n = min(n, a.first)
    print("| # | kernel | LDS busy cyc | conflict share | VALU inst | LDS inst | LDS wait / wave cyc | HBM MB |")
    print("|---:|---|---:|---:|---:|---:|---:|---:|")
    for i in range(n):
        c = defaultdict(float)
        name = ""
        for r in runs:
            if i < len(r):
                name = r[i]["name"]
                for k, v in r[i]["ctr"].items():
                    c[k] = v
        short = name.split("(")[0].replace("void ", "").replace("fa::", "")[:34]
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
        share = f"{100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.0f} %" if lds else ""
        wait = f"{100 * c.get('SQ_WAIT_INST_LDS', 0) / c['SQ_WAVE_CYCLES']:.0f} %" if c.get("SQ_WAVE_CYCLES") else ""
        hbm = (c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) / 1024.0
        print(f"| {i} | `{short}` | {lds:.3g} | {share} | {c.get('SQ_INSTS_VALU', 0):.3g} | "
              f"{c.get('SQ_INSTS_LDS', 0):.3g} | {wait} | {hbm:.0f} |")


if __name__ == "__main__":
    main()
