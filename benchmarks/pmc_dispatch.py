"""Per-dispatch PMC comparison of two runs of the same workload (scripts/gpu_pmc_ab.sh).

    python benchmarks/pmc_dispatch.py gpurun_out/pmcab/0_a gpurun_out/pmcab/1_a [--b gpurun_out/pmcab/0_b gpurun_out/pmcab/1_b]

Dispatches of the traced kernels are taken in order and aligned by index (both runs
launch the same levels and passes); prints, per dispatch, the kernel, its duration
(when a kernel trace was taken with the counters) and LDS / VALU counters of A and B.
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    disp = defaultdict(lambda: {"ctr": defaultdict(float)})
    for r in csv.DictReader(open(f[0])):
        x = disp[int(r["Dispatch_Id"])]
        x["name"] = r.get("Kernel_Name", "")
        x["ctr"][r["Counter_Name"]] += float(r["Counter_Value"])
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if kt:
        for r in csv.DictReader(open(kt[0])):
            i = int(r["Dispatch_Id"])
            if i in disp:
                disp[i]["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return [disp[i] for i in sorted(disp)]


def short(n):
    return n.split("(")[0].replace("void fa::k_count_slab_rec", "rec")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--b2", nargs=2, default=None, help="second counter pass of A and B")
    args = ap.parse_args()
    A, B = load(args.a), load(args.b)
    if args.b2:
        for run, d in zip((A, B), args.b2):
            for x, y in zip(run, load(d)):
                for k, v in y["ctr"].items():
                    x["ctr"].setdefault(k, v)
    n = min(len(A), len(B))
    cols = ["SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VALU", "SQ_WAIT_INST_LDS",
            "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"]
    print(f"{len(A)} / {len(B)} dispatches")
    print("| # | kernel A | kernel B | us A | us B | " + " | ".join(f"{c[3:]} B/A" for c in cols) + " |")
    print("|---" * (5 + len(cols)) + "|")
    for i in range(n):
        a, b = A[i], B[i]
        r = []
        for c in cols:
            va, vb = a["ctr"].get(c), b["ctr"].get(c)
            r.append(f"{vb / va:.2f}" if va and vb is not None else "-")
        print(f"| {i} | {short(a['name'])} | {short(b['name'])} | {a.get('us', 0):.0f} | {b.get('us', 0):.0f} | "
              + " | ".join(r) + " |")


if __name__ == "__main__":
    main()
