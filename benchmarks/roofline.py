"""Roofline lines of the hot kernels from rocprofv3 output (docs/PERF.md).

    python benchmarks/roofline.py --stats gpurun_out/kernels/T10 --pmc gpurun_out/pmc/a gpurun_out/pmc/b \
        gpurun_out/pmc/c --runs 2 --stat-runs 2 [--top 8]

--stats: a `rocprofv3 --kernel-trace --stats` output directory (kernel time; its run
count --stat-runs); --pmc: `--pmc` pass directories of the same workload (counters
summed over dispatches, divided by --runs).  Per kernel it prints the time per run and,
against the MI355X peaks (MI355X_MICROARCH.md: 256 CUs at 2.4 GHz, a wave64 VALU
instruction issued over 2 cycles per SIMD -> 1.23e12 wave-instructions/s; HBM 8.0 TB/s
spec, 6.29 TB/s measured by a float4 copy; ds_read_b128 ~150 TB/s aggregate):
  VALU  = SQ_INSTS_VALU / time, and its share of the VALU issue peak;
  LDS   = SQ_INSTS_LDS / time (wave-instructions);
  HBM   = (FETCH_SIZE + WRITE_SIZE) / time, and its share of the measured copy rate;
  busy  = SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_ANY (the share of issue cycles that are VALU).
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

VALU_PEAK = 256 * 4 * 2.4e9 / 2        # wave64 VALU instructions per second (4 SIMDs, 2 cycles each)
HBM_MEASURED = 6.29e12
HBM_SPEC = 8.0e12


def short(n: str) -> str:
    return n.split("(")[0].replace("void ", "").replace("fa::", "")[:44]


def load_stats(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    out = {}
    for r in csv.DictReader(open(f[0])):
        out[r["Name"]] = float(r["TotalDurationNs"]) / 1e6
    return out


def load_pmc(dirs):
    acc = defaultdict(lambda: defaultdict(float))
    for d in dirs:
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        for r in csv.DictReader(open(f[0])):
            try:
                acc[r.get("Kernel_Name", "")][r.get("Counter_Name", "")] += float(r.get("Counter_Value", 0))
            except ValueError:
                pass
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--runs", type=float, default=1.0, help="mining runs in each PMC pass")
    ap.add_argument("--stat-runs", type=float, default=1.0, help="mining runs in the kernel-stats trace")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    ms = {k: v / a.stat_runs for k, v in load_stats(a.stats).items()}
    pmc = {k: {c: x / a.runs for c, x in v.items()} for k, v in load_pmc(a.pmc).items()}
    print("| kernel | ms / run | VALU inst/s | % VALU peak | VALU issue share | LDS inst/s | HBM GB/s "
          "| % of 6.29 TB/s |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for name, t in sorted(ms.items(), key=lambda kv: -kv[1])[:a.top]:
        p = pmc.get(name, {})
        s = t / 1e3
        cells = [f"`{short(name)}`", f"{t:.2f}"]
        if "SQ_INSTS_VALU" in p and s > 0:
            v = p["SQ_INSTS_VALU"] / s
            cells += [f"{v:.3g}", f"{100 * v / VALU_PEAK:.0f} %"]
        else:
            cells += ["", ""]
        if p.get("SQ_ACTIVE_INST_ANY"):
            cells.append(f"{100 * p.get('SQ_ACTIVE_INST_VALU', 0) / p['SQ_ACTIVE_INST_ANY']:.0f} %")
        else:
            cells.append("")
        cells.append(f"{p['SQ_INSTS_LDS'] / s:.3g}" if "SQ_INSTS_LDS" in p and s > 0 else "")
        if ("FETCH_SIZE" in p or "WRITE_SIZE" in p) and s > 0:
            b = (p.get("FETCH_SIZE", 0) + p.get("WRITE_SIZE", 0)) * 1024.0 / s     # counters in KB
            cells += [f"{b / 1e9:.0f}", f"{100 * b / HBM_MEASURED:.0f} %"]
        else:
            cells += ["", ""]
        print("| " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
