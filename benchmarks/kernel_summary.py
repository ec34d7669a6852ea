"""Summarise a rocprofv3 run (rocpd .db or kernel_stats.csv) into a compact table.

    python benchmarks/kernel_summary.py gpurun_out/prof/run_results.db [-o profiles/x.md]
"""
import argparse
import csv
import glob
import os
import subprocess
import tempfile


def load_rows(path):
    if path.endswith(".db"):
        d = tempfile.mkdtemp()
        path = os.path.abspath(path)
        subprocess.run(["rocpd2summary", "-i", path, "-f", "csv", "-d", d, "-o", "s"], check=True,
                       capture_output=True, cwd="/tmp")
        path = glob.glob(os.path.join(d, "*kernels_summary.csv"))[0]
    rows = list(csv.DictReader(open(path)))
    out = []
    for r in rows:
        k = {kk.lower(): v for kk, v in r.items()}
        out.append((k["name"], int(k["calls"]), float(k.get("duration (nsec)") or k.get("totaldurationns")),
                    float(k.get("percent (inc)") or k.get("percentage") or 0)))
    out.sort(key=lambda x: -x[2])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("-o", "--out")
    ap.add_argument("-n", type=int, default=30)
    a = ap.parse_args()
    rows = load_rows(a.path)
    total = sum(r[2] for r in rows)
    lines = ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for name, calls, dur, pct in rows[: a.n]:
        short = name.split("(")[0][:80]
        lines.append(f"| `{short}` | {calls} | {dur / 1e6:.3f} | {dur / 1e3 / max(calls, 1):.1f} | {100 * dur / total:.1f} |")
    lines.append(f"| **total GPU kernel time** | {sum(r[1] for r in rows)} | {total / 1e6:.3f} | | 100 |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
