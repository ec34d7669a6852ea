"""List the GPU-idle gaps of the last mining run in a kernel + roctx marker trace, with
the kernel that ends each gap and the innermost host range at its middle.

    python benchmarks/gap_list.py DIR/run_kernel_trace.csv DIR/run_marker_api_trace.csv [min_us]
"""
import csv
import sys


def main():
    kt = list(csv.DictReader(open(sys.argv[1])))
    mk = list(csv.DictReader(open(sys.argv[2])))
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0
    rng = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in mk]
    t0 = max(s for s, e, n in rng if n == "F1")
    ker = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48]) for r in kt)
    ker = [k for k in ker if k[1] >= t0]
    runs = [r for r in rng if r[0] >= t0]

    def inner(t):
        ins = [r for r in runs if r[0] <= t < r[1]]
        return max(ins, key=lambda r: r[0])[2] if ins else "-"
    end, tot = t0, 0.0
    for s, e, n in ker:
        gap = (s - end) / 1e3
        if gap > min_us:
            print(f"{(end - t0) / 1e3:9.1f} us  gap {gap:7.1f} us  before {n:48s} [{inner(end + (s - end) / 2)}]")
        if gap > 0:
            tot += gap
        end = max(end, e)
    print(f"kernels {len(ker)}  idle {tot:.1f} us")


if __name__ == "__main__":
    main()
