"""Attribute GPU idle time of the last mining run to the innermost roctx range.

    python benchmarks/gap_attrib.py gpurun_out/mk12/run_kernel_trace.csv gpurun_out/mk12/run_marker_api_trace.csv

Kernel-trace and marker-trace timestamps share the host clock; the run starts at
the last "F1" range.  For every elementary interval the GPU is busy if any kernel
runs; idle time goes to the innermost open range (latest start), "(none)" outside.
"""
import csv
import sys
from collections import defaultdict


def main():
    kt = list(csv.DictReader(open(sys.argv[1])))
    mk = list(csv.DictReader(open(sys.argv[2])))
    rng = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in mk]
    t0 = max(s for s, e, n in rng if n == "F1")
    runs = [(s, e, n) for s, e, n in rng if s >= t0]
    ker = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt)
    ker = [(s, e) for s, e in ker if e >= t0]
    t1 = max([e for _, e, _ in runs] + [e for _, e in ker])
    pts = sorted(set([t0, t1] + [x for s, e, _ in runs for x in (s, e)] + [max(x, t0) for s, e in ker for x in (s, e)]))
    idle, busy = defaultdict(float), defaultdict(float)
    ki = 0
    active = []
    for a, b in zip(pts[:-1], pts[1:]):
        if b <= a:
            continue
        m = (a + b) / 2
        on = any(s <= m < e for s, e in ker[max(0, ki - 64):ki + 64])
        while ki < len(ker) and ker[ki][1] < a:
            ki += 1
        inner = [r for r in runs if r[0] <= m < r[1]]
        name = max(inner, key=lambda r: r[0])[2] if inner else "(none)"
        name = "level*" if name.startswith("level") else name
        (busy if on else idle)[name] += (b - a) / 1e3
    tot_i, tot_b = sum(idle.values()), sum(busy.values())
    print(f"span {(t1 - t0) / 1e6:.3f} ms  busy {tot_b / 1e3:.3f} ms  idle {tot_i / 1e3:.3f} ms")
    for k in sorted(set(idle) | set(busy), key=lambda k: -idle.get(k, 0)):
        print(f"  {k:12s} idle {idle.get(k, 0) / 1e3:7.3f} ms   busy {busy.get(k, 0) / 1e3:7.3f} ms")


if __name__ == "__main__":
    main()
