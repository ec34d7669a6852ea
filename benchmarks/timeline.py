"""Kernel timeline of one bench step from a rocprofv3 kernel-trace CSV: kernel busy time
vs host gaps, grouped between long gaps.  Used to find fixed (launch / host) costs that
limit strong scaling.

    python benchmarks/timeline.py gpurun_out/kt_small/run_kernel_trace.csv
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--gap-us", type=float, default=50.0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # the last step = kernels from the last F1 kernel that follows a long pause
    marks = [i for i, e in enumerate(ev) if "k_histogram" in e[2] or "k_f1_sketch" in e[2]]
    i0 = marks[0]
    for p, m in zip(marks, marks[1:]):
        if ev[m][0] - ev[p][1] > 5e6:
            i0 = m
    ev = ev[i0:]
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    busy = sum(e[1] - e[0] for e in ev)
    print(f"kernels {len(ev)}  span {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(t1 - t0 - busy) / 1e6:.3f} ms")
    prev_end = t0
    seg = []
    for s, e, n in ev:
        gap = (s - prev_end) / 1e3
        if gap > a.gap_us and seg:
            names = sorted(set(x[2].split('(')[0].split('<')[0][-28:] for x in seg))
            print(f"  [{sum(x[1] - x[0] for x in seg) / 1e3:8.1f} us busy, {len(seg):3d} kernels] {', '.join(names)[:150]}")
            print(f"  -- gap {gap:8.1f} us")
            seg = []
        seg.append((s, e, n))
        prev_end = max(prev_end, e)
    if seg:
        print(f"  [{sum(x[1] - x[0] for x in seg) / 1e3:8.1f} us busy, {len(seg):3d} kernels]")


if __name__ == "__main__":
    main()
