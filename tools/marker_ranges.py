#!/usr/bin/env python3
"""Per-range wall and kernel time of the last ``oni:flow.run`` (one bench day) in rocprofv3
marker + kernel traces, side by side for several runs (e.g. world 1 vs a forced 1-rank group).

  python tools/marker_ranges.py w1=gpurun_out/x5/mprof_1 fd=gpurun_out/x4c/mprof_2 > profiles/r5/dp1_ranges.txt

Kernel time of a range = Σ durations of the kernels that start and end inside it (ms).
"""
from __future__ import annotations

import csv
import os
import sys


def ranges(d: str, top: str = "oni:flow.run") -> dict:
    marks = list(csv.DictReader(open(os.path.join(d, "run_marker_api_trace.csv"))))
    kern = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"])) for k in kern)
    day = [m for m in marks if m["Function"] == top][-1]
    t0, t1 = int(day["Start_Timestamp"]), int(day["End_Timestamp"])
    out: dict = {}
    for m in marks:
        a, b = int(m["Start_Timestamp"]), int(m["End_Timestamp"])
        if a < t0 or b > t1:
            continue
        kt = sum(e - s for s, e in ks if s >= a and e <= b)
        w, k = out.get(m["Function"], (0.0, 0.0))
        out[m["Function"]] = (w + (b - a) / 1e6, k + kt / 1e6)
    return out


def main() -> int:
    runs = [a.split("=", 1) for a in sys.argv[1:]]
    data = [(name, ranges(d)) for name, d in runs]
    names = sorted(set().union(*[set(r) for _, r in data]), key=lambda n: -max(r.get(n, (0, 0))[0] for _, r in data))
    print("range".ljust(32) + " | ".join(f"{n:>8s} wall {n:>8s} kern" for n, _ in data))
    for n in names:
        cells = []
        for _, r in data:
            w, k = r.get(n, (0.0, 0.0))
            cells.append(f"{w:13.3f} {k:13.3f}")
        print(n[:31].ljust(32) + " | ".join(cells))
    return 0


if __name__ == "__main__":
    sys.exit(main())
