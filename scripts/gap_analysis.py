#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of a rocprofv3 --kernel-trace run (csv): total kernel
time, total gap time, and the gaps grouped by (previous kernel class -> next kernel class).
    python3 scripts/gap_analysis.py <rocprof output dir> [top]"""
import collections
import csv
import glob
import os
import sys


def cls(name):
    n = name.replace("void ", "").replace("nk::(anonymous namespace)::", "")
    return n.split("<")[0].split("(")[0]


def main(root, top=15):
    f = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    busy = gap = 0
    by = collections.defaultdict(lambda: [0, 0.0])
    for a, b in zip(rows, rows[1:]):
        s0, e0 = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
        s1 = int(b["Start_Timestamp"])
        busy += e0 - s0
        g = s1 - e0
        if 0 < g < 5_000_000:  # ignore > 5 ms (host work outside the solve: setup, checks)
            gap += g
            k = (cls(a["Kernel_Name"]), cls(b["Kernel_Name"]))
            by[k][0] += 1
            by[k][1] += g
    print(f"kernels {len(rows)}  busy {busy / 1e6:.1f} ms  gaps (<5 ms) {gap / 1e6:.1f} ms")
    for (p, n), (c, t) in sorted(by.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t / 1e6:8.2f} ms {c:6d} x {t / max(c, 1) / 1e3:7.2f} us  {p} -> {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15)
