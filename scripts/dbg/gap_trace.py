"""Kernel durations and the gaps between consecutive kernels from a rocprofv3 kernel trace
(trace_kernel_trace.csv): per class (fused Arnoldi, control / reduction, other) the mean device
duration, and per (previous class -> next class) pair the mean idle gap between one kernel's end
and the next one's start on the queue.  Tells the device time of a launch apart from what an
event pair around it also holds.
    python3 scripts/dbg/gap_trace.py <trace_kernel_trace.csv> [--skip N]"""
import csv
import sys
from collections import defaultdict


def cls(name):
    if "arnoldi_kernel" in name or "arnoldi_wide_kernel" in name:
        return "fused"
    if "arn_reduce" in name or "arn_ctl" in name:
        return "ctl"
    if "reduce_final" in name:
        return "reduce_final"
    return "other"


rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else len(rows) // 4
rows = rows[skip:]
dur = defaultdict(list)
gap = defaultdict(list)
for i, (s, e, n) in enumerate(rows):
    dur[cls(n)].append((e - s) / 1e3)
    if i + 1 < len(rows):
        g = (rows[i + 1][0] - e) / 1e3
        if g < 200:  # host waits longer than this are not launch boundaries
            gap[(cls(n), cls(rows[i + 1][2]))].append(g)
for k, v in sorted(dur.items()):
    print(f"dur  {k:14s} n={len(v):5d} mean={sum(v) / len(v):8.2f} us")
for k, v in sorted(gap.items()):
    print(f"gap  {k[0]:>12s} -> {k[1]:12s} n={len(v):5d} mean={sum(v) / len(v):7.2f} us "
          f"min={min(v):6.2f}")
