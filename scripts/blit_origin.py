#!/usr/bin/env python3
"""For a rocprofv3 run with --kernel-trace --hip-trace (csv): the HIP API calls whose correlation
id matches each runtime blit kernel (__amd_rocclr_*), counted, plus the API call stats."""
import collections
import csv
import glob
import os
import sys


def find(root, suffix):
    hits = glob.glob(os.path.join(root, "**", "*" + suffix), recursive=True)
    return hits[0] if hits else None


def main(root):
    kt, ht = find(root, "kernel_trace.csv"), find(root, "hip_api_trace.csv")
    if not kt or not ht:
        print("missing traces", kt, ht)
        return
    api = {}
    with open(ht) as f:
        for r in csv.DictReader(f):
            api[r["Correlation_Id"]] = r["Function"]
    blits = collections.Counter()
    for r in csv.DictReader(open(kt)):
        name = r["Kernel_Name"]
        if "__amd_rocclr" in name:
            blits[(name, api.get(r["Correlation_Id"], "?"))] += 1
    for (k, fn), c in blits.most_common():
        print(f"{c:6d}  {k:40s} <- {fn}")
    calls = collections.Counter(api.values())
    print("\nHIP API calls:")
    for fn, c in calls.most_common(40):
        print(f"{c:8d}  {fn}")


if __name__ == "__main__":
    main(sys.argv[1])
