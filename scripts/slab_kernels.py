#!/usr/bin/env python3
"""Per-instantiation view of the fused Arnoldi kernel on one grid height: rocprofv3 kernel-trace
average duration, fraction of 8 TB/s for its algorithmic bytes 8 (nv + 4 [+1 with z]) ny nx, and
the HBM traffic from separate --pmc FETCH_SIZE / WRITE_SIZE passes (gfx950 corrections of
MI355X_MICROARCH.md: FETCH_SIZE in KiB counts half of a 16-B/lane streaming read -> x2 KiB;
WRITE_SIZE in KiB is exact).
    python3 scripts/slab_kernels.py <stats.csv> <fetch.csv|-> <write.csv|-> <ny> [nx]"""
import collections
import csv
import re
import sys

PEAK = 8000.0  # GB/s


def key(name):
    m = re.search(r"(arnoldi(?:_wide)?_kernel)<(\d+), (true|false),[^>]*>", name)
    if not m:
        return None
    return (m.group(1), int(m.group(2)), m.group(3) == "true")


def pmc(path, counter):
    agg = collections.defaultdict(lambda: [0, 0.0])
    if path == "-":
        return agg
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        k = key(r["Kernel_Name"])
        if k:
            agg[k][0] += 1
            agg[k][1] += float(r["Counter_Value"])
    return agg


def main():
    stats, fpath, wpath, ny = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    nx = int(sys.argv[5]) if len(sys.argv) > 5 else 4096
    fetch, write = pmc(fpath, "FETCH_SIZE"), pmc(wpath, "WRITE_SIZE")
    rows = []
    tot_t = tot_b = 0.0
    for r in csv.DictReader(open(stats)):
        k = key(r["Name"])
        if not k:
            continue
        kind, nv, ext = k
        alg = 8.0 * (nv + 4 + (1 if ext else 0)) * ny * nx
        calls, avg = int(r["Calls"]), float(r["AverageNs"]) / 1e3
        tot_t += calls * avg
        tot_b += calls * alg
        f, w = fetch.get(k), write.get(k)
        hbm = None
        if f and w and f[0] and w[0]:
            hbm = (2.0 * f[1] / f[0] + w[1] / w[0]) * 1024.0
        rows.append((kind, nv, ext, calls, avg, alg / (avg * 1e-6) / 1e9 / PEAK,
                     hbm / alg if hbm else None))
    rows.sort(key=lambda t: (t[2], t[1]))
    print(f"ny={ny} nx={nx}")
    print("kernel nv ext calls avg_us frac traffic")
    for kind, nv, ext, calls, avg, frac, tr in rows:
        trs = f"{tr:.3f}" if tr else "-"
        print(f"{kind} {nv} {int(ext)} {calls} {avg:.1f} {frac:.3f} {trs}")
    if tot_t:
        print(f"aggregate frac {tot_b / (tot_t * 1e-6) / 1e9 / PEAK:.3f} over {tot_t / 1e3:.1f} ms")


if __name__ == "__main__":
    main()
