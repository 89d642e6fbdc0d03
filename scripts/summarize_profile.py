#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output directory into profiles/<tag>_*.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats, copied as is) and
profiles/<tag>_summary.md: per kernel the rocprof average duration, and the HBM bytes from the
separate FETCH_SIZE / WRITE_SIZE passes, corrected as MI355X_MICROARCH.md prescribes for gfx950
(FETCH_SIZE is reported in KiB and counts exactly half of a 16-B/lane streaming read: x2;
WRITE_SIZE is exact for 16-B/lane streaming stores).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("void ", "").replace("nk::(anonymous namespace)::", "")
    return name.split("(")[0] if not name.startswith("march_kernel") else name.split(">")[0] + ">"


def pmc(path, counter):
    agg = collections.defaultdict(lambda: [0, 0.0])
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += float(r["Counter_Value"])
    return agg


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    fetch = pmc(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    bench = None
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                bench = json.loads(line)
    out = [f"# rocprofv3 summary `{tag}`", "",
           "Command: `scripts/profile.sh` = `rocprofv3 --kernel-trace --stats` over "
           "`python3 bench.py " + (" ".join(sys.argv[2:]) or "--steps 3 --warmup 1 --cpu-baseline off --extra off")
           + "`, then two separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes.", "",
           "| kernel | calls | avg us (rocprof) | % time | HBM read MB/launch (2x FETCH_SIZE) "
           "| HBM write MB/launch |", "|---|---|---|---|---|---|"]
    for r in rows:
        k = short(r["Name"])
        f = fetch.get(k)
        w = write.get(k)
        fr = f"{2 * f[1] / f[0] / 1024:.1f}" if f and f[0] else "-"
        wr = f"{w[1] / w[0] / 1024:.1f}" if w and w[0] else "-"
        out.append(f"| `{k}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                   f"{float(r['Percentage']):.2f} | {fr} | {wr} |")
    if bench:
        out += ["", "Bench line of the traced run (HIP-event kernel timings, same process):", "",
                "```json", json.dumps({k: bench[k] for k in ("value", "ms_per_step", "roofline",
                                                             "jvp_roofline", "kernels")
                                       if k in bench}, indent=1), "```"]
    open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w").write("\n".join(out) + "\n")
    print("\n".join(out))
    # per-kernel-class traffic: the per-dispatch match (scripts/traffic_match.py) of the same run
    tj = os.path.join(ROOT, "profiles", f"{tag}_traffic.json")
    if os.path.exists(tj):
        t = json.load(open(tj))
        extra = ["", "Per-dispatch HBM traffic against algorithmic bytes (`" + os.path.basename(tj)
                 + "`, " + t["source"] + "):", "",
                 "| class | dispatches | traffic / algorithmic | per-dispatch min..max | avg us | "
                 "algorithmic GB/s |", "|---|---|---|---|---|---|"]
        for c, v in sorted(t["classes"].items()):
            extra.append(f"| {c} | {v['dispatches_matched']} | {v['traffic_over_alg']:.4f} | "
                         f"{v['per_dispatch_ratio_min']:.3f}..{v['per_dispatch_ratio_max']:.3f} | "
                         f"{v.get('avg_us', 0):.1f} | {v.get('alg_GBps', 0):.0f} |")
        with open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "a") as fh:
            fh.write("\n".join(extra) + "\n")
        print("\n".join(extra))


if __name__ == "__main__":
    main()
