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
           "`python3 bench.py " + (" ".join(sys.argv[2:]) or "--steps 3 --warmup 0 --cpu-baseline off")
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
    # per-kernel-class HBM traffic per launch (PMC) next to the algorithmic bytes of the SAME run;
    # a class sums every instantiation of its kernel template (arnoldi_kernel<nv, ext, pf, nt>)
    def klass(k):
        if k.startswith("arnoldi_kernel<"):
            return "arnoldi_fused"
        if k.startswith("arnoldi_edge_kernel"):
            return "arnoldi_edge"
        if k.startswith("combo_kernel<"):
            return "krylov_combo"
        if k.startswith("mdot_kernel<"):
            return "krylov_mdot"
        if k.startswith("reduce_final_kernel"):
            return "reduce_final"
        for mode, cls in (("5", "sh_fdjvp"), ("6", "sh_ajvp"), ("4", "sh_trial"), ("3", "sh_bold")):
            if k.startswith(f"march_kernel<(nk::SMode){mode},"):
                return cls
        return None

    def by_class(agg):
        out = collections.defaultdict(lambda: [0, 0.0])
        for k, (n, v) in agg.items():
            c = klass(k)
            if c:
                out[c][0] += n
                out[c][1] += v
        return out

    fc, wc = by_class(fetch), by_class(write)
    traffic = {"tag": tag, "source": f"profiles/{tag}_summary.md", "classes": {}}
    for cls in sorted(fc):
        f, w = fc[cls], wc.get(cls)
        if not w or not f[0] or not w[0]:
            continue
        rec = {"launches": f[0], "hbm_read_bytes_per_launch": 2 * f[1] * 1024 / f[0],
               "hbm_write_bytes_per_launch": w[1] * 1024 / w[0]}
        if bench and cls in bench.get("kernels", {}):
            kb = bench["kernels"][cls]
            alg = (kb["alg_MB_per_launch"] * 1e6 if "alg_MB_per_launch" in kb
                   else kb["GB/s"] * 1e9 * kb["ms"] * 1e-3 / kb["launches"])
            rec["alg_bytes_per_launch"] = alg
            rec["traffic_over_alg"] = (rec["hbm_read_bytes_per_launch"]
                                       + rec["hbm_write_bytes_per_launch"]) / alg
        traffic["classes"][cls] = rec
    for name in (f"{tag}_traffic.json", "latest_traffic.json"):
        json.dump(traffic, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)


if __name__ == "__main__":
    main()
