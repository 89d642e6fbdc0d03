#!/usr/bin/env python3
"""Per-dispatch HBM traffic of the solver's kernels against their algorithmic bytes.

Inputs (one deterministic program run three times, see scripts/profile.sh):
  * the solver's launch log (NKHIP_LAUNCH_LOG): one "<class> <algorithmic bytes>" line per
    Engine launch, in launch order;
  * rocprofv3 --kernel-trace CSV (per-dispatch duration), --pmc FETCH_SIZE CSV and
    --pmc WRITE_SIZE CSV (per-dispatch counters).
The i-th dispatch of a class's kernels (by kernel name, in dispatch-id order) is the i-th
launch of that class in the log, so every dispatch carries its own algorithmic bytes and its own
counters: traffic / algorithmic is computed dispatch by dispatch, never from sampled means.
HBM bytes follow MI355X_MICROARCH.md for gfx950: read = 2 x FETCH_SIZE KiB (FETCH_SIZE counts half
of a 16-B/lane streaming read), write = WRITE_SIZE KiB.  Dispatches not in the log (kernels run
outside the solver, e.g. bench.py's isolated JVP launches after the timed region) are left out.

    python scripts/traffic_match.py <tag> <prof dir> <launch log>
writes profiles/<tag>_traffic.json and profiles/latest_traffic.json.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def klass(name):
    k = name.replace("void ", "").replace("nk::(anonymous namespace)::", "")
    if k.startswith("arnoldi_kernel<") or k.startswith("arnoldi_wide_kernel<"):
        return "arnoldi_fused"
    if k.startswith("arn_ctl_kernel") or k.startswith("arn_reduce_ctl_kernel"):
        return "arnoldi_ctl"
    if k.startswith("edge_gather_kernel"):
        return "edge_gather"
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


def find(d, suffix):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith(suffix):
                return os.path.join(root, f)
    return None


def per_dispatch(path, counter=None):
    """{dispatch id: (class, value)} in dispatch order (value: counter sum or duration ns)."""
    out = collections.OrderedDict()
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        c = klass(r["Kernel_Name"])
        if c is None:
            continue
        d = int(r["Dispatch_Id"])
        if counter is None:
            out[d] = (c, float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
        elif r["Counter_Name"] == counter:
            prev = out.get(d, (c, 0.0))[1]
            out[d] = (c, prev + float(r["Counter_Value"]))
    return collections.OrderedDict(sorted(out.items()))


def by_class(disp):
    q = collections.defaultdict(list)
    for _, (c, v) in disp.items():
        q[c].append(v)
    return q


def match(fetch_csv, write_csv, trace_csv, launch_log, tag):
    """Per-class traffic of the dispatches in the FETCH_SIZE / WRITE_SIZE counter CSVs matched to
    the launch log (trace_csv, optional: per-dispatch durations)."""
    log = collections.defaultdict(list)
    for line in open(launch_log):
        c, b = line.split()
        log[c].append(float(b))
    fetch = by_class(per_dispatch(fetch_csv, "FETCH_SIZE"))
    write = by_class(per_dispatch(write_csv, "WRITE_SIZE"))
    trace = by_class(per_dispatch(trace_csv)) if trace_csv else {}
    res = {"tag": tag, "source": ("per-dispatch match of rocprofv3 FETCH_SIZE / WRITE_SIZE / "
                                  "kernel-trace passes to the solver's launch log "
                                  "(scripts/traffic_match.py)"), "classes": {}}
    for c in sorted(log):
        n = min(len(log[c]), len(fetch.get(c, [])), len(write.get(c, [])))
        if n == 0:
            continue
        alg = log[c][:n]
        rd = [2 * 1024 * v for v in fetch[c][:n]]
        wr = [1024 * v for v in write[c][:n]]
        ratio = [(a + b) / g for a, b, g in zip(rd, wr, alg) if g > 0]
        rec = {"dispatches_matched": n, "logged": len(log[c]), "profiled": len(fetch[c]),
               "alg_bytes": sum(alg), "hbm_read_bytes": sum(rd), "hbm_write_bytes": sum(wr),
               "traffic_over_alg": (sum(rd) + sum(wr)) / sum(alg) if sum(alg) else None,
               "per_dispatch_ratio_min": min(ratio) if ratio else None,
               "per_dispatch_ratio_max": max(ratio) if ratio else None,
               "alg_bytes_per_launch": sum(alg) / n,
               "hbm_bytes_per_launch": (sum(rd) + sum(wr)) / n}
        dur = trace.get(c, [])[:n]
        if dur and len(dur) == n:
            rec["avg_us"] = sum(dur) / n / 1e3
            rec["alg_GBps"] = sum(alg) / sum(dur)  # bytes per ns = GB/s
        res["classes"][c] = rec
    return res


def main():
    tag, prof, logf = sys.argv[1], sys.argv[2], sys.argv[3]
    res = match(find(os.path.join(prof, "fetch"), "counter_collection.csv"),
                find(os.path.join(prof, "write"), "counter_collection.csv"),
                find(os.path.join(prof, "trace"), "kernel_trace.csv"), logf, tag)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for name in (f"{tag}_traffic.json", "latest_traffic.json"):
        json.dump(res, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
