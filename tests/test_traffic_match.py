"""CPU: the per-dispatch HBM-traffic match that bench.py runs live (scripts/traffic_match.py).

rocprofv3 --pmc writes one row per (dispatch, counter); the solver's launch log has one
"<class> <algorithmic bytes>" line per launch.  The i-th dispatch of a class is the i-th logged
launch of that class; HBM bytes = 2 x FETCH_SIZE KiB + WRITE_SIZE KiB (MI355X_MICROARCH.md, gfx950).
Synthetic CSVs pin that arithmetic, the class mapping and the handling of unlogged kernels.
"""
import csv
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import traffic_match as tm  # noqa: E402

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def _csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(FIELDS, r)))
    return str(path)


def test_per_dispatch_ratios(tmp_path):
    fused = "void nk::(anonymous namespace)::arnoldi_kernel<24, false, 1, true, true, 2>(nk::ArnoldiArgs)"
    wide = "void nk::(anonymous namespace)::arnoldi_wide_kernel<8, false, 2, true, 4, false>(nk::ArnoldiArgs)"
    jvp = "void nk::(anonymous namespace)::march_kernel<(nk::SMode)5, 128, 1>(nk::StencilArgs, int, int, int)"
    other = "void at::native::vectorized_elementwise_kernel<4>(int)"  # not the solver's: ignored
    fetch = _csv(tmp_path / "f.csv", [
        (1, fused, "FETCH_SIZE", 1000.0), (2, jvp, "FETCH_SIZE", 400.0),
        (3, other, "FETCH_SIZE", 9999.0), (4, wide, "FETCH_SIZE", 500.0),
        (5, jvp, "FETCH_SIZE", 410.0)])
    write = _csv(tmp_path / "w.csv", [
        (1, fused, "WRITE_SIZE", 200.0), (2, jvp, "WRITE_SIZE", 100.0),
        (3, other, "WRITE_SIZE", 9999.0), (4, wide, "WRITE_SIZE", 100.0),
        (5, jvp, "WRITE_SIZE", 100.0)])
    log = tmp_path / "launches"
    # KiB -> bytes: the fused class (two dispatches) 2*1024*1000 + 1024*200 = 2252800 and
    # 2*1024*500 + 1024*100 = 1126400 against 2000000 and 1000000 algorithmic bytes
    log.write_text("arnoldi_fused 2000000\nsh_fdjvp 900000\narnoldi_fused 1000000\n"
                   "sh_fdjvp 900000\n")
    res = tm.match(fetch, write, None, str(log), "t")
    c = res["classes"]
    assert set(c) == {"arnoldi_fused", "sh_fdjvp"}
    f = c["arnoldi_fused"]
    assert f["dispatches_matched"] == 2
    assert f["hbm_read_bytes"] == 2 * 1024 * 1500 and f["hbm_write_bytes"] == 1024 * 300
    assert f["traffic_over_alg"] == pytest.approx((2252800 + 1126400) / 3000000)
    assert f["per_dispatch_ratio_min"] == pytest.approx(1.1264)
    assert f["per_dispatch_ratio_max"] == pytest.approx(1.1264)
    j = c["sh_fdjvp"]
    assert j["hbm_read_bytes"] == 2 * 1024 * 810
    assert j["alg_bytes_per_launch"] == 900000


def test_more_dispatches_than_logged_launches(tmp_path):
    """Dispatches past the logged launches of a class (e.g. a probe after the solver) are not
    matched: only min(logged, profiled) dispatches count."""
    k = "void nk::(anonymous namespace)::combo_kernel<true, true, 2>(double*)"
    fetch = _csv(tmp_path / "f.csv", [(i, k, "FETCH_SIZE", 50.0) for i in range(1, 4)])
    write = _csv(tmp_path / "w.csv", [(i, k, "WRITE_SIZE", 10.0) for i in range(1, 4)])
    log = tmp_path / "launches"
    log.write_text("krylov_combo 110592\n")
    c = tm.match(fetch, write, None, str(log), "t")["classes"]["krylov_combo"]
    assert c["dispatches_matched"] == 1 and c["profiled"] == 3 and c["logged"] == 1
    assert c["traffic_over_alg"] == pytest.approx((2 * 1024 * 50 + 1024 * 10) / 110592)


def test_fallback_traffic_file_is_the_newest_profile():
    """The N > 1 line takes roofline.traffic from profiles/latest_traffic.json (no live PMC pass
    there): it must be the newest committed profile's per-dispatch match, and every class in it a
    class that profiled run of the solver launched (the file lists only logged classes)."""
    import glob
    import json
    import re
    prof = os.path.join(ROOT, "profiles")
    tagged = {}
    for p in glob.glob(os.path.join(prof, "r*_traffic.json")):
        m = re.match(r"r(\d+)([a-z]*)_traffic\.json$", os.path.basename(p))
        if m:
            tagged[(int(m.group(1)), m.group(2))] = p
    newest = tagged[max(tagged)]
    latest = json.load(open(os.path.join(prof, "latest_traffic.json")))
    assert latest == json.load(open(newest)), f"latest_traffic.json is not {newest}"
    assert latest["classes"], latest
    for name, c in latest["classes"].items():
        assert c["logged"] > 0 and c["dispatches_matched"] > 0, (name, c)
        assert c["traffic_over_alg"] and 0.5 < c["traffic_over_alg"] < 2.0, (name, c)
