"""The bench line's roofline (bench.make_roofline) from the committed counter summaries
profiles/r03/roofline_config<K>.json: every number recomputes from that one file (bytes or
instructions per launch over the counter run's own launch time, against the spec peak), the kernel
it names is the one the same command's rocprofv3 kernel stats list, and the bench copies it."""
import csv
import json
import os
import types

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = {"lds": 256 * 256 * 2.4, "hbm": 8000.0, "valu": 4 * 256 * 2.4 / 2}


@pytest.mark.parametrize("config,n", [(2, 400), (3, 400), (4, 400), (5, 800)])
def test_roofline_summary_recomputes(config, n):
    s = json.load(open(os.path.join(ROOT, "profiles", "r03", f"roofline_config{config}.json")))
    r, c = s["roofline"], s["counters_per_launch"]
    res = {"lds": c["SQ_LDS_IDX_ACTIVE"] * 256.0, "valu": c["SQ_INSTS_VALU"],
           "hbm": 2.0 * c["FETCH_SIZE"] * 1024.0 + c["WRITE_SIZE"] * 1024.0}[r["bound"]]
    assert r["achieved"] == pytest.approx(res / s["avg_ns"], rel=1e-12)
    assert r["peak"] == pytest.approx(PEAK[r["bound"]]) and r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    assert 0.0 < r["frac"] <= 1.0
    assert r["traffic"] == pytest.approx(2.0 * c["FETCH_SIZE"] * 1024.0 + c["WRITE_SIZE"] * 1024.0)
    # the same command's kernel-trace stats list the kernel, with an agreeing average duration
    stats = os.path.join(ROOT, "profiles", "r03", "pmc", f"config{config}_kernel_stats.csv")
    rows = [row for row in csv.DictReader(open(stats)) if row["Name"].startswith(s["kernel"] + "(")]
    assert len(rows) == 1
    assert float(rows[0]["AverageNs"]) == pytest.approx(s["avg_ns"], rel=0.05)
    assert f"--config {config} --n {n}" in s["command"]
    # bench.py copies it into the line at the BASELINE size
    args = types.SimpleNamespace(config=config, filter_radon=False)
    prob = types.SimpleNamespace()
    line = bench.make_roofline(args, n, n, 1, prob, 1e10, 1e7, 3e-3, 4e-3)
    assert line["frac"] == r["frac"] and line["kernel"] == s["kernel"] and line["bound"] == r["bound"]
    assert line["traffic"] == r["traffic"]
    # other sizes carry no roofline
    assert bench.make_roofline(args, 64, 64, 1, prob, 1e6, 1e4, 1e-3, 1e-3)["frac"] is None
