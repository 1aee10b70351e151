"""The bench line's roofline (bench.make_roofline) from the committed counter summaries
profiles/r05/roofline_config<K>.json: every number recomputes from that one file (bytes or
instructions per launch over the counter run's own launch time, against the spec peak), the kernel
it names is the one the same command's rocprofv3 kernel stats list, and the bench copies it only
while the summary's kernel-source digest is the tree's (otherwise the line says stale, no frac)."""
import csv
import json
import os
import types

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = {"lds": 256 * 256 * 2.4, "hbm": 8000.0, "valu": 4 * 256 * 2.4 / 2}


CONFIGS = [(2, 400), (3, 400), (4, 400), (5, 800)]


def summary_path(config):
    return os.path.join(bench.ROOFLINE_DIR, f"roofline_config{config}.json")


@pytest.mark.parametrize("config,n", CONFIGS)
def test_roofline_summary_recomputes(config, n):
    if not os.path.exists(summary_path(config)):
        pytest.skip(f"no counter summary for config {config} in {bench.ROOFLINE_DIR}")
    s = json.load(open(summary_path(config)))
    r, c = s["roofline"], s["counters_per_launch"]
    res = {"lds": c["SQ_LDS_IDX_ACTIVE"] * 256.0, "valu": c["SQ_INSTS_VALU"],
           "hbm": 2.0 * c["FETCH_SIZE"] * 1024.0 + c["WRITE_SIZE"] * 1024.0}[r["bound"]]
    assert r["achieved"] == pytest.approx(res / s["avg_ns"], rel=1e-12)
    assert r["peak"] == pytest.approx(PEAK[r["bound"]]) and r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    assert 0.0 < r["frac"] <= 1.0
    assert r["traffic"] == pytest.approx(2.0 * c["FETCH_SIZE"] * 1024.0 + c["WRITE_SIZE"] * 1024.0)
    # the same command's kernel-trace stats list the kernel, with an agreeing average duration
    stats = os.path.join(bench.ROOFLINE_DIR, "pmc", f"config{config}_kernel_stats.csv")
    rows = [row for row in csv.DictReader(open(stats)) if row["Name"].startswith(s["kernel"] + "(")]
    assert len(rows) == 1
    assert float(rows[0]["AverageNs"]) == pytest.approx(s["avg_ns"], rel=0.05)
    assert f"--config {config} --n {n}" in s["command"]
    # bench.py copies it into the line at the BASELINE size
    args = types.SimpleNamespace(config=config, filter_radon=False)
    prob = types.SimpleNamespace()
    line = bench.make_roofline(args, n, n, 1, prob, 1e10, 1e7, 3e-3, 4e-3)
    assert line["kernel"] == s["kernel"] and line["bound"] == r["bound"]
    assert line["stale"] == (s["csrc_sha16"] != bench.csrc_digest())
    if not line["stale"]:
        assert line["frac"] == r["frac"] and line["traffic"] == r["traffic"]
        # with the live launch time of the timed iterations: the same bytes over that time
        live = bench.make_roofline(args, n, n, 1, prob, 1e10, 1e7, 3e-3, 4e-3, kt=(40.0, 16))
        assert live["live"]["launch_ns"] == pytest.approx(2.5e6)
        assert live["achieved"] == pytest.approx(r["resource_bytes_per_launch"] / 2.5e6)
        assert live["frac"] == pytest.approx(live["achieved"] / r["peak"]) and live["frac_counter_run"] == r["frac"]
    # other sizes carry no roofline
    assert bench.make_roofline(args, 64, 64, 1, prob, 1e6, 1e4, 1e-3, 1e-3)["frac"] is None


def test_stale_counters_claim_no_fraction(tmp_path, monkeypatch):
    """A summary collected on other kernel sources: bench reports it as stale, with no frac,
    achieved or traffic; the same summary with the tree's digest is copied."""
    s = {"build": "0" * 12, "kernel": "void k<1>", "avg_ns": 1e6, "clock_ghz_measured": 2.2,
         "csrc_sha16": "feedfacefeedface",
         "roofline": {"bound": "hbm", "achieved": 4000.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.5,
                      "traffic": 4e9, "traffic_over_min": 2.0, "min_bytes": 2e9, "valu_issue_frac": 0.1,
                      "hbm_frac": 0.5, "lds_frac": 0.1, "lds_bank_conflict_frac": 0.0,
                      "frac_at_measured_clock": None}}
    monkeypatch.setattr(bench, "ROOFLINE_DIR", str(tmp_path))
    (tmp_path / "roofline_config4.json").write_text(json.dumps(s))
    args = types.SimpleNamespace(config=4, filter_radon=False)
    line = bench.make_roofline(args, 400, 400, 1, None, 1e10, 1e7, 1.0, 1.5)
    assert line["stale"] is True and line["frac"] is None and line["achieved"] is None and line["traffic"] is None
    assert line["stale_frac"] == 0.5 and line["counters_csrc_sha16"] == "feedfacefeedface"
    s["csrc_sha16"] = bench.csrc_digest()
    (tmp_path / "roofline_config4.json").write_text(json.dumps(s))
    line = bench.make_roofline(args, 400, 400, 1, None, 1e10, 1e7, 1.0, 1.5)
    assert line["stale"] is False and line["frac"] == 0.5 and line["traffic"] == 4e9


def test_csrc_digest_tracks_kernel_sources(tmp_path, monkeypatch):
    """The digest covers every .hip / .h under csrc, build.sh and include/tvam.h: editing any
    of them changes it."""
    import shutil
    for d in ("drtvam_amd/csrc", "include"):
        shutil.copytree(os.path.join(ROOT, d), tmp_path / d)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    d0 = bench.csrc_digest()
    assert d0 == bench.csrc_digest()
    monkeypatch.setattr(bench, "ROOT", ROOT)
    assert d0 == bench.csrc_digest()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    for f in ("drtvam_amd/csrc/tvam_scatter.hip", "drtvam_amd/csrc/tvam_common.h", "include/tvam.h"):
        with open(tmp_path / f, "a") as fh:
            fh.write("\n")
        d1 = bench.csrc_digest()
        assert d1 != d0
        d0 = d1


def test_host_info_threads_are_the_affinity(monkeypatch):
    """The CPU baseline's reported value runs on every CPU of the process's affinity; the
    OMP_NUM_THREADS share is the second timing."""
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    h = bench.host_info()
    assert h["threads"] == h["affinity"] == len(os.sched_getaffinity(0))
    assert h["omp_threads"] == 1
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.host_info()["omp_threads"] == h["affinity"]
