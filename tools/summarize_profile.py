"""Turns a tools/profile_round.sh output directory into committed profile artefacts.

usage: python tools/summarize_profile.py gpurun_out/r1a profiles/r01
Writes <prefix>_kernel_stats.csv (rocprofv3 --stats of bench.py), <prefix>_bench.json,
<prefix>_summary.md and profiles/pmc_traffic.json (forward-kernel HBM bytes per launch,
FETCH_SIZE x2 for gfx950 wide reads + WRITE_SIZE, both reported in KiB by rocprofv3;
MI355X_MICROARCH.md section HBM).
"""
import csv
import json
import os
import shutil
import sys


def per_kernel(path):
    out = {}
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if "tvam_fwd_planar_kernel" in n:
            key = "forward"
        elif "tvam_adj_planar_kernel" in n:
            key = "adjoint"
        elif "tvam_tile_kernel" in n:
            key = {"0": "forward_tile", "1": "adjoint_tile", "2": "count"}[n.split("<")[1][0]]
        elif "tvam_ray_setup" in n:
            key = "ray_setup"
        elif "tvam_planar_rays" in n:
            key = "planar_rays"
        else:
            continue
        out.setdefault(key, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    os.makedirs(os.path.dirname(prefix), exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "bench_kernel_stats.csv"), prefix + "_kernel_stats.csv")
    bench = json.load(open(os.path.join(src, "bench.json")))
    json.dump(bench, open(prefix + "_bench.json", "w"), indent=1)
    fetch = per_kernel(os.path.join(src, "fetch", "p_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "write", "p_counter_collection.csv"))
    traffic = {}
    for k in fetch:
        traffic[k] = {"FETCH_SIZE_KiB": fetch[k], "WRITE_SIZE_KiB": write.get(k, 0.0),
                      "hbm_bytes": 2 * fetch[k] * 1024 + write.get(k, 0.0) * 1024}
    json.dump({"workload": "config2 400^3 / 400 angles (tools/kernel_sweep.py 400 0)", "per_launch": traffic,
               "note": "FETCH_SIZE doubled per the gfx950 wide-read calibration; mixed 4/8/16-B accesses are "
                       "uncalibrated, so treat as an estimate"},
              open(os.path.join(os.path.dirname(prefix), "pmc_traffic.json"), "w"), indent=1)
    rows = list(csv.DictReader(open(prefix + "_kernel_stats.csv")))
    lines = [f"# Profile {os.path.basename(prefix)}", "",
             f"bench: {bench['value']:.2f} it/s, {bench['ms_per_step']:.1f} ms/step, fwd {bench['config']['fwd_ms']:.2f} ms, "
             f"adj {bench['config']['adj_ms']:.2f} ms (HIP events, bench.py)", "",
             "## rocprofv3 --kernel-trace --stats (bench.py --steps 5 --warmup 2)", "",
             "| kernel | calls | avg ms | % |", "|---|---|---|---|"]
    for r in rows[:12]:
        lines.append(f"| {r['Name'][:80]} | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
    lines += ["", "## HBM traffic per launch (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)", "",
              "| kernel | FETCH_SIZE KiB | WRITE_SIZE KiB | est. bytes |", "|---|---|---|---|"]
    for k, v in traffic.items():
        lines.append(f"| {k} | {v['FETCH_SIZE_KiB']:.4g} | {v['WRITE_SIZE_KiB']:.4g} | {v['hbm_bytes']:.4g} |")
    open(prefix + "_summary.md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
