"""Turns a tools/pmc_round.sh output directory into the committed counter summary that bench.py's
roofline reads.  usage: python tools/summarize_pmc.py gpurun_out/<dir>/pmc profiles/r02/pmc_config2.json

Per kernel family (forward = tvam_slice_bin_kernel + tvam_fwd_planar_kernel, the two launches of one
tvam_forward call; adjoint = tvam_adj_planar_kernel) it writes the per-launch averages of every
counter of the four --pmc passes and the average duration from the --kernel-trace --stats pass.
SQ counters are summed over the chip; GRBM_GUI_ACTIVE over the 8 XCDs (its per-XCD value / duration
is the clock the kernel ran at)."""
import csv
import json
import os
import sys
from collections import defaultdict

FAMILIES = {
    "forward": ("tvam_fwd_planar_kernel", "tvam_slice_bin_kernel"),
    "adjoint": ("tvam_adj_planar_kernel",),
    "forward_rays": ("tvam_fwd_rays_planar_kernel",),
    "forward_tile": ("tvam_tile_kernel<0>",),
    "adjoint_tile": ("tvam_tile_kernel<1>",),
}


def family(name):
    for fam, keys in FAMILIES.items():
        if any(k in name for k in keys):
            return fam
    return None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))  # fam -> kernel -> counter -> values
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "p_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            fam = family(r["Kernel_Name"])
            if fam:
                per[fam][r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(dict)
    stats = os.path.join(src, "trace", "k_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        fam = family(r["Name"])
        if fam:
            dur[fam][r["Name"].split("(")[0]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    out = {"source": f"tools/pmc_round.sh (rocprofv3 --pmc, 4 passes; --kernel-trace --stats) of "
                     f"tools/kernel_sweep.py 400 0: config 2, 400^3, 400 angles", "kernels": {}}
    for fam, ks in per.items():
        fam_out = {"launches": {}, "sum": defaultdict(float)}
        for kname, cs in ks.items():
            avg = {c: sum(v) / len(v) for c, v in cs.items()}
            d = dur[fam].get(kname, {})
            fam_out["launches"][kname] = {"counters_per_launch": avg, "avg_ns": d.get("avg_ns"), "calls": d.get("calls")}
            for c, v in avg.items():
                fam_out["sum"][c] += v
            fam_out["sum"]["avg_ns"] += d.get("avg_ns") or 0.0
        main_k = max(fam_out["launches"], key=lambda k: fam_out["launches"][k]["avg_ns"] or 0.0)
        m = fam_out["launches"][main_k]
        ns = m["avg_ns"]
        c = m["counters_per_launch"]
        if ns and "GRBM_GUI_ACTIVE" in c:
            m["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / ns
        fam_out["sum"] = dict(fam_out["sum"])
        fam_out["main"] = main_k
        out["kernels"][fam] = fam_out
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({f: {"main": v["main"], "avg_ns": v["sum"]["avg_ns"]} for f, v in out["kernels"].items()}))


if __name__ == "__main__":
    main()
