"""profiles/<round>_configs.md (+ per-config bench json / kernel stats) from a
tools/profile_configs.sh output directory.  usage: summarize_configs.py OUTDIR PREFIX"""
import json
import os
import re
import shutil
import sys

TITLES = {
    3: "config 3: cylindrical vial, 400^3, 400 angles, regular sampling",
    4: "config 4: cylindrical vial + scattering resin, 400^3, 400 angles, 16 spp",
    5: "config 5: square vial + occluder, 800^3, 800 angles, 4 spp",
}


def short(name):
    name = name.strip('"')
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", name)
    s = m.group(1) if m else name
    return s[:80]


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    lines = ["# Kernel profiles of BASELINE configs 3-5", "",
             "`rocprofv3 --kernel-trace --stats -- python3 bench.py --config N ...` (tools/profile_configs.sh);",
             "the bench line of the same (profiled) run beside each table; top kernels by total time.", ""]
    for c in (3, 4, 5):
        bj = os.path.join(src, f"c{c}_bench.json")
        stats = os.path.join(src, f"c{c}", f"c{c}_kernel_stats.csv")
        if not (os.path.exists(bj) and os.path.exists(stats)):
            continue
        d = json.loads(open(bj).read().strip().splitlines()[-1])
        cf = d["config"]
        lines += [f"## {TITLES[c]} (steps {d['steps']}, warmup {d['warmup']})", "",
                  f"bench (under the profiler): {d['value']:.4g} it/s, fwd {cf['fwd_ms']:.2f} ms, "
                  f"adj {cf['adj_ms']:.2f} ms, visits/pass {cf['visits_per_pass']:.4g}", "",
                  "| kernel | calls | total ms | avg ms |", "|---|---|---|---|"]
        import csv
        rows = list(csv.DictReader(open(stats)))
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        for r in rows[:12]:
            lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                         f"{float(r['AverageNs']) / 1e6:.3f} |")
        lines.append("")
        shutil.copy(bj, f"{prefix}_config{c}_bench.json")
        shutil.copy(stats, f"{prefix}_config{c}_kernel_stats.csv")
    lines += ["Notes: `tvam_tile_kernel<2>` / `tvam_scatter_kernel<2>` are the one-off visit counts of the bench "
              "setup", "(not in the timed loop); `tvam_ray_setup_kernel` reruns per call under jittered sampling "
              "(new seed)."]
    open(f"{prefix}_configs.md", "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
