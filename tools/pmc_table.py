"""Per-kernel counter table of a tools/pmc_jitter.sh (or pmc_round.sh) output directory.
usage: python tools/pmc_table.py DIR [min_ms]"""
import csv
import os
import sys
from collections import defaultdict


def short(name):
    """Kernel name without its argument list ('(anonymous namespace)::' kept out of the split)."""
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0][:60]


def main():
    src = sys.argv[1]
    min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    cnt = defaultdict(lambda: defaultdict(list))
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "p_counter_collection.csv")
        if os.path.exists(f):
            for r in csv.DictReader(open(f)):
                cnt[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "k_kernel_stats.csv"))):
        dur[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6)
    print(f"{'kernel':60s} {'calls':>5s} {'avg ms':>8s} {'VALU%':>6s} {'lane':>5s} {'LDS%':>5s} {'bank%':>5s} "
          f"{'act/wait_any/inst':>17s} {'HBM GB/s':>8s} {'waves':>8s}")
    for k, (calls, avg, tot) in sorted(dur.items(), key=lambda kv: -kv[1][2]):
        if avg < min_ms:
            continue
        c = {n: sum(v) / len(v) for n, v in cnt.get(k, {}).items()}
        if not c:
            print(f"{k:60s} {calls:5d} {avg:8.2f}")
            continue
        s = avg * 1e-3
        clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / s if c.get("GRBM_GUI_ACTIVE") else 2.4e9
        valu = c.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (1024 * clk * s) if "SQ_ACTIVE_INST_VALU" in c else float("nan")
        lane = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]) if c.get("SQ_ACTIVE_INST_VALU") else float("nan")
        lds = c.get("SQ_LDS_IDX_ACTIVE", float("nan")) / (256 * clk * s)
        bank = c.get("SQ_LDS_BANK_CONFLICT", float("nan")) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1)
        wc = c.get("SQ_WAVE_CYCLES", float("nan"))
        aw = f"{c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}/{c.get('SQ_WAIT_ANY', 0) / wc:.2f}/{c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}" if wc == wc else ""
        hbm = 2 * c.get("FETCH_SIZE", 0) * 1024 / s / 1e9
        print(f"{k:60s} {calls:5d} {avg:8.2f} {100 * valu:6.1f} {lane:5.2f} {100 * lds:5.1f} {100 * bank:5.1f} {aw:>17s} "
              f"{hbm:8.0f} {c.get('SQ_WAVES', 0):8.0f}")


if __name__ == "__main__":
    main()
