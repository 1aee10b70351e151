"""Summarise rocprofv3 --pmc CSVs per kernel: python tools/pmc_summary.py DIR..."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "tvam_" not in name:
                continue
            mode = name.replace("(anonymous namespace)::", "").split("(")[0]
            agg[mode][r["Counter_Name"]].append(float(r["Counter_Value"]))
for mode, cs in sorted(agg.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(f"mode {mode}: " + ", ".join(f"{c}={x:.4g}" for c, x in sorted(m.items())))
    if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m:
        print(f"   lane utilisation (THREAD_CYCLES_VALU / (ACTIVE_INST_VALU*64)) = {m['SQ_THREAD_CYCLES_VALU'] / (64 * m['SQ_ACTIVE_INST_VALU']):.3f}")
    if "SQ_WAIT_ANY" in m and "SQ_ACTIVE_INST_ANY" in m:
        tot = m["SQ_WAIT_ANY"] + m["SQ_WAIT_INST_ANY"] + m["SQ_ACTIVE_INST_ANY"]
        print(f"   wave time: wait_any {m['SQ_WAIT_ANY'] / tot:.2f}, wait_inst {m['SQ_WAIT_INST_ANY'] / tot:.2f}, active {m['SQ_ACTIVE_INST_ANY'] / tot:.2f}")
