"""Print a rocprofv3 kernel-stats CSV compactly: python tools/kstats.py FILE [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in rows[:n]:
    name = r["Name"].replace("(anonymous namespace)::", "")
    name = name.split("(")[0] if "rocprim" not in name else "rocprim " + name.split("detail::")[2][:40]
    print(f"{name[:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e6:9.3f} ms {float(r['TotalDurationNs']) / 1e6:9.1f} ms "
          f"{float(r['Percentage']):6.2f}%")
