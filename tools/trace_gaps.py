"""Idle gaps of one stream in a rocprofv3 kernel trace: for each kernel name, the median time from its
end to the next kernel's start (over the last N iterations of the trace), and the busy fraction.

usage: python tools/trace_gaps.py TRACE.csv [last_ms]
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70]) for r in rows))
    t_end = ks[-1][1]
    ks = [k for k in ks if k[0] >= t_end - last_ms * 1e6]
    gaps = defaultdict(list)
    busy = 0
    cur_end = ks[0][0]
    for a, b in zip(ks, ks[1:]):
        gaps[a[2]].append(max(0, b[0] - a[1]) / 1e3)
    for s, e, _ in ks:  # union of busy intervals
        if e > cur_end:
            busy += e - max(s, cur_end)
            cur_end = e
    # per optimiser iteration: the period between successive history passes and the busy time in it
    marks = [s for s, _, n in ks if "tvam_lbfgs_hist_kernel" in n]
    per, idle = [], []
    for t0, t1 in zip(marks, marks[1:]):
        b, ce = 0, t0
        for s, e, _ in ks:
            if e <= t0 or s >= t1:
                continue
            s, e = max(s, t0, ce), min(e, t1)
            if e > s:
                b += e - s
                ce = e
        per.append((t1 - t0) / 1e3)
        idle.append((t1 - t0 - b) / 1e3)
    if per:
        print(f"iteration period median {statistics.median(per):.1f} us, idle in it median {statistics.median(idle):.1f} us"
              f" over {len(per)} iterations")
    # the timeline around the second-to-last Armijo probe pass (host read, update, next iteration)
    pr = [i for i, k in enumerate(ks) if "tvam_loss_probes_kernel" in k[2]]
    if len(pr) >= 2:
        i0 = pr[-2]
        t0 = ks[i0][0]
        for s, e, n in ks[i0:i0 + 8]:
            print(f"  {(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us  {n}")
    span = ks[-1][1] - ks[0][0]
    print(f"span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms ({busy / span:.3f}), {len(ks)} kernels")
    tot = sorted(((sum(v), statistics.median(v), len(v), k) for k, v in gaps.items()), reverse=True)
    for s, m, n, k in tot[:15]:
        print(f"{s / 1e3:8.3f} ms total  {m:8.1f} us median  x{n:4d}  after {k}")


if __name__ == "__main__":
    main()
