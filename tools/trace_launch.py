#!/usr/bin/env python3
"""Per-launch view of one kernel in a rocprofv3 --kernel-trace CSV: duration, gap since the previous
kernel on the queue ended, the previous kernel's name, and overlaps with it.

Usage: trace_launch.py KERNEL_TRACE_CSV SUBSTRING [--last-ms T]
(used to compare the library's per-launch dispatch events with the profiler's kernel durations)
"""
import csv
import statistics as st
import sys
from collections import Counter


def short(n):
    return n.split("(")[0].replace("void ", "").replace("pucfem::dev::", "")


def main():
    path, pat = sys.argv[1], sys.argv[2]
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)))
    rows.sort()
    if "--last-ms" in sys.argv:
        tend = max(r[1] for r in rows)
        cut = tend - float(sys.argv[sys.argv.index("--last-ms") + 1]) * 1e6
        rows = [r for r in rows if r[0] >= cut]
    dur, gap, prev, ov = [], [], Counter(), 0
    for i, (s, e, n, g) in enumerate(rows):
        if pat not in n or i == 0:
            continue
        ps, pe, pn, pg = rows[i - 1]
        dur.append((e - s) / 1e3)
        gap.append((s - pe) / 1e3)
        prev[f"{short(pn)} grid={pg}"] += 1
        ov += s < pe
    if not dur:
        print("no launches match", pat)
        return
    q = lambda v: f"mean {st.mean(v):8.1f}  median {st.median(v):8.1f}  min {min(v):8.1f}  max {max(v):8.1f} us"
    print(f"{len(dur)} launches of *{pat}*")
    print("duration ", q(dur))
    qs = st.quantiles(dur, n=10) if len(dur) > 1 else dur
    print("duration deciles", " ".join(f"{x:.1f}" for x in qs))
    print("gap      ", q(gap))
    print("duration+gap mean", f"{st.mean(d + max(g, 0) for d, g in zip(dur, gap)):.1f} us; overlaps {ov}")
    for k, v in prev.most_common(8):
        print(f"  after {v:5d} x {k}")


if __name__ == "__main__":
    main()
