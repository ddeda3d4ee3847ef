#!/usr/bin/env python3
"""Per-launch view of one kernel inside the bench's timed window of a rocprofv3 kernel trace: each
launch's duration, the kernel before it on its own stream, and the kernels of other streams that
overlap it (with the overlapped time).

  python tools/trace_overlap.py kernel_trace.csv[.gz] "k_div<" --warmup 5 --steps 20
"""
import argparse
import csv
import gzip
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"pucfem::dev::", "", name)
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("kernel")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--max", type=int, default=40)
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    rows = list(csv.DictReader(op(a.trace, "rt")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    col = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    sl = [r[col] for r in rows if "k_sl<" in r["Kernel_Name"]]
    nst = [r[col] for r in rows if "k_stats" in r["Kernel_Name"]]
    two = sl and len(set(nst)) > 1
    stats_idx = [i for i, r in enumerate(rows) if "k_stats" in r["Kernel_Name"] and (not two or r[col] == sl[0])]
    win = rows[stats_idx[a.warmup - 1] + 1: stats_idx[a.warmup + a.steps - 1] + 1]
    prev = {}
    out = []
    for i, r in enumerate(win):
        s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[col]
        if a.kernel in r["Kernel_Name"]:
            ov = defaultdict(int)
            for o in win[max(0, i - 400): i + 400]:
                if o[col] == q:
                    continue
                os_, oe = int(o["Start_Timestamp"]), int(o["End_Timestamp"])
                t = min(e, oe) - max(s, os_)
                if t > 0:
                    ov[short(o["Kernel_Name"])] += t
            out.append((e - s, prev.get(q, "-"), q, dict(ov)))
        prev[q] = short(r["Kernel_Name"])
    by_prev = defaultdict(list)
    for d, p, q, ov in out:
        by_prev[(p, q)].append(d)
    print(f"{len(out)} launches of {a.kernel!r} in the window")
    for (p, q), ds in sorted(by_prev.items(), key=lambda kv: -sum(kv[1])):
        print(f"  after {p[:50]:50s} stream {q}: {len(ds):3d} launches, avg {sum(ds) / len(ds) / 1e3:7.1f} us, "
              f"min {min(ds) / 1e3:7.1f}, max {max(ds) / 1e3:7.1f}")
    for d, p, q, ov in out[: a.max]:
        top = sorted(ov.items(), key=lambda kv: -kv[1])[:4]
        print(f"  {d / 1e3:7.1f} us after {p[:36]:36s} | " + ", ".join(f"{k[:28]} {v / 1e3:.0f}" for k, v in top))


if __name__ == "__main__":
    main()
