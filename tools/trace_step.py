#!/usr/bin/env python3
"""Per-step timeline analysis of a rocprofv3 --kernel-trace CSV (bench.py run).

Usage: trace_step.py KERNEL_TRACE_CSV [--last-ms T]
Takes the kernel activity after the last gap > 50 ms (the bench's steps), or only its last T ms
(--last-ms: the timed steps after the warm-up), and prints the busy time per kernel name, the sum
of gaps between consecutive kernels, and the wall span.
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)))
    rows.sort()
    # the timed region: kernels after the last gap > 50 ms (setup / warm-up / host work before it)
    start = 0
    for i in range(1, len(rows)):
        if rows[i][0] - rows[i - 1][1] > 50_000_000:
            start = i
    rows = rows[start:]
    if "--last-ms" in sys.argv:
        tend = max(r[1] for r in rows)
        cut = tend - float(sys.argv[sys.argv.index("--last-ms") + 1]) * 1e6
        rows = [r for r in rows if r[0] >= cut]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    busy = defaultdict(float)
    cnt = defaultdict(int)
    gaps = 0.0
    last_end = rows[0][0]
    for s, e, n, g in rows:
        key = n.split("(")[0].replace("void ", "").replace("pucfem::dev::", "")
        key = f"{key} grid={g}" if ("cheb" in key or "resid" in key or "transfer" in key) else key
        busy[key] += (e - s) / 1e6
        cnt[key] += 1
        if s > last_end:
            gaps += (s - last_end) / 1e6
        last_end = max(last_end, e)
    span = (t1 - t0) / 1e6
    print(f"kernels {len(rows)}  span {span:.2f} ms  busy {sum(busy.values()):.2f} ms  gaps {gaps:.2f} ms")
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:60]:
        print(f"{v:9.3f} ms {cnt[k]:6d}  {v / cnt[k] * 1e3:8.1f} us  {k[:110]}")


if __name__ == "__main__":
    main()
