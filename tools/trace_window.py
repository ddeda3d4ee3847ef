#!/usr/bin/env python3
"""Per-kernel time inside the bench's timed window from a rocprofv3 kernel trace.

The window is the kernels between the end of warm-up step W (the W-th k_stats launch; with the
overlapped dye advection, the W-th on the k_sl stream) and the end of the last timed step (k_stats
launch W+K).  Prints total / calls / average per kernel (name shortened,
grid size kept so multigrid levels stay apart), the window's span, busy time and idle gaps.

  python tools/trace_window.py kernel_trace.csv --warmup 5 --steps 20
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
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    # only the last N timed steps (the bench's per-launch events cover the last 5 of the 20 timed steps)
    ap.add_argument("--last", type=int, default=0)
    # a kernel name prefix: also print its launches' average over the window (every template instance)
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    rows = list(csv.DictReader(op(a.trace, "rt")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a step ends with its last k_stats: with the dye advection on a side stream (one k_stats per
    # stream per step) that is the side stream's, the stream k_sl runs on
    col = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    sl = [r[col] for r in rows if "k_sl<" in r["Kernel_Name"]]
    nst = [r[col] for r in rows if "k_stats" in r["Kernel_Name"]]
    two = sl and len(nst) > 0 and len(set(nst)) > 1
    stats_idx = [i for i, r in enumerate(rows)
                 if "k_stats" in r["Kernel_Name"] and (not two or r[col] == sl[0])]
    if a.last:
        a.warmup, a.steps = a.warmup + a.steps - a.last, a.last
    i0 = stats_idx[a.warmup - 1] + 1
    i1 = stats_idx[a.warmup + a.steps - 1] + 1
    win = rows[i0:i1]
    t0 = int(win[0]["Start_Timestamp"])
    t1 = int(win[-1]["End_Timestamp"])
    agg = defaultdict(lambda: [0, 0])
    busy = 0
    last_end = t0
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        key = f'{short(r["Kernel_Name"])} grid={r.get("Grid_Size_X", r.get("Grid_Size", "?"))}'
        agg[key][0] += e - s
        agg[key][1] += 1
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    span = t1 - t0
    print(f"window: {len(win)} kernels, span {span / 1e6:.2f} ms ({span / 1e6 / a.steps:.3f} ms/step), "
          f"busy {busy / 1e6:.2f} ms, gaps {(span - busy) / 1e6:.2f} ms")
    if a.kernel:
        ks = [(t, n) for k, (t, n) in agg.items() if k.startswith(a.kernel)]
        if ks:
            tt, nn = sum(t for t, _ in ks), sum(n for _, n in ks)
            print(f"{a.kernel}*: {nn} launches, average {tt / nn / 1e3:.1f} us")
    for k, (tot, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{tot / 1e6:9.3f} ms {n:6d} {tot / n / 1e3:9.1f} us  {tot / span * 100:5.1f}%  {k}")


if __name__ == "__main__":
    main()
