#!/usr/bin/env python3
"""Per-launch listing of the last hipGraph replays of the small-mesh step (tools/fine_probe.py under rocprofv3
--kernel-trace): every kernel of the last REPLAYS steps (a step ends with k_stats, or with k_mix2 when that kernel
appends the step record, and the record's copy) with its
start offset, duration and the gap before it, then the per-step totals.
Usage: trace_replay.py KERNEL_TRACE_CSV [REPLAYS]"""
import csv
import sys


def short(n):
    return n.split("(")[0].replace("void ", "").replace("pucfem::dev::", "")[:70]


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if r[2].startswith("k_stats")]
    if len(ends) < k + 1:  # (the record appended by k_mix2: the step ends there)
        ends = [i for i, r in enumerate(rows) if r[2].startswith("k_mix2")]
    if len(ends) < k + 1:
        print("not enough k_stats / k_mix2 launches")
        return
    a, b = ends[-k - 1] + 1, len(rows)
    # the record copy after the last k_stats belongs to that step
    sel = rows[a:b]
    t0 = sel[0][0]
    prev_end = rows[a - 1][1]
    busy = 0
    print(f"{'start us':>9} {'dur us':>8} {'gap us':>8}  kernel")
    for s, e, n in sel:
        print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} {(s - prev_end) / 1e3:8.2f}  {n}")
        busy += e - s
        prev_end = max(prev_end, e)
    span = sel[-1][1] - t0
    print(f"{len(sel)} launches over {k} steps: span {span / 1e3:.1f} us ({span / 1e3 / k:.1f} us/step), "
          f"busy {busy / 1e3:.1f} us, gaps {(span - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
