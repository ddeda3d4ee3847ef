#!/usr/bin/env python3
"""Per-kernel averages of the counters of one rocprofv3 --pmc pass (counter_collection csv):
  python tools/pmc_kernels.py DIR [kernel-substring ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
pats = sys.argv[2:] or ["k_div<", "k_grad_proj<", "k_cheb<float, float, float, float, false, 1>", "k_vcheb<2",
                        "k_cg_init<1", "k_cg_upd<1>", "k_diff2", "k_cg_dir<1"]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True) + glob.glob(os.path.join(d, "pass*.csv")):
    for row in csv.DictReader(open(f, newline="")):
        name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "").replace("pucfem::dev::", "")
        g = row.get("Grid_Size") or row.get("Grid_Size_X") or ""
        acc[(name, g)][row["Counter_Name"]].append(float(row["Counter_Value"]))
for (name, g), cs in sorted(acc.items()):
    if not any(p in name for p in pats):
        continue
    line = ", ".join(f"{k} {sum(v) / len(v):.4g}" for k, v in sorted(cs.items()))
    h, m = cs.get("TCC_HIT_sum"), cs.get("TCC_MISS_sum")
    extra = ""
    if h and m:
        extra = f"  L2 hit {sum(h) / (sum(h) + sum(m)):.3f}"
    print(f"{name} grid={g} (n={len(next(iter(cs.values())))}): {line}{extra}")
