#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE pass, WRITE_SIZE pass).

Usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [--level 7 --world 1]
       pmc_traffic.py OLD_OUT.json - OUT_JSON     (re-derive from raw averages kept in an earlier output)

MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE come from the L2's memory-side request
counters, FETCH_SIZE under-reports wide streaming reads by exactly 2x on gfx950, and other access
widths must be calibrated on a known byte count in one's own access pattern.  The guide's
corrections (FETCH_SIZE x2, WRITE_SIZE x1, KiB units) are checked on k_diff2_fin (the projection update
of the pressure solves fused with the finish), a pure elementwise kernel whose algorithmic traffic is
36 B/row read (y, x0, A v or b, r_final; master_of) and 24 B/row written (v, A v, p), nrows from the bench
line.  (Round 3 checked k_diff2, rounds 1-2 k_visc_fin.)  Raw counter values are kept next
to the corrected bytes.  Caveat: the L2 is write-back, so up to ~32 MiB of one kernel's dirty lines
are evicted (and counted) during the next kernel.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    per = defaultdict(list)  # kernel -> values (one per dispatch)
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                g = row.get("Grid_Size") or row.get("Grid_Size_X") or ""
                per[(row["Kernel_Name"], g)].append(float(row["Counter_Value"]))
    return per


def short(name):
    """k_cheb<float, double, float>(...) -> k_cheb<float,double,float>"""
    name = re.sub(r"^void\s+", "", name)
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"pucfem::|dev::|\(anonymous namespace\)::", "", name)
    return name.replace(" ", "")


def main():
    fdir, wdir, out = sys.argv[1:4]
    level = 7
    world = 1
    if "--level" in sys.argv:
        level = int(sys.argv[sys.argv.index("--level") + 1])
    if "--world" in sys.argv:
        world = int(sys.argv[sys.argv.index("--world") + 1])
    if fdir.endswith(".json"):  # re-derive from an earlier output's raw per-kernel averages
        old = json.load(open(fdir))["kernels"]
        key = lambda k: tuple(k.split(" grid=")) if " grid=" in k else (k, "")
        fetch = {key(k): [v["fetch_raw_avg"]] * v["dispatches_fetch"] for k, v in old.items() if v["fetch_raw_avg"] is not None}
        write = {key(k): [v["write_raw_avg"]] * v["dispatches_write"] for k, v in old.items() if v["write_raw_avg"] is not None}
    else:
        fetch = load(fdir, "FETCH_SIZE")
        write = load(wdir, "WRITE_SIZE")
    kern = sorted(set(fetch) | set(write))
    # rows of the finest pressure operator: from the bench line of the PMC pass
    nrows = None
    for f in glob.glob(os.path.join(os.path.dirname(out), "bench.out")):
        try:
            rec = json.loads(open(f).read().strip().splitlines()[-1])
            nrows = rec["config"]["nodes"]
        except Exception:
            pass
    # gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of a
    # streaming read, WRITE_SIZE counts streaming stores exactly; both in KiB.  Checked on k_diff2,
    # a pure elementwise kernel with exactly 32 B/row read and 16 B/row written (all fp64): the
    # corrected values must equal the algorithmic bytes.
    res = {"counters": "FETCH_SIZE, WRITE_SIZE (separate passes, --kernel-trace only)", "kernels": {}}
    fr, fw = 2.0 * 1024.0, 1.0 * 1024.0
    check = None
    # calibration kernel: k_diff2_fin (round 4: the projection update fused with the pressure finish), a pure
    # elementwise pass: 36 B/row read (y, x0, A v or b, r_final fp64; master_of int32; the slave rows' master
    # values are 0.05 % of the rows) and 24 B/row written (v, A v, p); k_diff2 (32 / 16 B/row) before it
    check = None
    for name, rd, wr in (("k_diff2_fin", 36.0, 24.0), ("k_diff2", 32.0, 16.0)):
        cal = [k for k in kern if short(k[0]).endswith(name)]
        if cal and nrows and fetch.get(cal[0]) and write.get(cal[0]):
            f_avg = sum(fetch[cal[0]]) / len(fetch[cal[0]])
            w_avg = sum(write[cal[0]]) / len(write[cal[0]])
            check = {"kernel": name, "nrows": nrows, "algorithmic_read": rd * nrows, "corrected_read": f_avg * fr,
                     "algorithmic_write": wr * nrows, "corrected_write": w_avg * fw}
            break
    res["calibration"] = {"read_bytes_per_unit": fr, "write_bytes_per_unit": fw,
                          "note": "FETCH_SIZE x2 KiB, WRITE_SIZE x1 KiB (guide's gfx950 corrections)",
                          "check": check}
    for k in kern:
        fv, wv = fetch.get(k, []), write.get(k, [])
        e = {"dispatches_fetch": len(fv), "dispatches_write": len(wv),
             "fetch_raw_avg": sum(fv) / len(fv) if fv else None,
             "write_raw_avg": sum(wv) / len(wv) if wv else None}
        if fr and fw and fv and wv:
            e["read_bytes"] = e["fetch_raw_avg"] * fr
            e["write_bytes"] = e["write_raw_avg"] * fw
            e["hbm_bytes_per_launch"] = e["read_bytes"] + e["write_bytes"]
        res["kernels"][short(k[0]) + (f" grid={k[1]}" if k[1] else "")] = e
    # the bench's roofline kernels, finest level only: the k_cheb instances with level tag 1 (the
    # finest level's smoothing steps; tag 0 = coarser levels, 2 = pucfem_bench_kernel's batch), and
    # the pressure CG's k_cg_dir<1>
    summary = {}
    cheb = [k for k in res["kernels"] if k.startswith("k_cheb<") and "hbm_bytes_per_launch" in res["kernels"][k]]
    fine = [k for k in cheb if re.match(r"^k_cheb<[^>]*,1> grid=", k)]

    def widest(ks):  # the full launches only (the step pairs' SELL-only launches have smaller grids)
        if not ks:
            return ks
        g = max(int(k.rsplit("grid=", 1)[1]) for k in ks)
        return [k for k in ks if int(k.rsplit("grid=", 1)[1]) == g]

    fine = widest(fine)
    def pick(prefix, exclude=()):
        return [k for k in res["kernels"] if k.startswith(prefix) and not any(k.startswith(x) for x in exclude)
                and "hbm_bytes_per_launch" in res["kernels"][k]]

    # keys: the bench's kernel classes (bench.py `kernels`, roofline.kernel); k_vcheb: the whole-grid steps
    # only (the step pairs' SELL-only launches have smaller grids); k_mdot2 / k_pcomb: every basis size
    for key, ks in (("k_cheb", fine),
                    ("k_cg_dir", pick("k_cg_dir<1,")),
                    ("k_cg_upd", pick("k_cg_upd<1>")),
                    ("k_sl", pick("k_sl", ("k_sl_",))),
                    ("k_sl_slow", pick("k_sl_slow")),
                    ("k_vcheb", widest(pick("k_vcheb<"))),
                    # the step's divergence kernel (interleaved u, the full grid): the bench's kernel_batch
                    # also launches its face / skeleton parts (smaller grids)
                    ("k_div", widest(pick("k_div<", ("k_div<false,false>", "k_div<true,false>")))),
                    ("k_grad_proj", pick("k_grad_proj<")),
                    ("k_visc_prep", pick("k_visc_prep")),
                    ("k_mdot2", pick("k_mdot2<")),
                    ("k_pcomb", pick("k_pcomb<")),
                    # step pairs (both modes of the multigrid pair: the bench's class 10 averages them too)
                    ("k_cheb_pair", pick("k_cheb_pair<")),
                    ("k_vcheb_pair", pick("k_vcheb_pair"))):
        if ks:
            n = sum(res["kernels"][k]["dispatches_fetch"] for k in ks)
            summary[key] = sum(res["kernels"][k]["hbm_bytes_per_launch"] * res["kernels"][k]["dispatches_fetch"]
                               for k in ks) / n
    # the projection passes' bytes depend on the basis size M (their template argument): the ratio of PMC to
    # algorithmic bytes over the instances with M >= 16 ((4 M + 44) n for k_mdot2 -- b, the CG's accumulated v and
    # A v = r0 - r_final, with the pressure right-hand side formed in the pass: braw and slave_of read, b written
    # (+12) -- and (4 M + 24) n for k_pcomb with the production path's pending directions; PUCFEM_P_FROM_Y=0 runs:
    # 36 / 32), which bench.py applies to the algorithmic bytes of the launches it timed
    ratios = {}
    pend = os.environ.get("PUCFEM_P_FROM_Y", "1") != "0"
    if nrows:
        for key, extra in (("k_mdot2", 44.0 if pend else 36.0), ("k_pcomb", 24.0 if pend else 32.0)):
            pmc = alg = 0.0
            for k, e in res["kernels"].items():
                mm = re.match(r"^" + key + r"<(\d+)>", k)
                if mm and int(mm.group(1)) >= 16 and "hbm_bytes_per_launch" in e:
                    pmc += e["hbm_bytes_per_launch"] * e["dispatches_fetch"]
                    alg += (4.0 * int(mm.group(1)) + extra) * nrows * e["dispatches_fetch"]
            if alg > 0:
                ratios[key] = pmc / alg
    res[f"L{level}_n{world}_ratio"] = ratios
    res[f"L{level}_n{world}"] = summary
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({"calibration": res["calibration"], f"L{level}_n{world}": summary,
                      f"L{level}_n{world}_ratio": res[f"L{level}_n{world}_ratio"]}))


if __name__ == "__main__":
    main()
