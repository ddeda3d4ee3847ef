"""Per-rank multi-GPU data flow of the StokesColor step on W LocalComm ranks (one GPU, one process):
the wide dye halo each rank receives vs a full all-gather, after each of S steps, and per step the
communicator's traffic (pucfem_comm_counters: all-reduce calls and values, point-to-point sends and
bytes, grouped launches, broadcasts), the pressure / viscous iteration counts and the kernel launches.
The same call sequence runs over RCCL on W GPUs (NcclComm), so the counts are the production path's.
  python tools/comm_probe.py LEVEL W STEPS [MG_REP_NODES]"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg  # noqa: E402

pf = load_pkg()
level, world, steps = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (5, 8, 6)))
rep_nodes = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # coarse levels up to this size replicated (0: default)
mesh = pf.load_mesh("fine", refine=level)
uid = b"PUCFEM-LOCALCOMM" + os.urandom(112)
rows = [[None] * steps for _ in range(world)]
errs = []


def worker(r):
    try:
        sim = pf.StokesSimulation(mesh, pf.SquirmerBC(), 0.05, "color", 0,
                                  pf.Tolerances.production(mg_rep_nodes=rep_nodes), dist=(r, world, uid))
        for k in range(steps):
            c0, (n0, _) = sim.ctx.comm_counters(), sim.ctx.counters()
            st = sim.step(1)[0]
            c1, (n1, _) = sim.ctx.comm_counters(), sim.ctx.counters()
            rows[r][k] = sim.ctx.comm_info()
            rows[r][k]["traffic"] = {key: c1[key] - c0[key] for key in c1}
            rows[r][k]["traffic"]["launches"] = n1 - n0
            rows[r][k]["its"] = (st.it_visc, st.it_p, st.it_p2)
        sim.close()
    except Exception as e:  # pragma: no cover
        errs.append((r, repr(e)))


th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
for t in th:
    t.start()
for t in th:
    t.join()
assert not errs, errs
print(f"L{level} N={mesh.N} W={world} mg_rep_nodes={rep_nodes or 'default'}")
pts = []
for k in range(steps):
    h = [rows[r][k]["dye_halo_values"] for r in range(world)]
    a = [rows[r][k]["allgather_values"] for r in range(world)]
    print(f"step {k}: dye halo values per rank {h} (max {max(h) * 8 / 1e6:.2f} MB) vs all-gather "
          f"{max(a) * 8 / 1e6:.2f} MB")
    t = [rows[r][k]["traffic"] for r in range(world)]
    mx = {key: max(x[key] for x in t) for key in t[0]}
    print(f"        iterations visc/p/p2 {rows[0][k]['its']}; per rank (max over ranks): "
          f"{mx['allreduce_calls']} all-reduces ({mx['allreduce_values']} values), {mx['sends']} sends "
          f"({mx['send_bytes'] / 1e6:.2f} MB), {mx['broadcasts']} broadcasts, {mx['groups']} groups, "
          f"{mx['launches']} kernel launches")
    pts.append((rows[0][k]["its"][1] + rows[0][k]["its"][2], mx["allreduce_calls"], mx["groups"]))
# per pressure PCG iteration: the slope over the steps (least squares of the counts against the iterations)
import numpy as np  # noqa: E402

it_, ar_, gr_ = (np.array(v, dtype=float) for v in zip(*pts))
if len(pts) > 1 and np.ptp(it_) > 0:
    A = np.stack([it_, np.ones_like(it_)], 1)
    sa = np.linalg.lstsq(A, ar_, rcond=None)[0]
    sg = np.linalg.lstsq(A, gr_, rcond=None)[0]
    print(f"per pressure PCG iteration: {sa[0]:.2f} all-reduces, {sg[0]:.2f} grouped exchanges "
          f"(per step outside the iterations: {sa[1]:.1f} all-reduces, {sg[1]:.1f} groups)")
