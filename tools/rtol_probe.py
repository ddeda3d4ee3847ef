"""Accuracy of the production path against the oracle as a function of the CG tolerances: 48
StokesColor steps on mesh_fine x3 (the tests/test_gpu_production.py setting), max |u - oracle| and
max |c - oracle| along the trajectory, per (rtol_pres, rtol_visc) pair.
  python tools/rtol_probe.py [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
from conftest import load_pkg  # noqa: E402

pf = load_pkg()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 48
mesh = pf.load_mesh("fine", refine=3)
ref = O.StokesRef(mesh.coords, mesh.markers, mesh.triangles, 0.05, 0.1, -2.0, 0.0, "color")
u, c = ref.initial()
traj = []
for k in range(steps):
    out = ref.step(u, c)
    u, c = out["u"], out["c"]
    traj.append((u.copy(), c.copy()))
for rp, rv in ((1e-8, 1e-12), (1e-7, 1e-12), (1e-8, 1e-10), (1e-7, 1e-10), (1e-6, 1e-12)):
    tol = pf.Tolerances.production(rtol_pres=rp, rtol_visc=rv)
    sim = pf.StokesSimulation(mesh, pf.SquirmerBC(), 0.05, "color", 0, tol)
    wu = wc = 0.0
    its = [0, 0, 0]
    for k in range(steps):
        st = sim.step(1)[0]
        its[0] += st.it_visc
        its[1] += st.it_p
        its[2] += st.it_p2
        wu = max(wu, float(np.abs(sim.u - traj[k][0]).max()))
        wc = max(wc, float(np.abs(sim.c - traj[k][1]).max()))
    sim.close()
    print(f"rtol_pres {rp:.0e} rtol_visc {rv:.0e}: max|u-oracle| {wu:.2e} max|c-oracle| {wc:.2e} "
          f"iters visc/p/p2 {its}", flush=True)
