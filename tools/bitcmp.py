"""Hash of the fields after K production steps (compare two builds bit for bit: run once per PUCFEM_LIB_VARIANT).
  python tools/bitcmp.py LEVEL STEPS [RTOL_PRES]"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg  # noqa: E402

pf = load_pkg()
level, steps = int(sys.argv[1]), int(sys.argv[2])
tol = pf.Tolerances.production(rtol_pres=float(sys.argv[3])) if len(sys.argv) > 3 else pf.Tolerances.production()
sim = pf.StokesSimulation(pf.load_mesh("fine", refine=level), pf.SquirmerBC(), 0.05, "color", 0, tol)
its = [(s.it_visc, s.it_p, s.it_p2) for k in (1, 4, steps - 5) for s in sim.step(k)]
h = hashlib.sha256()
for a in (sim.u, sim.c):
    h.update(a.tobytes())
print(os.environ.get("PUCFEM_LIB_VARIANT", "default"), f"L{level} {steps} steps {sys.argv[3:]}", h.hexdigest()[:24], its[-3:])
sim.close()
